// libh3d.so: the prepare_data entry points (union of the replicate band
// matrices, size factors of every norm); shares the ctx / scratch / error
// helpers of h3d_api.hip through h3d_ctx.h.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <vector>

#include "h3d.h"
#include "h3d_ctx.h"
#include "h3d_errors.h"
#include "h3d_host.h"
#include "h3d_kernels.h"
#include "h3d_prepare.h"

using namespace h3d;
using namespace h3dint;
using h3derr::fail;

extern "C" {

int h3d_union_count(h3d_ctx* ctx, int R, int n_bins,
                    const int64_t* const* indptr, const int32_t* const* indices,
                    const double* const* data, const int64_t* nnz,
                    const double* bias, int dist_max, int64_t* n_px_out) {
  if (!ctx || !indptr || !indices || !data || !nnz || !bias || !n_px_out)
    return fail(H3D_EARG, "null argument");
  if (R < 1 || R > kMaxReps || n_bins < 1 || dist_max < 0)
    return fail(H3D_EARG, "R=%d n_bins=%d dist_max=%d", R, n_bins, dist_max);
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  PrepUnion& P = ctx->prep;
  P = PrepUnion();
  P.R = R;
  P.n_bins = n_bins;
  int64_t max_m = 0;
  for (int r = 0; r < R; ++r) {
    if (nnz[r] < 0 || (nnz[r] > 0 && (!indices[r] || !data[r])) || !indptr[r])
      return fail(H3D_EARG, "replicate %d CSR", r);
    if (indptr[r][n_bins] != nnz[r]) return fail(H3D_EARG, "replicate %d indptr[-1] != nnz", r);
    if (nnz[r] >= ((int64_t)1 << 31)) return fail(H3D_EARG, "replicate %d: too many entries", r);
    max_m = std::max(max_m, nnz[r]);
  }
  const int64_t sentinel = (int64_t)n_bins * n_bins;
  int end_bit = 1;
  while (end_bit < 63 && (((int64_t)1) << end_bit) <= sentinel) ++end_bit;
  // per-replicate staging (reused): only the in-band entries reach the
  // per-entry key / sort / scan buffers, so their size and the 2^31 cap
  // follow the band, not the whole-chromosome nnz
  const size_t mm = (size_t)std::max<int64_t>(max_m, 1);
  double* d_bias = (double*)scratch(ctx, "u_bias", (size_t)n_bins * R * 8);
  int64_t* d_indptr = (int64_t*)scratch(ctx, "u_indptr", (size_t)(n_bins + 1) * 8);
  int32_t* d_row = (int32_t*)scratch(ctx, "u_row_of", mm * 4);
  int32_t* d_col = (int32_t*)scratch(ctx, "u_col", mm * 4);
  double* d_val = (double*)scratch(ctx, "u_val_in", mm * 8);
  int32_t* d_flag = (int32_t*)scratch(ctx, "u_flag", mm * 4);
  int32_t* d_pos = (int32_t*)scratch(ctx, "u_pos", mm * 4);
  int32_t* d_cnt = (int32_t*)scratch(ctx, "u_cnt", 4);
  if (!d_bias || !d_indptr || !d_row || !d_col || !d_val || !d_flag || !d_pos || !d_cnt)
    return fail(H3D_ENOMEM, "union staging");
  P.bias = d_bias;
  if (int rc = h2d_pinned(ctx, d_bias, bias, (size_t)n_bins * R * 8, s)) return rc;
  int64_t tot = 0;  // kept entries so far
  int64_t* d_keys = nullptr;
  int32_t* d_ent = nullptr;
  for (int r = 0; r < R; ++r) {
    const int64_t m = nnz[r];
    if (m == 0) continue;
    HIP_TRY(hipMemcpyAsync(d_indptr, indptr[r], (size_t)(n_bins + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_col, indices[r], m * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_val, data[r], m * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_csr_rows, dim3((n_bins + 255) / 256), dim3(256), 0, s,
                       d_indptr, n_bins, d_row);
    hipLaunchKernelGGL(k_union_flags, dim3(grid_for(ctx, m)), dim3(kBlock), 0, s, d_row,
                       d_col, d_val, m, n_bins, dist_max, d_flag);
    size_t tbs = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tbs, d_flag, d_pos, (int)m, s));
    void* tmps = scratch(ctx, "cub_tmp_s", tbs);
    if (!tmps) return fail(H3D_ENOMEM, "scan temp");
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmps, tbs, d_flag, d_pos, (int)m, s));
    int32_t last[2] = {0, 0};
    if (int rc = d2h_sync(ctx, &last[0], d_pos + m - 1, 4, s)) return rc;
    if (int rc = d2h_sync(ctx, &last[1], d_flag + m - 1, 4, s)) return rc;
    const int64_t kept = (int64_t)last[0] + last[1];
    if (tot + kept >= ((int64_t)1 << 31)) return fail(H3D_EARG, "too many in-band entries");
    // the kept-entry arrays grow (keeping what earlier replicates wrote)
    const size_t need = (size_t)std::max<int64_t>(tot + kept, 1);
    d_keys = (int64_t*)scratch_keep(ctx, "u_keys", need * 8, tot * 8);
    d_ent = (int32_t*)scratch_keep(ctx, "u_ent", need * 4, tot * 4);
    P.ent_rep = (int32_t*)scratch_keep(ctx, "u_ent_rep", need * 4, tot * 4);
    P.ent_val = (double*)scratch_keep(ctx, "u_ent_val", need * 8, tot * 8);
    if (!d_keys || !d_ent || !P.ent_rep || !P.ent_val) return fail(H3D_ENOMEM, "union entries");
    hipLaunchKernelGGL(k_union_keys, dim3(grid_for(ctx, m)), dim3(kBlock), 0, s, d_row, d_col,
                       d_val, d_flag, d_pos, m, tot, r, n_bins, d_keys, d_ent, P.ent_rep,
                       P.ent_val);
    // the staging buffers are reused by the next replicate
    HIP_TRY(hipStreamSynchronize(s));
    tot += kept;
  }
  P.n_entries = tot;
  if (tot == 0) {
    P.n_px = 0;
    *n_px_out = 0;
    return 0;
  }
  P.keys_sorted = (int64_t*)scratch(ctx, "u_keys_s", tot * 8);
  P.ent_sorted = (int32_t*)scratch(ctx, "u_ent_s", tot * 4);
  int32_t* d_head = (int32_t*)scratch(ctx, "u_head", tot * 4);
  P.run_of = (int32_t*)scratch(ctx, "u_run_incl", tot * 4);
  if (!P.keys_sorted || !P.ent_sorted || !d_head || !P.run_of)
    return fail(H3D_ENOMEM, "union scratch");
  size_t tb = 0;
  HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, d_keys, P.keys_sorted, d_ent,
                                             P.ent_sorted, (int)tot, 0, end_bit, s));
  void* tmp = scratch(ctx, "cub_tmp_u", tb);
  if (!tmp) return fail(H3D_ENOMEM, "sort temp");
  HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, d_keys, P.keys_sorted, d_ent,
                                             P.ent_sorted, (int)tot, 0, end_bit, s));
  hipLaunchKernelGGL(k_run_heads, dim3(grid_for(ctx, tot)), dim3(kBlock), 0, s,
                     P.keys_sorted, tot, sentinel, d_head);
  tb = 0;
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tb, d_head, P.run_of, (int)tot, s));
  tmp = scratch(ctx, "cub_tmp_s", tb);
  if (!tmp) return fail(H3D_ENOMEM, "scan temp");
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(tmp, tb, d_head, P.run_of, (int)tot, s));
  int32_t n_runs = 0;
  if (int rc = d2h_sync(ctx, &n_runs, P.run_of + tot - 1, 4, s)) return rc;
  P.n_runs = n_runs;
  P.run_start = (int64_t*)scratch(ctx, "u_run_start", std::max<int64_t>(n_runs, 1) * 8);
  int32_t* keep = (int32_t*)scratch(ctx, "u_keep", std::max<int64_t>(n_runs, 1) * 4);
  P.px_of_run = (int32_t*)scratch(ctx, "u_px_incl", std::max<int64_t>(n_runs, 1) * 4);
  if (!P.run_start || !keep || !P.px_of_run) return fail(H3D_ENOMEM, "runs");
  if (n_runs == 0) {
    P.n_px = 0;
    *n_px_out = 0;
    return 0;
  }
  hipLaunchKernelGGL(k_run_starts, dim3(grid_for(ctx, tot)), dim3(kBlock), 0, s,
                     d_head, P.run_of, tot, P.run_start);
  hipLaunchKernelGGL(k_run_keep, dim3(grid_for(ctx, n_runs)), dim3(kBlock), 0, s,
                     P.keys_sorted, P.ent_sorted, P.run_start, (int64_t)n_runs, tot,
                     sentinel, P.ent_rep, P.ent_val, R, n_bins, d_bias, keep);
  tb = 0;
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tb, keep, P.px_of_run, (int)n_runs, s));
  tmp = scratch(ctx, "cub_tmp_s", tb);
  if (!tmp) return fail(H3D_ENOMEM, "scan temp");
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(tmp, tb, keep, P.px_of_run, (int)n_runs, s));
  int32_t n_px = 0;
  if (int rc = d2h_sync(ctx, &n_px, P.px_of_run + n_runs - 1, 4, s)) return rc;
  P.n_px = n_px;
  *n_px_out = n_px;
  return 0;
}

int h3d_union_fill(h3d_ctx* ctx, int32_t* row, int32_t* col, int64_t* raw,
                   double* balanced, int64_t n_px) {
  return h3d_union_fill_dev(ctx, row, col, raw, balanced, n_px, nullptr, nullptr, nullptr,
                            nullptr);
}

int h3d_union_fill_dev(h3d_ctx* ctx, int32_t* row, int32_t* col, int64_t* raw,
                       double* balanced, int64_t n_px, int32_t* d_row_out,
                       int32_t* d_col_out, int32_t* d_raw_out, double* d_bal_out) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  PrepUnion& P = ctx->prep;
  if (n_px != P.n_px) return fail(H3D_EARG, "n_px %lld != counted %lld", (long long)n_px, (long long)P.n_px);
  if (n_px == 0) return 0;
  // raw may be NULL when the device copy d_raw_out is requested (the caller
  // fetches it in the background, analysis/d2h.py)
  if (!row || !col || (!raw && !d_raw_out) || (!balanced && !d_bal_out))
    return fail(H3D_EARG, "null output");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const int R = P.R;
  int32_t* d_row = (int32_t*)scratch(ctx, "u_out_row", n_px * 4);
  int32_t* d_col = (int32_t*)scratch(ctx, "u_out_col", n_px * 4);
  int64_t* d_raw = (int64_t*)scratch(ctx, "u_out_raw", n_px * R * 8);
  double* d_bal = (double*)scratch(ctx, "u_out_bal", n_px * R * 8);
  int32_t* keep = (int32_t*)scratch(ctx, "u_keep", std::max<int64_t>(P.n_runs, 1) * 4);
  int* d_ovf = (int*)scratch(ctx, "ovf", 4);
  if (!d_row || !d_col || !d_raw || !d_bal || !d_ovf) return fail(H3D_ENOMEM, "union out");
  hipLaunchKernelGGL(k_union_fill, dim3(grid_for(ctx, P.n_runs)), dim3(kBlock), 0, s,
                     P.keys_sorted, P.ent_sorted, P.run_start, keep, P.px_of_run,
                     P.n_runs, P.n_entries, P.ent_rep, P.ent_val, R, P.n_bins, P.bias,
                     d_row, d_col, d_raw, d_bal);
  // the caller's device copies (the product's resident chromosome): the
  // counts as int32, the width every disp / lrt kernel reads
  if (d_row_out) HIP_TRY(hipMemcpyAsync(d_row_out, d_row, n_px * 4, hipMemcpyDeviceToDevice, s));
  if (d_col_out) HIP_TRY(hipMemcpyAsync(d_col_out, d_col, n_px * 4, hipMemcpyDeviceToDevice, s));
  if (d_bal_out)
    HIP_TRY(hipMemcpyAsync(d_bal_out, d_bal, n_px * R * 8, hipMemcpyDeviceToDevice, s));
  int ovf = 0;
  if (d_raw_out) {
    HIP_TRY(hipMemsetAsync(d_ovf, 0, 4, s));
    hipLaunchKernelGGL(k_i64_to_i32, dim3(grid_for(ctx, n_px * R)), dim3(kBlock), 0, s, d_raw,
                       d_raw_out, n_px * R, d_ovf);
    HIP_TRY(hipMemcpyAsync(&ovf, d_ovf, 4, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipMemcpyAsync(row, d_row, n_px * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(col, d_col, n_px * 4, hipMemcpyDeviceToHost, s));
  if (raw) HIP_TRY(hipMemcpyAsync(raw, d_raw, n_px * R * 8, hipMemcpyDeviceToHost, s));
  if (balanced)
    HIP_TRY(hipMemcpyAsync(balanced, d_bal, n_px * R * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (ovf) return fail(H3D_EINPUT, "raw counts must be in [0, 2^31) for the device copy");
  return 0;
}

// d_disp_idx (n) 0/1 -> the chromosome's disp pixels (k_disp_pixels)
int h3d_disp_pixels_dev(h3d_ctx* ctx, const int32_t* d_row, const int32_t* d_col,
                        const int32_t* d_raw, const double* d_sf, int sf_per_rep,
                        const double* bias, int n_bins, const uint8_t* d_disp_idx,
                        int64_t n, int R, int64_t n_disp, int32_t* d_raw_out,
                        double* d_f_out, int32_t* d_dist_out) {
  if (!ctx || !bias) return fail(H3D_EARG, "null argument");
  if (R < 1 || R > kMaxReps || n_bins < 1 || n < 0 || n_disp < 0 || n_disp > n)
    return fail(H3D_EARG, "R=%d n_bins=%d n=%lld n_disp=%lld", R, n_bins, (long long)n,
                (long long)n_disp);
  if (n >= ((int64_t)1 << 31)) return fail(H3D_EARG, "n=%lld exceeds 2^31", (long long)n);
  if (n == 0) return 0;
  if (!d_row || !d_col || !d_raw || !d_sf || !d_disp_idx)
    return fail(H3D_EARG, "null device input");
  if (n_disp > 0 && (!d_raw_out || !d_f_out || !d_dist_out))
    return fail(H3D_EARG, "null device output");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  int32_t* d_sel = (int32_t*)scratch(ctx, "dp_sel", (size_t)std::max<int64_t>(n, 1) * 4);
  int32_t* d_cnt = (int32_t*)scratch(ctx, "dp_cnt", 4);
  double* d_bias = (double*)scratch(ctx, "dp_bias", (size_t)n_bins * R * 8);
  if (!d_sel || !d_cnt || !d_bias) return fail(H3D_ENOMEM, "disp pixel scratch");
  if (int rc = h2d_pinned(ctx, d_bias, bias, (size_t)n_bins * R * 8, s)) return rc;
  hipcub::CountingInputIterator<int32_t> it(0);
  size_t tb = 0;
  HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, it, d_disp_idx, d_sel, d_cnt, (int)n, s));
  void* tmp = scratch(ctx, "cub_tmp_sel", tb);
  if (!tmp) return fail(H3D_ENOMEM, "select temp");
  HIP_TRY(hipcub::DeviceSelect::Flagged(tmp, tb, it, d_disp_idx, d_sel, d_cnt, (int)n, s));
  int32_t* land = (int32_t*)pinned_rd(ctx, 4);
  if (!land) return fail(H3D_ENOMEM, "pinned landing zone");
  HIP_TRY(hipMemcpyAsync(land, d_cnt, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const int32_t cnt = land[0];
  if (cnt != n_disp)
    return fail(H3D_EARG, "disp_idx selects %d pixels, caller expects %lld", cnt,
                (long long)n_disp);
  if (n_disp == 0) return 0;
  hipLaunchKernelGGL(k_disp_pixels, dim3(grid_for(ctx, n_disp)), dim3(kBlock), 0, s, d_sel,
                     n_disp, d_row, d_col, d_raw, d_sf, sf_per_rep, d_bias, R, d_raw_out,
                     d_f_out, d_dist_out);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(s));
  return 0;
}

int h3d_pixel_f_dev(h3d_ctx* ctx, const int32_t* d_row, const int32_t* d_dist,
                    const int32_t* d_chrom, const int32_t* d_sfi, int64_t n, int R,
                    const double* d_bias, const int64_t* d_boff, const double* d_sf,
                    const int64_t* d_soff, int nchrom, double* d_f_out) {
  if (!ctx) return fail(H3D_EARG, "null argument");
  if (R < 1 || R > kMaxReps || n < 0 || nchrom < 1)
    return fail(H3D_EARG, "R=%d n=%lld nchrom=%d", R, (long long)n, nchrom);
  if (n == 0) return 0;
  if (!d_row || !d_dist || !d_chrom || !d_sfi || !d_bias || !d_boff || !d_sf || !d_soff ||
      !d_f_out)
    return fail(H3D_EARG, "null device pointer");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  int* d_bad = (int*)scratch(ctx, "pf_bad", 4);
  if (!d_bad) return fail(H3D_ENOMEM, "pixel f scratch");
  HIP_TRY(hipMemsetAsync(d_bad, 0, 4, s));
  hipLaunchKernelGGL(k_pixel_f, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s, d_row, d_dist,
                     d_chrom, d_sfi, n, R, d_bias, d_boff, d_sf, d_soff, nchrom, d_f_out,
                     d_bad);
  HIP_TRY(hipGetLastError());
  int bad = 0;
  if (int rc = d2h_sync(ctx, &bad, d_bad, 4, s)) return rc;
  if (bad) return fail(H3D_EINPUT, "pixel keys outside the bias / size-factor tables");
  return 0;
}

int h3d_scale_disp_dev(h3d_ctx* ctx, const double* d_balanced, const double* d_sf,
                       int sf_per_rep, const int32_t* d_row, const int32_t* d_col, int64_t n,
                       int R, int C, const uint8_t* design, double mean_thresh,
                       int dist_thresh_min, double* scaled_out, uint8_t* flag_out,
                       uint8_t* d_flag_out, double* d_scaled_out) {
  if (!ctx || !design) return fail(H3D_EARG, "null argument");
  if (R < 1 || R > kMaxReps || C < 1 || C > kMaxConds || n < 0)
    return fail(H3D_EARG, "R=%d C=%d n=%lld", R, C, (long long)n);
  if (n == 0) return 0;
  if (!d_balanced || !d_sf || !d_row || !d_col) return fail(H3D_EARG, "null device input");
  if ((!scaled_out && !d_scaled_out) || !flag_out) return fail(H3D_EARG, "null output");
  ScaleDispArgs a{};
  for (int c = 0; c < C; ++c) {
    int cnt = 0;
    for (int k = 0; k < R; ++k)
      if (design[k * C + c]) {
        a.cond_mask[c] |= 1u << k;
        ++cnt;
      }
    // np.sum(design, axis=0): a condition without replicates divides by 0
    a.count[c] = (double)cnt;
  }
  a.C = C;
  a.mean_thresh = mean_thresh;
  a.dist_min = dist_thresh_min;
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  double* d_scaled =
      d_scaled_out ? d_scaled_out : (double*)scratch(ctx, "sd_scaled", (size_t)n * R * 8);
  uint8_t* d_flag = d_flag_out ? d_flag_out : (uint8_t*)scratch(ctx, "sd_flag", (size_t)n);
  if (!d_scaled || !d_flag) return fail(H3D_ENOMEM, "scale / disp scratch");
  hipLaunchKernelGGL(k_scale_disp, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s, d_balanced,
                     d_sf, sf_per_rep, d_row, d_col, n, R, a, d_scaled, d_flag);
  HIP_TRY(hipGetLastError());
  if (scaled_out)
    HIP_TRY(hipMemcpyAsync(scaled_out, d_scaled, (size_t)n * R * 8, hipMemcpyDeviceToHost, s));
  // (the flags through the pinned landing zone: see h2d_pinned)
  return d2h_sync(ctx, flag_out, d_flag, (size_t)n, s);
}

int h3d_table_gather_dev(h3d_ctx* ctx, const double* d_tables, int D, int C,
                         const int32_t* d_dist, int64_t n, double* d_out) {
  if (!ctx || !d_tables || D < 1 || C < 1 || C > kMaxConds || n < 0)
    return fail(H3D_EARG, "null argument / D / C / n");
  // a pending device smoother is settled first (a degenerate fit is redone
  // on the host into the same buffer)
  if (int rc = h3d_disp_tables_wait(ctx)) return rc;
  if (n == 0) return 0;
  if (!d_dist || !d_out) return fail(H3D_EARG, "null device buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(k_table_gather, dim3(grid_for(ctx, n)), dim3(kBlock), 0, ctx->stream,
                     d_tables, D, C, d_dist, n, d_out);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

namespace {
int size_factors_impl(h3d_ctx* ctx, const double* balanced, const double* d_balanced,
                      const int32_t* dist, int64_t n, int R, int norm, int n_bins,
                      double* sf_out, double* d_sf_out);
}  // namespace

int h3d_size_factors(h3d_ctx* ctx, const double* balanced, const int32_t* dist,
                     int64_t n, int R, int norm, int n_bins, double* sf_out) {
  return size_factors_impl(ctx, balanced, nullptr, dist, n, R, norm, n_bins, sf_out,
                           nullptr);
}

int h3d_size_factors_dev(h3d_ctx* ctx, const double* d_balanced, const int32_t* dist,
                         int64_t n, int R, int norm, int n_bins, double* sf_out,
                         double* d_sf_out) {
  if (n > 0 && !d_balanced) return fail(H3D_EARG, "null device balanced");
  return size_factors_impl(ctx, nullptr, d_balanced, dist, n, R, norm, n_bins, sf_out,
                           d_sf_out);
}

}  // extern "C"

namespace {
int size_factors_impl(h3d_ctx* ctx, const double* balanced, const double* d_balanced,
                      const int32_t* dist, int64_t n, int R, int norm, int n_bins,
                      double* sf_out, double* d_sf_out) {
  const bool cond_norm =
      norm == H3D_NORM_CONDITIONAL_MOR || norm == H3D_NORM_CONDITIONAL_SCALING;
  // sf_out may be NULL for the conditional norms when d_sf_out is given (the
  // caller fetches the (n, R) factors in the background)
  if (!ctx || (n > 0 && !balanced && !d_balanced) || (!sf_out && !(cond_norm && d_sf_out)))
    return fail(H3D_EARG, "null argument");
  if (R < 1 || R > kMaxReps || n_bins < 0) return fail(H3D_EARG, "R=%d n_bins=%d", R, n_bins);
  if (norm < H3D_NORM_CONDITIONAL_MOR || norm > H3D_NORM_NO_SCALING)
    return fail(H3D_EARG, "norm %d", norm);
  const bool conditional =
      norm == H3D_NORM_CONDITIONAL_MOR || norm == H3D_NORM_CONDITIONAL_SCALING;
  const bool mor = norm == H3D_NORM_CONDITIONAL_MOR || norm == H3D_NORM_MEDIAN_OF_RATIOS;
  // the (R,) factors of the global norms into the caller's device copy too
  auto global_out = [&]() -> int {
    if (d_sf_out) {
      HIP_TRY(hipSetDevice(ctx->device));
      HIP_TRY(hipMemcpyAsync(d_sf_out, sf_out, R * 8, hipMemcpyHostToDevice, ctx->stream));
      HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    return 0;
  };
  if (norm == H3D_NORM_NO_SCALING) {  // scaling.py:24: ones(R), no data pass
    for (int r = 0; r < R; ++r) sf_out[r] = 1.0;
    return global_out();
  }
  if (conditional && n > 0 && !dist) return fail(H3D_EARG, "null dist");
  if (n == 0) {
    if (!conditional) {
      for (int r = 0; r < R; ++r) sf_out[r] = NAN;  // median / sums of nothing
      return global_out();
    }
    return 0;
  }
  if (n >= ((int64_t)1 << 31) / R) return fail(H3D_EARG, "n too large");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  double* d_bal = d_balanced ? nullptr : (double*)scratch(ctx, "sf_bal", n * R * 8);
  int32_t* d_dist = (int32_t*)scratch(ctx, "sf_dist", n * 4);
  int32_t* d_dist_s = (int32_t*)scratch(ctx, "sf_dist_s", n * 4);
  int32_t* d_idx = (int32_t*)scratch(ctx, "sf_idx", n * 4);
  int32_t* d_perm = (int32_t*)scratch(ctx, "sf_perm", n * 4);
  int32_t* d_bin = (int32_t*)scratch(ctx, "sf_bin", n * 4);
  double* d_sf = (double*)scratch(ctx, "sf_out", n * R * 8);
  if ((!d_balanced && !d_bal) || !d_dist || !d_dist_s || !d_idx || !d_perm || !d_bin || !d_sf)
    return fail(H3D_ENOMEM, "size factor scratch");
  if (!d_balanced)
    HIP_TRY(hipMemcpyAsync(d_bal, balanced, n * R * 8, hipMemcpyHostToDevice, s));
  const double* bal = d_balanced ? d_balanced : d_bal;
  hipLaunchKernelGGL(k_iota, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s, d_idx, n);
  size_t tb = 0;
  void* tmp = nullptr;
  // 1. bins over the (stable) distance order: sorted position k -> bin[k]
  int nb = 1;
  if (!conditional) {
    // one bin holding every pixel, in the original order
    HIP_TRY(hipMemcpyAsync(d_perm, d_idx, n * 4, hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipMemsetAsync(d_bin, 0, n * 4, s));
  } else {
    if (int rc = h2d_pinned(ctx, d_dist, dist, n * 4, s)) return rc;
    // stable sort by distance (the pinned equal_bin tie order)
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, d_dist, d_dist_s, d_idx,
                                               d_perm, (int)n, 0, 31, s));
    tmp = scratch(ctx, "cub_tmp_sf", tb);
    if (!tmp) return fail(H3D_ENOMEM, "sort temp");
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, d_dist, d_dist_s, d_idx, d_perm,
                                               (int)n, 0, 31, s));
    if (n_bins > 0) {
      nb = n_bins;
      hipLaunchKernelGGL(k_equal_bin, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s, n,
                         n_bins, d_bin);
    } else {
      int32_t* d_head = (int32_t*)scratch(ctx, "sf_head", n * 4);
      if (!d_head) return fail(H3D_ENOMEM, "heads");
      hipLaunchKernelGGL(k_dist_heads, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s,
                         d_dist_s, n, d_head);
      tb = 0;
      HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tb, d_head, d_bin, (int)n, s));
      tmp = scratch(ctx, "cub_tmp_s", tb);
      if (!tmp) return fail(H3D_ENOMEM, "scan temp");
      HIP_TRY(hipcub::DeviceScan::InclusiveSum(tmp, tb, d_head, d_bin, (int)n, s));
      hipLaunchKernelGGL(k_minus_one, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s, d_bin, n);
      int32_t last = 0;
      if (int rc = d2h_sync(ctx, &last, d_bin + n - 1, 4, s)) return rc;
      nb = last + 1;
    }
  }
  int64_t* d_bstart = (int64_t*)scratch(ctx, "sf_bstart", (size_t)(nb + 1) * 8);
  double* d_spb = (double*)scratch(ctx, "sf_spb", (size_t)nb * R * 8);
  double* d_dpb = (double*)scratch(ctx, "sf_dpb", (size_t)nb * 8);
  if (!d_bstart || !d_spb || !d_dpb) return fail(H3D_ENOMEM, "bins");
  hipLaunchKernelGGL(k_bin_bounds, dim3((nb + 1 + 255) / 256), dim3(256), 0, s, d_bin,
                     n, nb, d_bstart);
  std::vector<int64_t> bstart(nb + 1);
  if (int rc = d2h_sync(ctx, bstart.data(), d_bstart, (nb + 1) * 8, s)) return rc;
  // 2. per-bin factors s_per_bin (nb, R)
  std::vector<double> spb((size_t)nb * R);
  if (mor) {
    // median_of_ratios (scaling.py:27-47): per replicate the median over the
    // bin's all-positive rows of data / gmean(row); a segmented sort of the
    // ratios per (replicate, bin), invalid rows keyed +inf past the valid ones
    int32_t* d_valid = (int32_t*)scratch(ctx, "sf_valid", (size_t)nb * 4);
    double* d_keys = (double*)scratch(ctx, "sf_keys", n * R * 8);
    double* d_keys_s = (double*)scratch(ctx, "sf_keys_s", n * R * 8);
    int64_t* d_segb = (int64_t*)scratch(ctx, "sf_segb", (size_t)nb * R * 8);
    int64_t* d_sege = (int64_t*)scratch(ctx, "sf_sege", (size_t)nb * R * 8);
    if (!d_valid || !d_keys || !d_keys_s || !d_segb || !d_sege)
      return fail(H3D_ENOMEM, "median scratch");
    HIP_TRY(hipMemsetAsync(d_valid, 0, (size_t)nb * 4, s));
    hipLaunchKernelGGL(k_mor_keys, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s, bal,
                       d_perm, n, R, d_bin, d_keys, d_valid);
    std::vector<int64_t> segb((size_t)nb * R), sege((size_t)nb * R);
    for (int r = 0; r < R; ++r)
      for (int b = 0; b < nb; ++b) {
        segb[(size_t)r * nb + b] = (int64_t)r * n + bstart[b];
        sege[(size_t)r * nb + b] = (int64_t)r * n + bstart[b + 1];
      }
    if (int rc = h2d_pinned(ctx, d_segb, segb.data(), segb.size() * 8, s)) return rc;
    if (int rc = h2d_pinned(ctx, d_sege, sege.data(), sege.size() * 8, s)) return rc;
    tb = 0;
    HIP_TRY(hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, tb, d_keys, d_keys_s,
                                                       (int)(n * R), nb * R, d_segb,
                                                       d_sege, 0, 64, s));
    tmp = scratch(ctx, "cub_tmp_seg", tb);
    if (!tmp) return fail(H3D_ENOMEM, "segmented sort temp");
    HIP_TRY(hipcub::DeviceSegmentedRadixSort::SortKeys(tmp, tb, d_keys, d_keys_s,
                                                       (int)(n * R), nb * R, d_segb,
                                                       d_sege, 0, 64, s));
    hipLaunchKernelGGL(k_mor_median, dim3((nb * R + 255) / 256), dim3(256), 0, s,
                       d_keys_s, d_bstart, d_valid, nb, n, R, d_spb);
    if (int rc = d2h_sync(ctx, spb.data(), d_spb, (size_t)nb * R * 8, s)) return rc;
  } else {
    // simple_scaling (scaling.py:50-65): column sums over the bin's rows in
    // their original order (members grouped by bin: a stable sort of the
    // original-order bin labels), then s / gmean(s, pseudocount 1)
    int32_t* members = d_idx;
    if (conditional) {
      int32_t* d_bin_orig = (int32_t*)scratch(ctx, "sf_bin_orig", n * 4);
      int32_t* d_bin_orig_s = (int32_t*)scratch(ctx, "sf_bin_orig_s", n * 4);
      int32_t* d_iota = (int32_t*)scratch(ctx, "sf_iota2", n * 4);
      members = (int32_t*)scratch(ctx, "sf_members", n * 4);
      if (!d_bin_orig || !d_bin_orig_s || !d_iota || !members)
        return fail(H3D_ENOMEM, "member scratch");
      hipLaunchKernelGGL(k_scatter_bin, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s,
                         d_perm, d_bin, n, d_bin_orig);
      hipLaunchKernelGGL(k_iota, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s, d_iota, n);
      int end_bit = 1;
      while (end_bit < 31 && (1 << end_bit) <= nb) ++end_bit;
      tb = 0;
      HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, d_bin_orig, d_bin_orig_s,
                                                 d_iota, members, (int)n, 0, end_bit, s));
      tmp = scratch(ctx, "cub_tmp_sf", tb);
      if (!tmp) return fail(H3D_ENOMEM, "sort temp");
      HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, d_bin_orig, d_bin_orig_s, d_iota,
                                                 members, (int)n, 0, end_bit, s));
    }
    hipLaunchKernelGGL(k_bin_colsum, dim3((nb * R + 255) / 256), dim3(256), 0, s, bal,
                       members, d_bstart, nb, R, d_spb);
    std::vector<double> colsum((size_t)nb * R);
    if (int rc = d2h_sync(ctx, colsum.data(), d_spb, (size_t)nb * R * 8, s)) return rc;
    for (int b = 0; b < nb; ++b) {
      const double* cs = &colsum[(size_t)b * R];
      double lg[kMaxReps];
      for (int r = 0; r < R; ++r) lg[r] = std::log(cs[r] + 1);
      const double gm = std::exp(np_sum<kMaxReps>(lg, R) / R) - 1;
      for (int r = 0; r < R; ++r) spb[(size_t)b * R + r] = cs[r] / gm;
    }
  }
  if (!conditional) {
    std::memcpy(sf_out, spb.data(), R * 8);
    return global_out();
  }
  // 3. per-pixel factors (scaling.py:88-105)
  if (n_bins > 0) {
    hipLaunchKernelGGL(k_bin_dist_sum, dim3(nb), dim3(256), 0, s, d_dist_s, d_bstart, nb,
                       d_dpb);
    std::vector<double> dpb(nb);
    HIP_TRY(hipMemcpyAsync(dpb.data(), d_dpb, nb * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    // np.unique(bins): only non-empty bins take part in the interpolation
    std::vector<double> xp, yp;
    for (int b = 0; b < nb; ++b)
      if (bstart[b + 1] > bstart[b]) {
        xp.push_back(dpb[b]);
        for (int r = 0; r < R; ++r) yp.push_back(spb[(size_t)b * R + r]);
      }
    const int m = (int)xp.size();
    if (m < 2) return fail(H3D_EARG, "fewer than two distance bins to interpolate");
    double* d_xp = (double*)scratch(ctx, "sf_xp", m * 8);
    double* d_yp = (double*)scratch(ctx, "sf_yp", (size_t)m * R * 8);
    if (!d_xp || !d_yp) return fail(H3D_ENOMEM, "interp");
    HIP_TRY(hipMemcpyAsync(d_xp, xp.data(), m * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_yp, yp.data(), (size_t)m * R * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_sf_interp, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s, d_dist, n,
                       R, d_xp, d_yp, m, d_sf);
  } else {
    HIP_TRY(hipMemcpyAsync(d_spb, spb.data(), (size_t)nb * R * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_sf_exact, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s, d_perm,
                       d_bin, n, R, d_spb, d_sf);
  }
  if (d_sf_out) HIP_TRY(hipMemcpyAsync(d_sf_out, d_sf, n * R * 8, hipMemcpyDeviceToDevice, s));
  if (sf_out) HIP_TRY(hipMemcpyAsync(sf_out, d_sf, n * R * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return 0;
}
}  // namespace

extern "C" {

int h3d_size_factors_cmor(h3d_ctx* ctx, const double* balanced,
                          const int32_t* dist, int64_t n, int R, int n_bins,
                          double* sf_out) {
  return h3d_size_factors(ctx, balanced, dist, n, R, H3D_NORM_CONDITIONAL_MOR, n_bins,
                          sf_out);
}

}  // extern "C"
