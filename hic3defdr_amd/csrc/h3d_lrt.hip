// libh3d.so: the lrt entry points (h3d_lrt_dev / h3d_lrt / h3d_lrt_wide;
// reference util/lrt.py:7-80 as called from analysis.py:244-270).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "h3d.h"
#include "h3d_ctx.h"
#include "h3d_errors.h"
#include "h3d_kernels.h"
#include "h3d_lrt_group.h"

using namespace h3d;
using namespace h3dint;
using h3derr::fail;

namespace {

// R <= 8: one lane per pixel (k_lrt); R > 8: one 8-lane group per pixel
// (k_lrt8, h3d_lrt_group.h)
template <int M, int CM>
void launch_lrt(h3d_ctx* ctx, const int32_t* raw, const double* f,
                const int32_t* dist, const double* table, int64_t n, int R,
                int C, int D, const int32_t* cond, int refit, double* p,
                double* llr, double* mu0, double* mu1, double* disp,
                int* flags, int wide) {
  if constexpr (M <= 8) {
    if (refit && dist && !wide)  // the pipeline's call (k_lrt TAB)
      hipLaunchKernelGGL((k_lrt<M, CM, true>), dim3(grid_for(ctx, n, 16)), dim3(kBlock),
                         0, ctx->stream, raw, f, dist, table, n, R, C, D, cond, refit,
                         p, llr, mu0, mu1, disp, flags, wide);
    else
      hipLaunchKernelGGL((k_lrt<M, CM>), dim3(grid_for(ctx, n, 16)), dim3(kBlock), 0,
                         ctx->stream, raw, f, dist, table, n, R, C, D, cond, refit, p,
                         llr, mu0, mu1, disp, flags, wide);
  } else {
    if (refit && dist && !wide)  // the pipeline's call (k_lrt8 TAB)
      hipLaunchKernelGGL((k_lrt8<M, CM, true>), dim3(grid_for(ctx, n * kGroup, 16)),
                         dim3(kBlock), 0, ctx->stream, raw, f, dist, table, n, R, C,
                         D, cond, refit, p, llr, mu0, mu1, disp, flags, wide);
    else
      hipLaunchKernelGGL((k_lrt8<M, CM>), dim3(grid_for(ctx, n * kGroup, 16)),
                         dim3(kBlock), 0, ctx->stream, raw, f, dist, table, n, R, C,
                         D, cond, refit, p, llr, mu0, mu1, disp, flags, wide);
  }
}

// wide: disp_table is per pixel AND replicate (n, R) (d_dist must be null)
// table_on_dev: disp_table is a device buffer (h3d_disp_tables_dev's output)
int lrt_run(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
            const int32_t* d_dist, const double* disp_table, int64_t n, int R,
            int C, const int32_t* cond_of_rep, int D, int refit_mu, double* d_p,
            double* d_llr, double* d_mu0, double* d_mu1, double* d_disp,
            int wide, int table_on_dev = 0) {
  if (!ctx || !disp_table || !cond_of_rep) return fail(H3D_EARG, "null argument");
  if (wide && (d_dist || d_disp)) return fail(H3D_EARG, "wide dispersions take no dist / disp_out");
  if (n == 0) return 0;
  if (!d_raw || !d_f || !d_p || !d_llr || !d_mu0 || !d_mu1)
    return fail(H3D_EARG, "null device buffer");
  std::vector<int> nrep;
  std::vector<int32_t> rep_idx;
  if (int rc = check_cond(cond_of_rep, R, C, &nrep, &rep_idx)) return rc;
  HIP_TRY(hipSetDevice(ctx->device));
  if (getenv("H3D_DEBUG")) {
    const hipError_t pe = hipGetLastError();
    if (pe != hipSuccess)
      fprintf(stderr, "[h3d] lrt entry: pending HIP error %s\n", hipGetErrorString(pe));
  }
  hipStream_t s = ctx->stream;
  // d_dist == NULL: disp_table holds per-pixel dispersions (n, C), or with
  // `wide` per pixel and replicate (n, R)
  const size_t tab_n = d_dist ? (size_t)D * C : (size_t)n * (wide ? R : C);
  double* d_tab = table_on_dev ? (double*)disp_table
                               : (double*)scratch(ctx, "disp_table", tab_n * 8);
  int32_t* d_cond = (int32_t*)scratch(ctx, "cond_of_rep", R * 4);
  int* d_fl = (int*)scratch(ctx, "lrt_flags", 4);
  if (!d_tab || !d_cond || !d_fl) return fail(H3D_ENOMEM, "lrt scratch");
  if (!table_on_dev)
    HIP_TRY(hipMemcpyAsync(d_tab, disp_table, tab_n * 8, hipMemcpyHostToDevice, s));
  if (int rc = h2d_pinned(ctx, d_cond, cond_of_rep, R * 4, s)) return rc;
  HIP_TRY(hipMemsetAsync(d_fl, 0, 4, s));
  {
    ProfScope ps(ctx, "lrt", n, 1);
    const int m = R <= 4 ? 4 : R <= 8 ? 8 : R <= 16 ? 16 : R <= 24 ? 24 : 32;
    const int cm = C <= 2 ? 2 : C <= 4 ? 4 : 8;
#define H3D_LRT(MM, CC)                                                          \
  launch_lrt<MM, CC>(ctx, d_raw, d_f, d_dist, d_tab, n, R, C, D, d_cond,   \
                     refit_mu, d_p, d_llr, d_mu0, d_mu1, d_disp, d_fl, wide)
    if (m == 4 && cm == 2) H3D_LRT(4, 2);
    else if (m == 4 && cm == 4) H3D_LRT(4, 4);
    else if (m == 8 && cm == 2) H3D_LRT(8, 2);
    else if (m == 8 && cm == 4) H3D_LRT(8, 4);
    else if (m == 16 && cm == 2) H3D_LRT(16, 2);
    else if (m == 16 && cm == 4) H3D_LRT(16, 4);
    else if (m <= 16) H3D_LRT(16, 8);
    else if (m == 24 && cm <= 4) H3D_LRT(24, 4);
    else if (m == 24) H3D_LRT(24, 8);
    else H3D_LRT(32, 8);
#undef H3D_LRT
  }
  HIP_TRY(hipGetLastError());
  int tst[kMaxConds];
  // (the flag and the table status land in pinned memory)
  int* land = (int*)pinned_rd(ctx, (1 + kMaxConds) * 4);
  if (!land) return fail(H3D_ENOMEM, "pinned landing zone");
  const int tab_check = table_on_dev ? table_status_copy(ctx, land + 1) : 0;
  if (tab_check < 0) return tab_check;
  HIP_TRY(hipMemcpyAsync(land, d_fl, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const int fl = land[0];
  std::memcpy(tst, land + 1, sizeof(tst));
  if (tab_check) {
    // a device table the host had to redo: the LRT over it again
    const int ts = table_settle(ctx, tst);
    if (ts < 0) return ts;
    if (ts == 1)
      return lrt_run(ctx, d_raw, d_f, d_dist, disp_table, n, R, C, cond_of_rep, D,
                     refit_mu, d_p, d_llr, d_mu0, d_mu1, d_disp, wide, 1);
  }
  return flags_to_code(fl);
}

// host buffers in and out (h3d_lrt / h3d_lrt_wide)
int lrt_host(h3d_ctx* ctx, const int64_t* raw, const double* f, const int32_t* dist,
             const double* disp_table, int64_t n, int R, int C,
             const int32_t* cond_of_rep, int D, int refit_mu, double* p, double* llr,
             double* mu0, double* mu1, double* disp_out, int wide) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  if (n == 0) return 0;
  if (!raw || !f || !p || !llr || !mu0 || !mu1) return fail(H3D_EARG, "null buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  int64_t* d_raw64 = (int64_t*)scratch(ctx, "in_raw64", n * R * 8);
  int32_t* d_raw = (int32_t*)scratch(ctx, "in_raw", n * R * 4);
  double* d_f = (double*)scratch(ctx, "in_f", n * R * 8);
  int32_t* d_dist = dist ? (int32_t*)scratch(ctx, "in_dist", n * 4) : nullptr;
  double* d_out = (double*)scratch(ctx, "lrt_out", n * (3 + 2 * C) * 8);
  int* d_ovf = (int*)scratch(ctx, "ovf", 4);
  if (!d_raw64 || !d_raw || !d_f || (dist && !d_dist) || !d_out || !d_ovf)
    return fail(H3D_ENOMEM, "lrt inputs");
  HIP_TRY(hipMemcpyAsync(d_raw64, raw, n * R * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_f, f, n * R * 8, hipMemcpyHostToDevice, s));
  if (dist) HIP_TRY(hipMemcpyAsync(d_dist, dist, n * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(d_ovf, 0, 4, s));
  hipLaunchKernelGGL(k_i64_to_i32, dim3(grid_for(ctx, n * R)), dim3(kBlock), 0, s,
                     d_raw64, d_raw, n * R, d_ovf);
  double *dp = d_out, *dl = d_out + n, *dm0 = d_out + 2 * n, *dm1 = d_out + 3 * n,
         *dd = d_out + (3 + C) * n;
  int rc = lrt_run(ctx, d_raw, d_f, d_dist, disp_table, n, R, C, cond_of_rep, D,
                   refit_mu, dp, dl, dm0, dm1, disp_out ? dd : nullptr, wide);
  int ovf = 0;
  HIP_TRY(hipMemcpyAsync(&ovf, d_ovf, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(p, dp, n * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(llr, dl, n * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(mu0, dm0, n * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(mu1, dm1, n * C * 8, hipMemcpyDeviceToHost, s));
  if (disp_out) HIP_TRY(hipMemcpyAsync(disp_out, dd, n * C * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (ovf) return fail(H3D_EINPUT, "raw counts must be in [0, 2^31)");
  return rc;
}

}  // namespace

extern "C" {

int h3d_lrt_dev(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                const int32_t* d_dist, const double* disp_table, int64_t n,
                int R, int C, const int32_t* cond_of_rep, int D, int refit_mu,
                double* d_p, double* d_llr, double* d_mu0, double* d_mu1,
                double* d_disp) {
  return lrt_run(ctx, d_raw, d_f, d_dist, disp_table, n, R, C, cond_of_rep, D, refit_mu,
                 d_p, d_llr, d_mu0, d_mu1, d_disp, 0);
}

int h3d_lrt_dev_tab(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                    const int32_t* d_dist, const double* d_disp_table, int64_t n,
                    int R, int C, const int32_t* cond_of_rep, int D, int refit_mu,
                    double* d_p, double* d_llr, double* d_mu0, double* d_mu1,
                    double* d_disp) {
  if (!d_dist) return fail(H3D_EARG, "h3d_lrt_dev_tab takes a per-distance table");
  return lrt_run(ctx, d_raw, d_f, d_dist, d_disp_table, n, R, C, cond_of_rep, D,
                 refit_mu, d_p, d_llr, d_mu0, d_mu1, d_disp, 0, 1);
}

int h3d_lrt_wide(h3d_ctx* ctx, const int64_t* raw, const double* f,
                 const double* disp_wide, int64_t n, int R, int C,
                 const int32_t* cond_of_rep, int refit_mu, double* p, double* llr,
                 double* mu0, double* mu1) {
  return lrt_host(ctx, raw, f, nullptr, disp_wide, n, R, C, cond_of_rep, 0, refit_mu, p,
                  llr, mu0, mu1, nullptr, 1);
}

int h3d_lrt(h3d_ctx* ctx, const int64_t* raw, const double* f,
            const int32_t* dist, const double* disp_table, int64_t n, int R,
            int C, const int32_t* cond_of_rep, int D, int refit_mu, double* p,
            double* llr, double* mu0, double* mu1, double* disp_out) {
  return lrt_host(ctx, raw, f, dist, disp_table, n, R, C, cond_of_rep, D, refit_mu, p,
                  llr, mu0, mu1, disp_out, 0);
}

}  // extern "C"
