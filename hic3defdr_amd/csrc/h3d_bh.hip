// libh3d.so: BH-FDR on the GPU (reference analysis.py:286-303 -> lib5c
// adjust_pvalues(method='fdr_bh') -> statsmodels fdrcorrection 'indep').
//
//   finite p only (NaN elsewhere); order = argsort(p); ecdf = (j + 1) / m;
//   q = reverse cumulative min of p[order] / ecdf, clipped at 1, scattered.
//
// One radix sort of (p, index) pairs, one elementwise ratio pass written in
// reverse order, one forward min-scan (min is exact: any association gives
// the reference's bits), one scatter. Ties need no stable order: for tied p
// at ranks j < k every ratio in [j, k) is >= the one at k (correctly rounded
// division is monotone), so the reverse minimum gives the whole tie the same
// q whatever order the sort left it in.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cmath>

#include "h3d.h"
#include "h3d_ctx.h"
#include "h3d_errors.h"

using namespace h3dint;
using h3derr::fail;

namespace {

constexpr int kBhBlock = 256;

// key = p where finite, +inf elsewhere (sorted behind every finite p);
// fin[i] = 1 where finite
__global__ void k_bh_keys(const double* __restrict__ p, int64_t n,
                          double* __restrict__ key, int32_t* __restrict__ idx,
                          int32_t* __restrict__ fin) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double v = p[i];
    const bool ok = isfinite(v);
    key[i] = ok ? v : INFINITY;
    idx[i] = (int32_t)i;
    fin[i] = ok ? 1 : 0;
  }
}

// rev[m - 1 - j] = p_sorted[j] / ((j + 1) / m)   (fdrcorrection: pvals / ecdf)
__global__ void k_bh_ratio(const double* __restrict__ ps, const int32_t* __restrict__ m_p,
                           double* __restrict__ rev) {
  const int64_t m = *m_p;
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m;
       j += (int64_t)gridDim.x * blockDim.x)
    rev[m - 1 - j] = ps[j] / ((double)(j + 1) / (double)m);
}

__global__ void k_bh_scatter(const double* __restrict__ scanned,
                             const int32_t* __restrict__ order,
                             const int32_t* __restrict__ m_p, int64_t n,
                             double* __restrict__ q) {
  const int64_t m = *m_p;
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    double v = NAN;
    if (j < m) {
      v = scanned[m - 1 - j];
      if (v > 1.0) v = 1.0;  // q[q > 1] = 1
    }
    q[order[j]] = v;
  }
}

struct MinOp {
  __device__ double operator()(double a, double b) const { return b < a ? b : a; }
};

// ---- BH over p-values sharded across ranks (parallel.bh_sharded) ----------
// Each rank sorts its own p-values (h3d_bh_sort_dev), ships them to the rank
// owning their VALUE range (equal values go to one rank), sorts what it
// receives, and knows from one all_gather of the bucket sizes the global
// rank of every value: ratio_j = p_(j) / ((offset + j + 1) / m), the same
// expression as h3d_bh_dev's at the same global j. The reverse minimum runs
// in the bucket (h3d_bh_scan_dev) and is completed with the minimum of the
// higher buckets (h3d_bh_finish_dev): min is exact, so every q has
// h3d_bh_dev's bits.

// key = p where finite, +inf elsewhere; val = the given values or 0..n-1
__global__ void k_bh_sort_in(const double* __restrict__ p,
                             const int64_t* __restrict__ val_in, int64_t n,
                             double* __restrict__ key, int64_t* __restrict__ val,
                             int32_t* __restrict__ fin) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double v = p[i];
    const bool ok = isfinite(v);
    key[i] = ok ? v : INFINITY;
    val[i] = val_in ? val_in[i] : i;
    fin[i] = ok ? 1 : 0;
  }
}

// rev[mb - 1 - j] = ps[j] / ((offset + j + 1) / m)
__global__ void k_bh_ratio_off(const double* __restrict__ ps, int64_t mb, int64_t offset,
                               int64_t m, double* __restrict__ rev) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < mb;
       j += (int64_t)gridDim.x * blockDim.x)
    rev[mb - 1 - j] = ps[j] / ((double)(offset + j + 1) / (double)m);
}

// scanned (ascending positions) <- the reverse-order inclusive min-scan
__global__ void k_bh_unreverse(const double* __restrict__ scan_rev, int64_t mb,
                               double* __restrict__ scanned) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < mb;
       j += (int64_t)gridDim.x * blockDim.x)
    scanned[j] = scan_rev[mb - 1 - j];
}

__global__ void k_bh_finish(const double* __restrict__ scanned, int64_t mb, double higher,
                            double* __restrict__ q) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < mb;
       j += (int64_t)gridDim.x * blockDim.x) {
    double v = scanned[j];
    if (higher < v) v = higher;
    if (v > 1.0) v = 1.0;
    q[j] = v;
  }
}

}  // namespace

extern "C" {

int h3d_bh_dev(h3d_ctx* ctx, const double* d_p, int64_t n, double* d_q) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  if (n == 0) return 0;
  if (n < 0 || !d_p || !d_q) return fail(H3D_EARG, "null argument");
  if (n >= ((int64_t)1 << 31)) return fail(H3D_EARG, "n too large (%lld)", (long long)n);
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  double* key = (double*)scratch(ctx, "bh_key", n * 8);
  double* key_s = (double*)scratch(ctx, "bh_key_s", n * 8);
  int32_t* idx = (int32_t*)scratch(ctx, "bh_idx", n * 4);
  int32_t* idx_s = (int32_t*)scratch(ctx, "bh_idx_s", n * 4);
  int32_t* fin = (int32_t*)scratch(ctx, "bh_fin", n * 4);
  int32_t* d_m = (int32_t*)scratch(ctx, "bh_m", 4);
  if (!key || !key_s || !idx || !idx_s || !fin || !d_m) return fail(H3D_ENOMEM, "bh scratch");
  ProfScope ps(ctx, "bh", n, 1);
  const int grid = grid_for(ctx, n);
  hipLaunchKernelGGL(k_bh_keys, dim3(grid), dim3(kBhBlock), 0, s, d_p, n, key, idx, fin);
  size_t tb = 0, tb2 = 0, tb3 = 0;
  HIP_TRY(hipcub::DeviceReduce::Sum(nullptr, tb, fin, d_m, (int)n, s));
  HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, key, key_s, idx, idx_s, (int)n, 0,
                                             64, s));
  // the ratios reuse `key` (SortPairs leaves its input unread afterwards)
  double* scanned = (double*)scratch(ctx, "bh_scan", n * 8);
  if (!scanned) return fail(H3D_ENOMEM, "bh scratch");
  HIP_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, tb3, key, scanned, MinOp(), (int)n, s));
  void* tmp = scratch(ctx, "cub_tmp_bh", std::max(tb, std::max(tb2, tb3)));
  if (!tmp) return fail(H3D_ENOMEM, "bh scratch");
  HIP_TRY(hipcub::DeviceReduce::Sum(tmp, tb, fin, d_m, (int)n, s));
  HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb2, key, key_s, idx, idx_s, (int)n, 0, 64,
                                             s));
  hipLaunchKernelGGL(k_bh_ratio, dim3(grid), dim3(kBhBlock), 0, s, key_s, d_m, key);
  // min-scan over the first m entries: the count lives on the device, so scan
  // all n -- entries >= m are never read (k_bh_scatter reads m - 1 - j < m)
  HIP_TRY(hipcub::DeviceScan::InclusiveScan(tmp, tb3, key, scanned, MinOp(), (int)n, s));
  hipLaunchKernelGGL(k_bh_scatter, dim3(grid), dim3(kBhBlock), 0, s, scanned, idx_s, d_m, n,
                     d_q);
  HIP_TRY(hipGetLastError());
  return 0;
}

int h3d_bh_sort_dev(h3d_ctx* ctx, const double* d_p, const int64_t* d_val, int64_t n,
                    double* d_key_out, int64_t* d_val_out, int64_t* m_finite) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  if (n < 0 || (n > 0 && (!d_p || !d_key_out || !d_val_out)))
    return fail(H3D_EARG, "null argument");
  if (n >= ((int64_t)1 << 31)) return fail(H3D_EARG, "n too large (%lld)", (long long)n);
  if (m_finite) *m_finite = 0;
  if (n == 0) return 0;
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  double* key = (double*)scratch(ctx, "bhs_key", n * 8);
  int64_t* val = (int64_t*)scratch(ctx, "bhs_val", n * 8);
  int32_t* fin = (int32_t*)scratch(ctx, "bhs_fin", n * 4);
  int32_t* d_m = (int32_t*)scratch(ctx, "bhs_m", 4);
  if (!key || !val || !fin || !d_m) return fail(H3D_ENOMEM, "bh sort scratch");
  ProfScope ps(ctx, "bh", n, 1);
  const int grid = grid_for(ctx, n);
  hipLaunchKernelGGL(k_bh_sort_in, dim3(grid), dim3(kBhBlock), 0, s, d_p, d_val, n, key, val,
                     fin);
  size_t tb = 0, tb2 = 0;
  HIP_TRY(hipcub::DeviceReduce::Sum(nullptr, tb, fin, d_m, (int)n, s));
  HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, key, d_key_out, val, d_val_out,
                                             (int)n, 0, 64, s));
  void* tmp = scratch(ctx, "cub_tmp_bhs", std::max(tb, tb2));
  if (!tmp) return fail(H3D_ENOMEM, "bh sort scratch");
  HIP_TRY(hipcub::DeviceReduce::Sum(tmp, tb, fin, d_m, (int)n, s));
  HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb2, key, d_key_out, val, d_val_out, (int)n,
                                             0, 64, s));
  HIP_TRY(hipGetLastError());
  if (m_finite) {
    int32_t hm = 0;
    HIP_TRY(hipMemcpyAsync(&hm, d_m, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *m_finite = hm;
  }
  return 0;
}

int h3d_bh_scan_dev(h3d_ctx* ctx, const double* d_ps, int64_t mb, int64_t offset,
                    int64_t m, double* d_scanned, double* bucket_min) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  if (bucket_min) *bucket_min = INFINITY;
  if (mb < 0 || offset < 0 || offset + mb > m) return fail(H3D_EARG, "bad bucket range");
  if (mb == 0) return 0;
  if (!d_ps || !d_scanned) return fail(H3D_EARG, "null argument");
  if (mb >= ((int64_t)1 << 31)) return fail(H3D_EARG, "bucket too large (%lld)", (long long)mb);
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  double* rev = (double*)scratch(ctx, "bhs_rev", mb * 8);
  double* srev = (double*)scratch(ctx, "bhs_srev", mb * 8);
  if (!rev || !srev) return fail(H3D_ENOMEM, "bh scan scratch");
  ProfScope ps(ctx, "bh", mb, 1);
  const int grid = grid_for(ctx, mb);
  hipLaunchKernelGGL(k_bh_ratio_off, dim3(grid), dim3(kBhBlock), 0, s, d_ps, mb, offset, m,
                     rev);
  size_t tb = 0;
  HIP_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, tb, rev, srev, MinOp(), (int)mb, s));
  void* tmp = scratch(ctx, "cub_tmp_bhs2", tb);
  if (!tmp) return fail(H3D_ENOMEM, "bh scan scratch");
  HIP_TRY(hipcub::DeviceScan::InclusiveScan(tmp, tb, rev, srev, MinOp(), (int)mb, s));
  hipLaunchKernelGGL(k_bh_unreverse, dim3(grid), dim3(kBhBlock), 0, s, srev, mb, d_scanned);
  HIP_TRY(hipGetLastError());
  if (bucket_min) {
    // the whole bucket's minimum = the scan's last entry
    HIP_TRY(hipMemcpyAsync(bucket_min, srev + (mb - 1), 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  return 0;
}

int h3d_bh_finish_dev(h3d_ctx* ctx, const double* d_scanned, int64_t mb, double higher_min,
                      double* d_q) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  if (mb < 0) return fail(H3D_EARG, "bad bucket size");
  if (mb == 0) return 0;
  if (!d_scanned || !d_q) return fail(H3D_EARG, "null argument");
  HIP_TRY(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(k_bh_finish, dim3(grid_for(ctx, mb)), dim3(kBhBlock), 0, ctx->stream,
                     d_scanned, mb, higher_min, d_q);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int h3d_bh_ctx(h3d_ctx* ctx, const double* p, int64_t n, double* q) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  if (n == 0) return 0;
  if (n < 0 || !p || !q) return fail(H3D_EARG, "null argument");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  double* d_p = (double*)scratch(ctx, "bh_in", n * 8);
  double* d_q = (double*)scratch(ctx, "bh_out", n * 8);
  if (!d_p || !d_q) return fail(H3D_ENOMEM, "bh buffers");
  HIP_TRY(hipMemcpyAsync(d_p, p, n * 8, hipMemcpyHostToDevice, s));
  if (int rc = h3d_bh_dev(ctx, d_p, n, d_q)) return rc;
  HIP_TRY(hipMemcpyAsync(q, d_q, n * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return 0;
}

}  // extern "C"
