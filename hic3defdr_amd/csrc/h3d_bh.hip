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
