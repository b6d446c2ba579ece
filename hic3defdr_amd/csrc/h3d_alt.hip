// libh3d.so, second TU: the alternative models of the reference's
// analysis/alternatives.py on the GPU.
//
//   h3d_lrt_poisson   <- alternatives.py:17-42 (poisson_fit_mu_hat,
//                        poisson_logpmf, poisson_lrt), Poisson3DeFDR.lrt
//   h3d_mme_per_pixel <- util/dispersion.py:83-104 mme_per_pixel (+ the
//                        np.maximum floor of Unsmoothed3DeFDR,
//                        alternatives.py:133-134)
//
// Global3DeFDR needs no kernel of its own: its single qcml per condition over
// the loop pixels is h3d_disp_per_dist with one distance segment.
//
// Layout as the main LRT (h3d_kernels.h): pixels in the reference order,
// replicate-minor rows; one lane per pixel. Both kernels are light (a few
// logs / lgammas per replicate), i.e. HBM-bound: 12R + 16C + 16 B/px
// (Poisson: raw int32 + f in; p, llr, mu0, mu1 out) and 8R + 8C B/px (MME).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "h3d.h"
#include "h3d_ctx.h"
#include "h3d_errors.h"
#include "h3d_model.h"

using namespace h3d;
using namespace h3dint;
using h3derr::fail;

namespace {

constexpr int kAltBlock = 256;

// scipy.stats.poisson(mu).logpmf(k) for integer k >= 0 (scipy 1.7.1
// rv_discrete.logpmf: mu < 0 or NaN -> NaN; _logpmf = xlogy(k, mu) -
// gammaln(k + 1) - mu, xlogy(0, mu) = 0 for non-NaN mu)
__device__ inline double poisson_logpmf(double k, double mu) {
  if (!(mu >= 0.0)) return NAN;
  const double xl = (k == 0.0) ? 0.0 : k * log(mu);
  return xl - lgam(k + 1.0) - mu;
}

// numpy sum of the replicates k < n selected by `mask`, in order: the
// compacted row (as raw[:, design[:, c]] builds it) summed with numpy's row
// association (sequential below 8 values, pairwise from 8)
template <int M>
__device__ inline double np_sum_mask(const double* v, int n, unsigned mask) {
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < M; ++k) cnt += (k < n && ((mask >> k) & 1u)) ? 1 : 0;
  if (cnt < 8) {
    double res = 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k)
      if (k < n && ((mask >> k) & 1u)) res += v[k];
    return res;
  }
  if constexpr (M >= 8) {
    double t[M];  // rare (>= 8 replicates in one condition)
    int j = 0;
    for (int k = 0; k < n; ++k)
      if ((mask >> k) & 1u) t[j++] = v[k];
    return np_sum<M>(t, cnt);
  }
  return NAN;
}

// np.average(raw / f, weights=f, axis=1) over the masked replicates
// (alternatives.py:17-18): sum((raw / f) * f) / sum(f)
template <int M>
__device__ inline double poisson_mu(const double* x, const double* f, int n,
                                    unsigned mask) {
  double aw[M];
#pragma unroll
  for (int k = 0; k < M; ++k) aw[k] = (k < n) ? (x[k] / f[k]) * f[k] : 0.0;
  return np_sum_mask<M>(aw, n, mask) / np_sum_mask<M>(f, n, mask);
}

template <int M, int CM>
__global__ __launch_bounds__(kAltBlock) void k_lrt_poisson(
    const int32_t* __restrict__ raw, const double* __restrict__ f, int64_t n,
    int R, int C, const int32_t* __restrict__ cond_of_rep,
    double* __restrict__ p, double* __restrict__ llr, double* __restrict__ mu0,
    double* __restrict__ mu1) {
  int cond[M];
#pragma unroll
  for (int k = 0; k < M; ++k) cond[k] = (k < R) ? cond_of_rep[k] : -1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double x[M], fv[M];
#pragma unroll
    for (int k = 0; k < M; ++k) {
      x[k] = (k < R) ? (double)raw[i * R + k] : 0.0;
      fv[k] = (k < R) ? f[i * R + k] : 1.0;
    }
    const double m0 = poisson_mu<M>(x, fv, R, ~0u);
    double m1[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) {
      unsigned mask = 0u;
#pragma unroll
      for (int k = 0; k < M; ++k)
        if (k < R && cond[k] == c) mask |= 1u << k;
      m1[c] = (c < C) ? poisson_mu<M>(x, fv, R, mask) : 0.0;
    }
    // null / alt log likelihoods, row sums in replicate order (:38-39);
    // mu_hat_alt_wide = dot(mu_hat_alt, design.T) picks each replicate's
    // own condition (one-hot design)
    double tn[M], ta[M];
#pragma unroll
    for (int k = 0; k < M; ++k) {
      if (k < R) {
        double ma = 0.0;
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (c == cond[k]) ma = m1[c];
        tn[k] = poisson_logpmf(x[k], m0 * fv[k]);
        ta[k] = poisson_logpmf(x[k], ma * fv[k]);
      } else {
        tn[k] = ta[k] = 0.0;
      }
    }
    const double l = np_sum<M>(tn, R) - np_sum<M>(ta, R);
    llr[i] = l;
    p[i] = chi2_sf((double)(C - 1), -2 * l);
    mu0[i] = m0;
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) mu1[i * C + c] = m1[c];
  }
}

// mme_per_pixel (dispersion.py:83-104) of every condition's replicate block:
// m = mean, v = var(ddof=1) (numpy: sum / n, then sum((x - m)^2) / (n - 1)),
// inverse_mvr = (v - m) / m^2 (scaled_nb.py:53-68); then
// np.maximum(., min_disp) (NaN propagates, as numpy's maximum)
template <int M>
__global__ __launch_bounds__(kAltBlock) void k_mme_per_pixel(
    const double* __restrict__ data, const double* __restrict__ f, int64_t n,
    int R, int C, const int32_t* __restrict__ cond_of_rep, double min_disp,
    double* __restrict__ disp) {
  int cond[M];
#pragma unroll
  for (int k = 0; k < M; ++k) cond[k] = (k < R) ? cond_of_rep[k] : -1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double v[M];
#pragma unroll
    for (int k = 0; k < M; ++k) {
      v[k] = (k < R) ? data[i * R + k] : 0.0;
      if (f && k < R) v[k] = v[k] / f[i * R + k];
    }
    for (int c = 0; c < C; ++c) {
      unsigned mask = 0u;
      int cnt = 0;
#pragma unroll
      for (int k = 0; k < M; ++k)
        if (k < R && cond[k] == c) {
          mask |= 1u << k;
          ++cnt;
        }
      const double m = np_sum_mask<M>(v, R, mask) / cnt;
      double sq[M];
#pragma unroll
      for (int k = 0; k < M; ++k) {
        const double d = v[k] - m;
        sq[k] = d * d;
      }
      const double var = np_sum_mask<M>(sq, R, mask) / (double)(cnt > 1 ? cnt - 1 : 0);
      double r = (var - m) / (m * m);
      if (r == r && r < min_disp) r = min_disp;
      disp[i * C + c] = r;
    }
  }
}

int alt_grid(h3d_ctx* ctx, int64_t n) { return grid_for(ctx, n, 16); }

// raw int64 (caller's host array) -> device int32, rejecting counts the
// int32 kernels cannot hold
__global__ void k_i64_to_i32_alt(const int64_t* __restrict__ in,
                                 int32_t* __restrict__ out, int64_t n,
                                 int* __restrict__ overflow) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = in[i];
    if (v < 0 || v > 0x7fffffffLL) atomicOr(overflow, 1);
    out[i] = (int32_t)v;
  }
}

}  // namespace

extern "C" {

int h3d_lrt_poisson_dev(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                        int64_t n, int R, int C, const int32_t* cond_of_rep,
                        double* d_p, double* d_llr, double* d_mu0,
                        double* d_mu1) {
  if (!ctx || !cond_of_rep) return fail(H3D_EARG, "null argument");
  std::vector<int> nrep;
  std::vector<int32_t> rep_idx;
  if (int rc = check_cond(cond_of_rep, R, C, &nrep, &rep_idx)) return rc;
  if (n == 0) return 0;
  if (!d_raw || !d_f || !d_p || !d_llr || !d_mu0 || !d_mu1)
    return fail(H3D_EARG, "null device buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  int32_t* d_cond = (int32_t*)scratch(ctx, "cond_of_rep", R * 4);
  if (!d_cond) return fail(H3D_ENOMEM, "poisson scratch");
  HIP_TRY(hipMemcpyAsync(d_cond, cond_of_rep, R * 4, hipMemcpyHostToDevice, s));
  const int grid = alt_grid(ctx, n);
  const int m = R <= 4 ? 4 : R <= 8 ? 8 : R <= 16 ? 16 : 32;
  const int cm = C <= 2 ? 2 : C <= 4 ? 4 : 8;
  {
    ProfScope ps(ctx, "lrt_poisson", n, 1);
#define H3D_PLRT(MM, CC)                                                      \
  hipLaunchKernelGGL((k_lrt_poisson<MM, CC>), dim3(grid), dim3(kAltBlock), 0, s, \
                     d_raw, d_f, n, R, C, d_cond, d_p, d_llr, d_mu0, d_mu1)
    if (m == 4 && cm == 2) H3D_PLRT(4, 2);
    else if (m == 4) H3D_PLRT(4, 4);
    else if (m == 8 && cm <= 4) H3D_PLRT(8, 4);
    else if (m <= 16) H3D_PLRT(16, 8);
    else H3D_PLRT(32, 8);
#undef H3D_PLRT
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

int h3d_lrt_poisson(h3d_ctx* ctx, const int64_t* raw, const double* f,
                    int64_t n, int R, int C, const int32_t* cond_of_rep,
                    double* p, double* llr, double* mu0, double* mu1) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  if (n == 0) return 0;
  if (!raw || !f || !p || !llr || !mu0 || !mu1) return fail(H3D_EARG, "null buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  int64_t* d_raw64 = (int64_t*)scratch(ctx, "in_raw64", n * R * 8);
  int32_t* d_raw = (int32_t*)scratch(ctx, "in_raw", n * R * 4);
  double* d_f = (double*)scratch(ctx, "in_f", n * R * 8);
  double* d_out = (double*)scratch(ctx, "plrt_out", n * (3 + C) * 8);
  int* d_ovf = (int*)scratch(ctx, "ovf", 4);
  if (!d_raw64 || !d_raw || !d_f || !d_out || !d_ovf)
    return fail(H3D_ENOMEM, "poisson inputs");
  HIP_TRY(hipMemcpyAsync(d_raw64, raw, n * R * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_f, f, n * R * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(d_ovf, 0, 4, s));
  hipLaunchKernelGGL(k_i64_to_i32_alt, dim3(grid_for(ctx, n * R)), dim3(kAltBlock), 0,
                     s, d_raw64, d_raw, n * R, d_ovf);
  double *dp = d_out, *dl = d_out + n, *dm0 = d_out + 2 * n, *dm1 = d_out + 3 * n;
  int rc = h3d_lrt_poisson_dev(ctx, d_raw, d_f, n, R, C, cond_of_rep, dp, dl, dm0, dm1);
  if (rc) return rc;
  int ovf = 0;
  HIP_TRY(hipMemcpyAsync(&ovf, d_ovf, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(p, dp, n * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(llr, dl, n * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(mu0, dm0, n * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(mu1, dm1, n * C * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (ovf) return fail(H3D_EINPUT, "raw counts must be in [0, 2^31)");
  return 0;
}

int h3d_mme_per_pixel(h3d_ctx* ctx, const double* data, const double* f,
                      int64_t n, int R, int C, const int32_t* cond_of_rep,
                      double min_disp, double* disp) {
  if (!ctx || !cond_of_rep) return fail(H3D_EARG, "null argument");
  std::vector<int> nrep;
  std::vector<int32_t> rep_idx;
  if (int rc = check_cond(cond_of_rep, R, C, &nrep, &rep_idx)) return rc;
  if (n == 0) return 0;
  if (!data || !disp) return fail(H3D_EARG, "null buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  double* d_data = (double*)scratch(ctx, "mme_in", n * R * 8);
  double* d_f = f ? (double*)scratch(ctx, "mme_f", n * R * 8) : nullptr;
  double* d_out = (double*)scratch(ctx, "mme_out", n * C * 8);
  int32_t* d_cond = (int32_t*)scratch(ctx, "cond_of_rep", R * 4);
  if (!d_data || (f && !d_f) || !d_out || !d_cond) return fail(H3D_ENOMEM, "mme scratch");
  HIP_TRY(hipMemcpyAsync(d_data, data, n * R * 8, hipMemcpyHostToDevice, s));
  if (f) HIP_TRY(hipMemcpyAsync(d_f, f, n * R * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_cond, cond_of_rep, R * 4, hipMemcpyHostToDevice, s));
  const int grid = alt_grid(ctx, n);
  {
    ProfScope ps(ctx, "mme", n, 1);
    if (R <= 4)
      hipLaunchKernelGGL(k_mme_per_pixel<4>, dim3(grid), dim3(kAltBlock), 0, s, d_data,
                         d_f, n, R, C, d_cond, min_disp, d_out);
    else if (R <= 8)
      hipLaunchKernelGGL(k_mme_per_pixel<8>, dim3(grid), dim3(kAltBlock), 0, s, d_data,
                         d_f, n, R, C, d_cond, min_disp, d_out);
    else
      hipLaunchKernelGGL(k_mme_per_pixel<32>, dim3(grid), dim3(kAltBlock), 0, s, d_data,
                         d_f, n, R, C, d_cond, min_disp, d_out);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(disp, d_out, n * C * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return 0;
}

}  // extern "C"
