// k_lrt8: the per-pixel LRT (lrt.py:7-50) for wide designs (R > 8, the
// R = 18 / C = 3 shape of BASELINE cfg4), one pixel per GROUP OF 8 LANES.
//
// k_lrt holds a pixel's R replicates in one lane's registers: past R = 8 that
// is > 256 VGPRs (x, f, a rows + the unrolled fits) and the compiler spills
// to scratch (measured at M = 32: 1 KiB scratch per lane, 1 wave/SIMD, 26.9 ms
// per cfg4 lrt). Here lane j of a group owns replicates j, j + 8, j + 16, ...
// (M / 8 slots), so the row reads are 8 contiguous values per group and the
// per-lane state is M / 8 slots.
//
// Sums over replicates go through a 3-level xor butterfly inside the group.
// For the two log-likelihood rows that butterfly IS numpy's association
// (pairwise_sum, n >= 8: accumulator j sums elements j, j + 8, ... of the
// 8-aligned block, then ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)),
// then the n % 8 tail in order) -- the same bits as lrt_pixel's np_sum, and
// every lane of the group ends with the same value (IEEE addition commutes),
// so the Newton iterations of the group stay in lockstep and the group exits
// its loops together.
#pragma once

#include "h3d_kernels.h"

namespace h3d {

constexpr int kGroup = 8;

__device__ inline double gsum8(double v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}
__device__ inline int gor8(int v) {
  v |= __shfl_xor(v, 1, 64);
  v |= __shfl_xor(v, 2, 64);
  v |= __shfl_xor(v, 4, 64);
  return v;
}

// numpy's sum of a group-distributed row of n >= 8 values (element k in lane
// k % 8, slot k / 8): the slot loop per lane, the butterfly, the tail.
template <int J>
__device__ inline double np_sum_g8(const double* v, int n, int lane, int base) {
  const int blk = n - n % 8;
  double r = v[0];
#pragma unroll
  for (int s = 1; s < J; ++s)
    if (lane + 8 * s < blk) r += v[s];
  double res = gsum8(r);
  // tail: elements blk .. n-1 all sit in slot blk / 8
  const int st = blk / 8;
  double tv = 0.0;
#pragma unroll
  for (int s = 0; s < J; ++s)
    if (s == st) tv = v[s];
  for (int t = 0; t < n - blk; ++t) res += __shfl(tv, base + t, 64);
  return res;
}

// fit_mu (h3d_model.h) over the group: same bracketed Newton on
// g(theta) = mu S(mu), sums by butterfly (any fixed order; the root is
// unique and the solve runs to full precision). `slots` = this lane's bits of
// the fit's replicate mask (bit s: replicate lane + 8 s).
template <int J>
__device__ double fit_mu_g8(const int32_t* x, const double* b, const double* a,
                            unsigned slots, int* status) {
  double sx = 0.0, init = 0.0, cnt = 0.0;
  int bad = 0;
#pragma unroll
  for (int s = 0; s < J; ++s)
    if ((slots >> s) & 1u) {
      bad |= (!(a[s] > 0.0) || !(b[s] > 0.0) || is_inf(a[s]) || is_inf(b[s]) ||
              !(x[s] >= 0))
                 ? 1
                 : 0;
      sx += (double)x[s];
      init += (double)x[s] / b[s];
      cnt += 1.0;
    }
  bad = gor8(bad);
  sx = gsum8(sx);
  init = gsum8(init);
  cnt = gsum8(cnt);
  if (bad) {
    *status |= kFlagBadInput;
    return NAN;
  }
  if (!(sx > 0.0)) {
    *status |= kFlagNoRoot;
    return NAN;
  }
  double th = log_fast_checked(init / cnt);
  double lo = -INFINITY, hi = INFINITY;
  for (int it = 0; it < 200; ++it) {
    const double mu = exp_fast(th);
    double g = 0.0, gp = 0.0;
#pragma unroll
    for (int s = 0; s < J; ++s)
      if ((slots >> s) & 1u) {
        const double mb = mu * b[s];
        const double den = 1.0 / (1.0 + a[s] * mb);
        g += ((double)x[s] - mb) * den;
        gp -= mb * (1.0 + a[s] * (double)x[s]) * den * den;
      }
    g = gsum8(g);
    gp = gsum8(gp);
    if (g > 0.0)
      lo = th;
    else if (g < 0.0)
      hi = th;
    else
      return mu;
    const double dn = g / gp;
    if (fabs(dn) <= 1e-8 * fmax(1.0, fabs(th))) return exp_fast(th - dn);
    double tn = th - dn;
    if (!(tn > lo && tn < hi)) {
      if (is_inf(lo))
        tn = hi - 2.0;
      else if (is_inf(hi))
        tn = lo + 2.0;
      else
        tn = 0.5 * (lo + hi);
    }
    const double step = fabs(tn - th);
    th = tn;
    if (step <= 1e-15 * fmax(1.0, fabs(th))) return exp_fast(th);
    if (!is_inf(lo) && !is_inf(hi) && (hi - lo) <= 4e-16 * fmax(1.0, fabs(th)))
      return exp_fast(th);
  }
  *status |= kFlagNoConv;
  return exp_fast(th);
}

// M = 16 / 24 / 32 (R <= M), CM >= C. Same arguments and outputs as k_lrt.
template <int M, int CM>
// 2 waves per SIMD (<= 256 registers). (With the table log in its logpmf
// rows the M = 32 instantiation grew into AGPRs at 1 wave -- cfg4 lrt 22.7
// -> 31.0 ms, r03i --, while the rows still carried the cancelling prefix;
// without it the rows take the table log from LDS, as k_lrt.)
__global__ __launch_bounds__(kBlock, 2) void k_lrt8(
    const int32_t* __restrict__ raw, const double* __restrict__ f,
    const int32_t* __restrict__ dist, const double* __restrict__ table,
    int64_t n, int R, int C, int D, const int32_t* __restrict__ cond_of_rep,
    int refit, double* __restrict__ p, double* __restrict__ llr,
    double* __restrict__ mu0, double* __restrict__ mu1,
    double* __restrict__ disp_out, int* __restrict__ flags, int wide) {
  constexpr int J = M / kGroup;
  const int lane = threadIdx.x & (kGroup - 1);
  const int base = (threadIdx.x & 63) & ~(kGroup - 1);  // group's first lane
  __shared__ LogTab s_tab[129];  // the rows' log table, as k_lrt
  for (int t = threadIdx.x; t < 129; t += blockDim.x) s_tab[t] = kLogTab[t];
  __syncthreads();
  int cnd[J];
#pragma unroll
  for (int s = 0; s < J; ++s) {
    const int k = lane + kGroup * s;
    cnd[s] = (k < R) ? cond_of_rep[k] : -1;
  }
  int fl_all = 0;
  const int64_t groups = (int64_t)gridDim.x * (blockDim.x / kGroup);
  for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kGroup; i < n;
       i += groups) {
    const int d = dist ? dist[i] : 0;
    const double* trow = dist ? table + (int64_t)d * C : table + i * (wide ? R : C);
    const bool inb = dist ? (d >= 0 && d < D) : true;
    double dc[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) dc[c] = (c < C && inb && !wide) ? trow[c] : NAN;
    int32_t x[J];
    double fv[J], a[J];
#pragma unroll
    for (int s = 0; s < J; ++s) {
      const int k = lane + kGroup * s;
      if (k < R) {
        x[s] = raw[i * R + k];
        fv[s] = f[i * R + k];
        double ak = 0.0;
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (c == cnd[s]) ak = dc[c];
        a[s] = wide ? trow[k] : ak;
      } else {
        x[s] = 0;
        fv[s] = 1.0;
        a[s] = 1.0;
      }
    }
    int st = 0;
    double m0 = 0.0, m1[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) m1[c] = 0.0;
    // fit 0 the null, fit t = c + 1 condition c (lrt_pixel's loop)
#pragma unroll 1
    for (int t = 0; t <= C; ++t) {
      unsigned slots = 0u;
#pragma unroll
      for (int s = 0; s < J; ++s)
        if (lane + kGroup * s < R && (t == 0 || cnd[s] == t - 1)) slots |= 1u << s;
      double mu;
      if (refit) {
        mu = fit_mu_g8<J>(x, fv, a, slots, &st);
      } else {
        // np.mean(raw / f) of the fit's replicates in replicate order: every
        // lane walks the compacted row (values fetched from their lanes)
        double q[J];
#pragma unroll
        for (int s = 0; s < J; ++s) q[s] = (double)x[s] / fv[s];
        unsigned rows = 0u;  // replicate mask of the fit (R <= 32)
#pragma unroll
        for (int s = 0; s < J; ++s)
          if ((slots >> s) & 1u) rows |= 1u << (lane + kGroup * s);
        rows = (unsigned)gor8((int)rows);
        const int cnt = __popc(rows);
        NpSumStream acc(cnt);
        int j = 0;
#pragma unroll
        for (int k = 0; k < M; ++k)
          if ((rows >> k) & 1u) {
            const double v = __shfl(q[k / kGroup], base + k % kGroup, 64);
            acc.add_dyn(j++, v);
          }
        mu = acc.sum() / cnt;
      }
      if (t == 0) m0 = mu;
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c == t - 1) m1[c] = mu;
    }
    // log-likelihood rows (lrt_pixel: same terms, same bits per replicate)
    double tn[J], ta[J];
#pragma unroll
    for (int s = 0; s < J; ++s) {
      double m1k = 0.0;
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c == cnd[s]) m1k = m1[c];
      const double xk = (double)x[s];
      const double r = 1.0 / a[s];
      // the mean-free prefix of logpmf is common to the null and alt rows
      // and cancels in llr: left out, as k_lrt (lrt_pixel)
      const double m0k = m0 * fv[s], m1f = m1k * fv[s];
      const double l0 = log_fast_checked(r + m0k, s_tab);
      const double l1 = log_fast_checked(r + m1f, s_tab);
      tn[s] = -r * l0 + xk * log_fast_checked(m0k, s_tab) - xk * l0;
      ta[s] = -r * l1 + xk * log_fast_checked(m1f, s_tab) - xk * l1;
    }
    const double lv = np_sum_g8<J>(tn, R, lane, base) - np_sum_g8<J>(ta, R, lane, base);
    fl_all |= st;
    if (lane == 0) {
      p[i] = chi2_sf((double)(C - 1), -2 * lv);
      llr[i] = lv;
      mu0[i] = m0;
    }
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C && c == lane) {
        mu1[i * C + c] = m1[c];
        if (disp_out) disp_out[i * C + c] = dc[c];
      }
  }
  fl_all = gor8(fl_all);
  if (fl_all && lane == 0) atomicOr(flags, fl_all);
}

}  // namespace h3d
