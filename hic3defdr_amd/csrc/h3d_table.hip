// libh3d.so: the dispersion-vs-distance smoother on the device
// (h3d_disp_tables_dev): weighted_lowess_fit / lowess_fit (reference
// util/lowess.py:10-244, as estimate_disp calls it at analysis.py:226-240)
// evaluated at every distance, one workgroup per condition, so the estimate_disp
// -> lrt step never leaves the GPU (the host smoother h3d_disp_tables costs a
// device->host->device round trip and ~0.3-0.5 ms of idle GPU per step).
//
// Same arithmetic as the host restatement (h3d_host.h, op for op, no FMA
// contraction), re-organised for a workgroup:
//  * the rolling variance (pandas Welford + Kahan) is one serial chain: one
//    thread;
//  * the weighted fit replicates distance i floor(w_i) times; every copy has
//    the same x and y, so the points are held as RUNS (distance, count) and a
//    point index maps to its run by binary search over the run starts;
//  * statsmodels' sliding window for a fit at x is the first window whose
//    midpoint (x[l] + x[l + k]) / 2 is >= x (the slide is monotone), so each
//    fit's window is found independently;
//  * the delta-skipping schedule (which points get a local fit, the others
//    interpolated) depends on x alone: the next fit run of each run is found
//    in parallel, the chain from run 0 followed by one thread;
//  * the local fits (the host's sequential sums over the window's runs, same
//    order) run one thread per fit point, the interpolation one thread per run;
//  * the median of |residual| over the points is a count-weighted order
//    statistic over the runs.
// Fits with a non-finite value (a degenerate window: every point at one x)
// are left to the host restatement, whose point-by-point NaN propagation
// this does not restate: the status word says so and h3d_lrt_dev_tab redoes
// the table on the host.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "h3d.h"
#include "h3d_ctx.h"
#include "h3d_errors.h"
#include "h3d_host.h"
#include "h3d_model.h"  // kMaxConds

#pragma clang fp contract(off)

using namespace h3dint;
using h3d::kMaxConds;
using h3derr::fail;

namespace h3dtab {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxD = h3dint::kTableMaxD;  // distances per table held in LDS
constexpr int kRobustIters = 3;
constexpr int kRollWindow = 20;
constexpr int kStamps = 16;

enum : int { kOk = 0, kFail = 1, kDegenerate = 2 };

// LDS bytes of one condition's working set at D distances
__host__ __device__ constexpr size_t lds_bytes(int D) {
  return (size_t)D * (10 * sizeof(double) + 2 * sizeof(int64_t) + 5 * sizeof(int)) +
         sizeof(int64_t);
}

// ---- block helpers (kThreads = 4 waves) -----------------------------------

struct Shared {
  int64_t i64[kWaves];
  double f64[kWaves];
  int i32[kWaves];
};

// exclusive prefix sum over the block; *total = the block's sum
__device__ int64_t scan_excl(int64_t v, Shared& sh, int64_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) sh.i64[wid] = x;
  __syncthreads();
  int64_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    if (w < wid) base += sh.i64[w];
    tot += sh.i64[w];
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

__device__ double block_min(double v, Shared& sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmin(v, __shfl_xor(v, off, 64));
  if (lane == 0) sh.f64[wid] = v;
  __syncthreads();
  double r = sh.f64[0];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) r = fmin(r, sh.f64[w]);
  __syncthreads();
  return r;
}

__device__ double block_max(double v, Shared& sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  if (lane == 0) sh.f64[wid] = v;
  __syncthreads();
  double r = sh.f64[0];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) r = fmax(r, sh.f64[w]);
  __syncthreads();
  return r;
}

__device__ int block_min_int(int v, Shared& sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
  if (lane == 0) sh.i32[wid] = v;
  __syncthreads();
  int r = sh.i32[0];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) r = min(r, sh.i32[w]);
  __syncthreads();
  return r;
}

__device__ int block_or(int v, Shared& sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v |= __shfl_xor(v, off, 64);
  if (lane == 0) sh.i32[wid] = v;
  __syncthreads();
  int r = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) r |= sh.i32[w];
  __syncthreads();
  return r;
}

// numpy pairwise_sum (h3d_host.h np_pairwise), unrolled recursion
template <int Depth>
__device__ double pairwise(const double* a, int64_t n) {
  if (n < 8) {
    double res = 0.0;
    for (int64_t i = 0; i < n; ++i) res += a[i];
    return res;
  }
  if (n <= 128 || Depth == 0) {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  if constexpr (Depth > 0) {
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise<Depth - 1>(a, n2) + pairwise<Depth - 1>(a + n2, n - n2);
  }
  return 0.0;
}

// run of point p: the last run whose start is <= p (rp[0] = 0, rp[U] = n)
__device__ int run_of(const int64_t* rp, int U, int64_t p) {
  int lo = 0, hi = U - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (rp[mid] <= p) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// scipy interp1d(kind='linear', fill_value='extrapolate') (h3d_host.h)
__device__ double interp_extrap(const double* xp, const double* yp, int m, double xn) {
  int lo = 0, hi = m;  // lower_bound
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (xp[mid] < xn) lo = mid + 1;
    else hi = mid;
  }
  int idx = lo < 1 ? 1 : (lo > m - 1 ? m - 1 : lo);
  const double slope = (yp[idx] - yp[idx - 1]) / (xp[idx] - xp[idx - 1]);
  return slope * (xn - xp[idx - 1]) + yp[idx - 1];
}

// a / b for b in {1, ..., 20} (the rolling window's counts), r = 1 / b:
// one Markstein correction of a * r -- correctly rounded, so equal to the
// IEEE quotient (r = RN(1/b) and the residual a - b y is exact with the FMA;
// 4e8 random (a, b) pairs checked on the host, and the tables are held
// bit-equal to the host smoother in tests/test_gpu_table.py). 3 dependent
// ops instead of the ~10 of the general division sequence, on the serial
// chain of the rolling variance.
__device__ double div_small(double a, double b, double r) {
  const double y = a * r;
  return fma(fma(-b, y, a), r, y);
}

// pandas rolling(20, center=True).var() (ddof 1) of v[0, n) into out: one
// thread (h3d_host.h rolling_var_center, whose Welford + Kahan updates are a
// single serial chain). The values are the finite points, so no update
// skips a NaN, and consecutive windows always overlap (they move by one:
// at most one removal and one addition per output); the next values are
// loaded one output ahead, off the chain.
__device__ void rolling_var(const double* v, int64_t n, double* out) {
  constexpr int64_t w = kRollWindow, offset = (w - 1) / 2;
  double mean_x = 0, ssqdm = 0, nobs = 0, comp_add = 0, comp_rem = 0;
  double prev = v[0];
  int64_t consec = 0;
  auto add = [&](double val) {
    nobs += 1;
    consec = (val == prev) ? consec + 1 : 1;
    prev = val;
    const double r = 1.0 / nobs;  // off the chain (nobs is a count)
    double prev_mean = mean_x - comp_add;
    double y = val - comp_add;
    double t = y - mean_x;
    comp_add = t + mean_x - y;
    mean_x = mean_x + div_small(t, nobs, r);
    ssqdm = ssqdm + (val - prev_mean) * (val - mean_x);
  };
  auto rem = [&](double val) {
    nobs -= 1;
    if (nobs) {
      const double r = 1.0 / nobs;
      double prev_mean = mean_x - comp_rem;
      double y = val - comp_rem;
      double t = y - mean_x;
      comp_rem = t + mean_x - y;
      mean_x = mean_x - div_small(t, nobs, r);
      ssqdm = ssqdm - (val - prev_mean) * (val - mean_x);
    } else {
      mean_x = 0;
      ssqdm = 0;
    }
  };
  auto emit = [&](int64_t i) {
    if (nobs >= w && nobs > 1)
      out[i] = (nobs == 1 || consec >= nobs) ? 0.0 : ssqdm / (nobs - 1.0);
    else
      out[i] = NAN;
  };
  // output 0: the window [0, min(offset + 1, n))
  int64_t ps = 0, pe = offset + 1 < n ? offset + 1 : n;
  for (int64_t j = 0; j < pe; ++j) add(v[j]);
  emit(0);
  // outputs 1.. : the window [max(i - 10, 0), min(i + 10, n)); a removal
  // for i >= 11, an addition for i <= n - 10 -- in between (the bulk) both,
  // with the counts fixed at 19 / 20 and the output divisor 19
  auto step = [&](int64_t i) {
    const int64_t s = i + 1 + offset - w > 0 ? i + 1 + offset - w : 0;
    const int64_t e = i + 1 + offset < n ? i + 1 + offset : n;
    if (s > ps) rem(v[ps]);
    if (e > pe) add(v[pe]);
    ps = s;
    pe = e;
    emit(i);
  };
  const int64_t b0 = w - offset;       // 11: the first output with a removal
  const int64_t b1 = n - offset - 1;   // n - 10: the last with an addition
  int64_t i = 1;
  for (; i < n && i < b0; ++i) step(i);
  if (i <= b1 && nobs == w) {
    constexpr double r19 = 1.0 / 19.0, r20 = 1.0 / 20.0;
    double nv_rem = v[i - b0], nv_add = v[i + offset];
    for (; i <= b1; ++i) {
      const double vr = nv_rem, va = nv_add;
      if (i < b1) {  // the next pair, loaded off the chain
        nv_rem = v[i + 1 - b0];
        nv_add = v[i + 1 + offset];
      }
      // rem (20 -> 19)
      double prev_mean = mean_x - comp_rem;
      double y = vr - comp_rem;
      double t = y - mean_x;
      comp_rem = t + mean_x - y;
      mean_x = mean_x - div_small(t, 19.0, r19);
      ssqdm = ssqdm - (vr - prev_mean) * (vr - mean_x);
      // add (19 -> 20)
      consec = (va == prev) ? consec + 1 : 1;
      prev = va;
      prev_mean = mean_x - comp_add;
      y = va - comp_add;
      t = y - mean_x;
      comp_add = t + mean_x - y;
      mean_x = mean_x + div_small(t, 20.0, r20);
      ssqdm = ssqdm + (va - prev_mean) * (va - mean_x);
      out[i] = (consec >= 20) ? 0.0 : div_small(ssqdm, 19.0, r19);
    }
    ps = i - b0;  // the window of output i - 1
    pe = i + offset;
  }
  for (; i < n; ++i) step(i);
}

// One condition's table: column c of dpd (D, C) -> column c of tables.
// status[c]: kOk, kFail (the reference raises: too few points, no finite
// weight, a non-finite scaled weight), kDegenerate (a non-finite local fit:
// the host redoes it).
__global__ __launch_bounds__(kThreads) void k_disp_table(
    const double* __restrict__ dpd, int D, int C, int weighted, double frac_in,
    double auto_frac_factor, double* __restrict__ tables, int* __restrict__ status,
    unsigned long long* __restrict__ stamps) {
  extern __shared__ double s_mem[];
  __shared__ Shared sh;
  __shared__ int s_F;
  __shared__ double s_med, s_med_lo, s_nanmean;
  const int c = blockIdx.x, tid = threadIdx.x;
  double* X = s_mem;  // finite points: distance, value
  double* Y = X + D;
  double* WT = Y + D;  // rolling variance, then the weight
  double* SW = WT + D;  // scaled weight
  double* RX = SW + D;  // runs: distance, value, local fit, robustness weight
  double* RY = RX + D;
  double* FIT = RY + D;
  double* RW = FIT + D;
  double* AB = RW + D;  // |residual| per run (scratch before that)
  double* CNTD = AB + D;  // copies per run as a double
  int64_t* RP = (int64_t*)(CNTD + D);  // run start points, D + 1
  int64_t* LEFT = RP + D + 1;          // window start of a fit at the run
  int* NXT = (int*)(LEFT + D);         // next fit run; later the bracketing fit
  int* FL = NXT + D;                   // fit runs in order
  int* CNT = FL + D;                   // copies per run
  int* WR0 = CNT + D;                  // the j-th fit's window: first and last run
  int* WR1 = WR0 + D;
  auto finish = [&](int st) {
    if (tid == 0) status[c] = st;
  };
  // H3D_TABLE_STAMPS: the phase boundaries (100 MHz wall clock) per condition
  auto stamp = [&](int k) {
    if (stamps && tid == 0) stamps[c * kStamps + k] = wall_clock64();
  };
  stamp(0);

  // ---- finite points (distance order) ----
  int64_t n0 = 0;
  for (int base = 0; base < D; base += kThreads) {
    const int d = base + tid;
    const double v = d < D ? dpd[(size_t)d * C + c] : NAN;
    const bool fin = d < D && isfinite(v);
    int64_t tot;
    const int64_t pos = n0 + scan_excl(fin ? 1 : 0, sh, &tot);
    if (fin) {
      X[pos] = (double)d;
      Y[pos] = v;
    }
    n0 += tot;
  }
  __syncthreads();
  if (n0 < 2) return finish(kFail);
  const double left_boundary = Y[0];  // (the reference's quirk, h3d_api.hip)

  int inc = 0;
  double frac = frac_in;
  int U = 0;
  if (weighted) {
    // ---- weights: rolling precision^(1/4), scaled to min 1 ----
    stamp(1);
    if (tid == 0) rolling_var(Y, n0, WT);
    __syncthreads();
    stamp(2);
    double lmin = INFINITY;
    for (int64_t i = tid; i < n0; i += kThreads) {
      const double prec = 1.0 / WT[i];
      const double w = isfinite(prec) ? pow(prec, 0.25) : NAN;
      WT[i] = w;
      if (w == w) lmin = fmin(lmin, w);
    }
    const double min_w = block_min(lmin, sh);
    if (!(min_w < INFINITY)) return finish(kFail);  // nanmin of all-NaN
    const double inv = 1.0 / min_w;
    double lmax = -INFINITY;
    for (int64_t i = tid; i < n0; i += kThreads) {
      double s = WT[i] * inv;
      // the pinned deviation (h3d_host.h); weighted == 2: the reference's
      // own w * (1 / w)
      if (WT[i] == min_w && weighted != 2) s = 1.0;
      SW[i] = s;
      if (s == s) lmax = fmax(lmax, s);
    }
    const double max_w = block_max(lmax, sh);
    int lfirst = (int)n0;
    for (int64_t i = tid; i < n0; i += kThreads) {
      double s = SW[i];
      if (isinf(s)) s = max_w;
      SW[i] = s;
      if (isfinite(s)) lfirst = min(lfirst, (int)i);
    }
    const int first_finite = block_min_int(lfirst, sh);
    const double left_w = SW[first_finite < n0 ? first_finite : 0];
    int bad = 0, linc = (int)n0;
    for (int64_t i = tid; i < n0; i += kThreads) {
      double s = SW[i];
      if (s != s) {
        if ((double)i < n0 / 2.0)
          s = left_w;
        else if ((double)i > n0 / 2.0)
          s = 1;
      }
      SW[i] = s;
      if (!isfinite(s)) bad = 1;
      if (i + 1 < n0 && Y[i + 1] - Y[i] > 0) linc = min(linc, (int)i);
    }
    if (block_or(bad, sh)) return finish(kFail);
    const int first_inc = block_min_int(linc, sh);
    inc = (first_inc < n0 ? first_inc : 0) + 1;
    if (!(frac >= 0)) {
      // nanmean of the (unscaled) weights, numpy's pairwise sum in order
      int64_t m = 0;
      for (int base = 0; base < n0; base += kThreads) {
        const int i = base + tid;
        const bool ok = i < n0 && WT[i] == WT[i];
        int64_t tot;
        const int64_t pos = m + scan_excl(ok ? 1 : 0, sh, &tot);
        if (ok) AB[pos] = WT[i];
        m += tot;
      }
      __syncthreads();
      if (tid == 0) s_nanmean = pairwise<4>(AB, m) / (double)m;
      __syncthreads();
      const double frac_auto = auto_frac_factor / (max_w * s_nanmean);
      frac = fmax(fmin(frac_auto, 2. / 3), 0.05);
    }
    stamp(3);
    // ---- runs: distance i >= inc replicated floor(sw_i) times ----
    int64_t u0 = 0;
    int big = 0;  // a weight beyond 2^30 copies: left to the host
    for (int base = inc; base < n0; base += kThreads) {
      const int i = base + tid;
      const int64_t cnt = i < n0 ? (int64_t)floor(SW[i]) : 0;
      int64_t tot;
      const int64_t pos = u0 + scan_excl(cnt >= 1 ? 1 : 0, sh, &tot);
      if (cnt >= 1) {
        RX[pos] = X[i];
        RY[pos] = Y[i];
        CNT[pos] = cnt > (1 << 30) ? (1 << 30) : (int)cnt;
        if (cnt > (1 << 30)) big = 1;
      }
      u0 += tot;
    }
    if (block_or(big, sh)) return finish(kDegenerate);
    U = (int)u0;
  } else {
    if (!(frac >= 0)) frac = 0.3;
    for (int64_t i = tid; i < n0; i += kThreads) {
      RX[i] = X[i];
      RY[i] = Y[i];
      CNT[i] = 1;
    }
    U = (int)n0;
  }
  __syncthreads();
  // run starts (point index of each run's first copy)
  int64_t n = 0;
  for (int base = 0; base < U; base += kThreads) {
    const int u = base + tid;
    const int64_t cnt = u < U ? CNT[u] : 0;
    int64_t tot;
    const int64_t pos = n + scan_excl(cnt, sh, &tot);
    if (u < U) {
      RP[u] = pos;
      CNTD[u] = (double)cnt;
    }
    n += tot;
  }
  if (tid == 0) RP[U] = n;
  __syncthreads();
  if (n < 2 || U < 2) return finish(kFail);
  if (n >= ((int64_t)1 << 31)) return finish(kDegenerate);  // (int counts below)
  int64_t k = (int64_t)(frac * n + 1e-10);
  k = min(max(k, (int64_t)2), n);
  const double delta = (RX[U - 1] - RX[0]) * 0.01;

  stamp(4);
  // ---- per run: the window of a fit there, the next fit run ----
  for (int u = tid; u < U; u += kThreads) {
    const double xval = RX[u];
    int64_t lo = 0, hi = n - k;  // first l with !(xval > midpoint(l)), else n - k
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      const double xl = RX[run_of(RP, U, mid)], xr = RX[run_of(RP, U, mid + k)];
      if (xval > (xl + xr) / 2.0)
        lo = mid + 1;
      else
        hi = mid;
    }
    LEFT[u] = lo;
    const double cut = xval + delta;
    int a = u + 1, b = U;  // first run after u beyond cut
    while (a < b) {
      const int mid = (a + b) >> 1;
      if (RX[mid] > cut) b = mid;
      else a = mid + 1;
    }
    int nxt;
    if (a < U)
      nxt = (a - 1 > u) ? a - 1 : u + 1;
    else if (u == U - 1)
      nxt = -1;
    else
      nxt = run_of(RP, U, max(n - 2, RP[u + 1]));
    NXT[u] = nxt;
  }
  __syncthreads();
  stamp(5);
  // the fit runs: the chain 0 -> NXT[0] -> ... -> U - 1, marked by pointer
  // doubling (round r marks the runs 2^r .. 2^(r+1) - 1 steps down the
  // chain), then compacted in order; the bracketing fit of a run is the
  // count of fit runs up to it, less one
  {
    int* ON = (int*)AB;  // (AB is free until the robustness passes)
    int* Ja = WR0;
    int* Jb = WR1;
    for (int u = tid; u < U; u += kThreads) {
      Ja[u] = NXT[u] >= 0 ? NXT[u] : U;
      ON[u] = u == 0;
    }
    __syncthreads();
    for (int span = 1; span < U; span <<= 1) {
      for (int u = tid; u < U; u += kThreads) {
        const int j = Ja[u];
        if (ON[u] && j < U) ON[j] = 1;  // (a race only marks chain runs early)
        Jb[u] = j < U ? Ja[j] : U;
      }
      __syncthreads();
      int* t = Ja;
      Ja = Jb;
      Jb = t;
    }
    int64_t f = 0;
    for (int base = 0; base < U; base += kThreads) {
      const int u = base + tid;
      const int on = u < U ? ON[u] : 0;
      int64_t tot;
      const int64_t pos = f + scan_excl(on, sh, &tot);
      if (on) FL[pos] = u;
      if (u < U) NXT[u] = (int)(pos + on - 1);
      f += tot;
    }
    if (tid == 0) s_F = (int)f;
    __syncthreads();
  }
  const int F = s_F;
  for (int u = tid; u < U; u += kThreads) RW[u] = 1.0;
  for (int j = tid; j < F; j += kThreads) {
    const int u = FL[j];
    WR0[j] = run_of(RP, U, LEFT[u]);
    WR1[j] = run_of(RP, U, LEFT[u] + k - 1);
  }
  __syncthreads();

  stamp(6);
  // ---- robustness iterations ----
  for (int rob = 0; rob <= kRobustIters; ++rob) {
    // fit j on lane j / 4 of wave j % 4: a few dozen fits keep every SIMD busy
    const int lane = tid & 63, wid = tid >> 6;
    for (int j = lane * kWaves + wid; j < F; j += kThreads) {
      const int u = FL[j];
      const double xval = RX[u];
      const int64_t left = LEFT[u], right = left + k;
      const int r0 = WR0[j], r1 = WR1[j];
      const double radius = fmax(xval - RX[r0], RX[r1] - xval);
      const double inv_radius = 1.0 / radius;
      double S0 = 0.0, S1 = 0.0, S2 = 0.0, T0 = 0.0, T1 = 0.0;
      // the host's sequential sums over the window's runs, in run order; the
      // window cuts only its first and last run, the rest count whole
      auto term = [&](double x, double y, double rw, double cc) {
        const double d = x - xval;
        double t = fabs(d) * inv_radius;
        double uu = 1 - t * (t * t);
        uu = uu > 0.0 ? uu : 0.0;
        double wt = uu * (uu * uu);
        wt = wt * rw;  // 1.0 before the first robustness pass: exact
        const double cw = cc * wt, cwd = cw * d;
        S0 += cw;
        S1 += cwd;
        S2 += cwd * d;
        T0 += cw * y;
        T1 += cwd * y;
      };
      auto cut = [&](int r) {
        return (double)(min(RP[r + 1], right) - max(RP[r], left));
      };
      term(RX[r0], RY[r0], RW[r0], cut(r0));
      int r = r0 + 1;
      for (; r + 4 <= r1; r += 4) {  // loads of four runs, then their terms
        double x4[4], y4[4], w4[4], c4[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          x4[q] = RX[r + q];
          y4[q] = RY[r + q];
          w4[q] = RW[r + q];
          c4[q] = CNTD[r + q];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) term(x4[q], y4[q], w4[q], c4[q]);
      }
      for (; r < r1; ++r) term(RX[r], RY[r], RW[r], CNTD[r]);
      if (r1 > r0) term(RX[r1], RY[r1], RW[r1], cut(r1));
      double fit;
      if (S0 <= 0.0) {
        fit = RY[u];
      } else {
        const double inv = 1.0 / S0;
        const double m = S1 * inv, t0 = T0 * inv;
        const double var = S2 * inv - m * m;
        fit = t0 - m * (T1 * inv - m * t0) / var;
      }
      FIT[u] = fit;
    }
    __syncthreads();
    stamp(7 + 2 * rob);
    for (int u = tid; u < U; u += kThreads) {
      const int j = NXT[u];
      if (FL[j] != u) {  // between fit runs FL[j] and FL[j + 1]
        const int ua = FL[j], ub = FL[j + 1];
        const double den = RX[ub] - RX[ua];
        const double a = (RX[u] - RX[ua]) / den;
        FIT[u] = a * FIT[ub] + (1.0 - a) * FIT[ua];
      }
    }
    __syncthreads();
    int bad = 0;
    for (int u = tid; u < U; u += kThreads)
      if (!isfinite(FIT[u])) bad = 1;
    if (block_or(bad, sh)) return finish(kDegenerate);
    stamp(8 + 2 * rob);
    if (rob == kRobustIters) break;
    // median of |y - fit| over the n points: count-weighted order statistics
    for (int u = tid; u < U; u += kThreads) AB[u] = fabs(RY[u] - FIT[u]);
    __syncthreads();
    const int64_t p_hi = n / 2, p_lo = n / 2 - 1;
    for (int u = tid; u < U; u += kThreads) {
      const double v = AB[u];
      // counts below and equal to v (both loads unconditional: a select on
      // the loaded count, not a guarded load -- that serialised the loop)
      int less = 0, eq = 0;  // (n < 2^31)
      int w = 0;
      for (; w + 4 <= U; w += 4) {
        double z[4];
        int cw[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          z[q] = AB[w + q];
          cw[q] = CNT[w + q];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          less += cw[q] & -(int)(z[q] < v);
          eq += cw[q] & -(int)(z[q] == v);
        }
      }
      for (; w < U; ++w) {
        const double z = AB[w];
        const int cw = CNT[w];
        less += cw & -(int)(z < v);
        eq += cw & -(int)(z == v);
      }
      // (every run holding the position writes the same value)
      if (less <= p_hi && p_hi < less + eq) s_med = v;
      if (less <= p_lo && p_lo < less + eq) s_med_lo = v;
    }
    __syncthreads();
    double med = s_med;
    if (n % 2 == 0) med = 0.5 * (s_med_lo + med);
    const double s6 = 6.0 * med;
    for (int u = tid; u < U; u += kThreads) {
      const double rj = RY[u] - FIT[u];
      double w;
      if (s6 > 0) {
        double t = fabs(rj / s6);
        w = (t < 1.0) ? (1 - t * t) * (1 - t * t) : 0.0;
      } else {
        w = (rj == 0) ? 1.0 : 0.0;
      }
      RW[u] = w;
    }
    __syncthreads();
  }

  // ---- the table at every distance ----
  for (int d = tid; d < D; d += kThreads) {
    const double xs = (double)d;
    double v = interp_extrap(RX, FIT, U, xs);
    if (xs <= left_boundary) v = FIT[0];
    if (weighted && xs < X[inc]) {
      v = interp_extrap(X, Y, (int)n0, xs);
      if (xs < X[0]) v = Y[0];
    }
    tables[(size_t)d * C + c] = v;
  }
  stamp(15);
  finish(kOk);
}

}  // namespace h3dtab

extern "C" {

int h3d_disp_tables_dev(h3d_ctx* ctx, const double* d_disp_per_dist, int D, int C,
                        int weighted, double frac, double auto_frac_factor,
                        double* d_tables_out) {
  using namespace h3dtab;
  if (!ctx || !d_disp_per_dist || !d_tables_out || D < 1 || C < 1 || C > kMaxConds)
    return fail(H3D_EARG, "null argument / D / C");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  int* d_status = (int*)scratch(ctx, "table_status", (size_t)kMaxConds * 4);
  if (!d_status) return fail(H3D_ENOMEM, "table status");
  ctx->tab_pending = {d_disp_per_dist, d_tables_out, D, C, weighted, frac,
                      auto_frac_factor, 1};
  if (D > kMaxD) {  // beyond the LDS working set: the host smoother
    ctx->tab_pending.on_host = 1;
    std::vector<double> dpd((size_t)D * C), tab((size_t)D * C);
    HIP_TRY(hipMemcpyAsync(dpd.data(), d_disp_per_dist, dpd.size() * 8,
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (int rc = h3d_disp_tables(dpd.data(), D, C, weighted, frac, auto_frac_factor,
                                 tab.data()))
      return rc;
    HIP_TRY(hipMemcpyAsync(d_tables_out, tab.data(), tab.size() * 8,
                           hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    return 0;
  }
  ctx->tab_pending.on_host = 0;
  int& attr = ctx->resident[(const void*)k_disp_table];
  if (!attr) {
    HIP_TRY(hipFuncSetAttribute((const void*)k_disp_table,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds_bytes(kMaxD)));
    attr = 1;
  }
  {
    ProfScope ps(ctx, "disp_table", D);
    unsigned long long* d_stamps = nullptr;
    if (getenv("H3D_TABLE_STAMPS")) {
      d_stamps = (unsigned long long*)scratch(ctx, "table_stamps", kMaxConds * kStamps * 8);
      if (d_stamps) HIP_TRY(hipMemsetAsync(d_stamps, 0, kMaxConds * kStamps * 8, s));
    }
    hipLaunchKernelGGL(k_disp_table, dim3(C), dim3(kThreads), lds_bytes(D), s,
                       d_disp_per_dist, D, C, weighted, frac, auto_frac_factor,
                       d_tables_out, d_status, d_stamps);
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

}  // extern "C"

namespace h3dint {

// the pending device table's per-condition status into h_st (stream-ordered,
// no wait); 0 when there is nothing to check
int table_status_copy(h3d_ctx* ctx, int* h_st) {
  const TablePending& tp = ctx->tab_pending;
  if (!tp.active || tp.on_host) return 0;
  const int* d_status = (const int*)scratch(ctx, "table_status", (size_t)kMaxConds * 4);
  HIP_TRY(hipMemcpyAsync(h_st, d_status, tp.C * 4, hipMemcpyDeviceToHost, ctx->stream));
  return 1;
}

// after the stream has drained: settles the pending device table from the
// copied status. A degenerate fit is redone by the host smoother into the same
// device buffer (returns 1: results computed from the table must be redone);
// a failure is the host smoother's error (the reference's)
int table_settle(h3d_ctx* ctx, const int* h_st) {
  using namespace h3dtab;
  TablePending& tp = ctx->tab_pending;
  if (!tp.active) return 0;
  tp.active = 0;
  if (tp.on_host) return 0;
  int worst = kOk;
  for (int c = 0; c < tp.C; ++c) worst = h_st[c] > worst ? h_st[c] : worst;
  if (worst == kOk) return 0;
  hipStream_t s = ctx->stream;
  std::vector<double> dpd((size_t)tp.D * tp.C), tab((size_t)tp.D * tp.C);
  HIP_TRY(hipMemcpyAsync(dpd.data(), tp.dpd, dpd.size() * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (int rc = h3d_disp_tables(dpd.data(), tp.D, tp.C, tp.weighted, tp.frac, tp.aff,
                               tab.data()))
    return rc;
  if (worst == kFail)
    return fail(H3D_ENOCONV, "device lowess failed where the host one did not");
  HIP_TRY(hipMemcpyAsync(tp.tables, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  return 1;
}

}  // namespace h3dint

extern "C" int h3d_disp_tables_wait(h3d_ctx* ctx) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  HIP_TRY(hipSetDevice(ctx->device));
  int st[kMaxConds];
  int* land = (int*)h3dint::pinned_rd(ctx, sizeof(st));  // pinned: see h2d_pinned
  if (!land) return fail(H3D_ENOMEM, "pinned landing zone");
  if (int rc = h3dint::table_status_copy(ctx, land); rc < 0) return rc;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  std::memcpy(st, land, sizeof(st));
  if (getenv("H3D_TABLE_STAMPS")) {  // per condition: us since the start
    using h3dtab::kStamps;
    unsigned long long h[kMaxConds * kStamps];
    const void* d = h3dint::scratch(ctx, "table_stamps", kMaxConds * kStamps * 8);
    HIP_TRY(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    for (int c = 0; c < ctx->tab_pending.C; ++c) {
      fprintf(stderr, "[h3d table] cond %d:", c);
      for (int k = 1; k < kStamps; ++k)
        if (h[c * kStamps + k])
          fprintf(stderr, " %d:%.1f", k, (h[c * kStamps + k] - h[c * kStamps]) / 100.0);
      fprintf(stderr, "\n");
    }
  }
  const int rc = h3dint::table_settle(ctx, st);
  return rc < 0 ? rc : 0;
}
