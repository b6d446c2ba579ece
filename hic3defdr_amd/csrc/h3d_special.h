// FP64 special functions for the hic3defdr hot path, host + device.
//
// The reference calls these through scipy.special (scipy 1.7.1 = cephes):
//   gammaln            -> scaled_nb.py:32, dispersion.py:68-70 (lgam)
//   norm cdf/sf/ppf/isf -> scaled_nb.py:256-265 (ndtr, ndtri)
//   gamma cdf/sf/ppf/isf-> scaled_nb.py:258-267 (igam, igamc, igami, igamci)
//   chi2.sf            -> lrt.py:49 (chdtrc = igamc(df/2, x/2))
// Restated from the published cephes / DiDonato & Morris (1986) algorithms.
// Deviations, all accuracy-preserving:
//   * the prefactor x^a e^-x / Gamma(a) near a ~ x (a >= 10) is computed from
//     log1pmx + the Stirling series instead of a Lanczos sum;
//   * the Temme uniform asymptotic branch of igam/igamc is not used (the power
//     series / continued fraction converge there too, O(sqrt(a)) terms);
//   * ndtri is an Acklam initial guess refined by Halley steps on erfc.
// Everything is plain C++ so the same code builds for gfx950 (hipcc) and for
// the host-side unit tests (g++), see tests/test_special_host.py.
#pragma once

#include <cmath>
#include <cstdint>

// FMA contraction off for everything built on these headers: it keeps the
// device arithmetic op-for-op with the host test build (g++
// -ffp-contract=off), and measured on gfx950 (r01) contracting the
// q2qnbinom / incomplete-gamma code raised the equalize kernel's register
// demand (W=4 budget: 128 -> 384 B of spills) and cost 8% (11.7 -> 12.6 ms
// per bench step).
#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#if defined(__HIPCC__)
#define H3D_HD __host__ __device__ inline
// a rarely taken path kept out of line, so its temporaries do not raise the
// register demand of the kernels that inline everything else
#define H3D_HD_COLD __host__ __device__ inline __attribute__((noinline))
// forced inline: a path whose out-of-line form measured slower (the call's
// presence changed the whole kernel's register allocation)
#define H3D_HD_INLINE __host__ __device__ inline __attribute__((always_inline))
#else
#define H3D_HD inline
#define H3D_HD_COLD inline
#define H3D_HD_INLINE inline
#endif

// Work counters for tools/q2q_stats (host builds with H3D_INSTRUMENT only;
// compiled out everywhere else).
#if defined(H3D_INSTRUMENT) && !defined(__HIP_DEVICE_COMPILE__)
namespace h3d {
struct Stats {
  long pq, cf, su, ser, cf_it, su_it, ser_it, fac_l1, l1_it, inv, halley, wh,
      lgam, lgam_small, lgam_it, fit, fit_it;
};
inline thread_local Stats* g_stats = nullptr;
inline thread_local double* g_pq_log = nullptr;  // (a, x, iterations, path)
inline thread_local int64_t g_pq_cap = 0, g_pq_n = 0;
inline void pq_log(double a, double x, long it, int path) {
  if (g_pq_log && g_pq_n < g_pq_cap) {
    double* o = g_pq_log + 4 * g_pq_n++;
    o[0] = a, o[1] = x, o[2] = (double)it, o[3] = path;
  }
}
}  // namespace h3d
#define H3D_PQ_LOG(a, x, it, path) h3d::pq_log(a, x, it, path)
#define H3D_STAT(field, v) \
  do {                     \
    if (h3d::g_stats) h3d::g_stats->field += (v); \
  } while (0)
#else
#define H3D_STAT(field, v) ((void)0)
#define H3D_PQ_LOG(a, x, it, path) ((void)0)
#endif

// Section timing of the equalize pass (a profiling build only: -DH3D_SECPROF,
// tools/secprof.py): H3D_SEC_BEGIN / H3D_SEC_END(k) add the wave's shader
// clock ticks spent in section k to g_h3d_secprof[k] (one lane of the wave
// adds; sections of a wave do not overlap). Compiled out everywhere else.
#if defined(H3D_SECPROF) && defined(__HIPCC__)
__device__ unsigned long long g_h3d_secprof[32];
#endif
#if defined(H3D_SECPROF) && defined(__HIP_DEVICE_COMPILE__)
// (sched_barrier: the machine scheduler moves nothing across a timestamp)
#define H3D_SEC_BEGIN(t)                                                      \
  __builtin_amdgcn_sched_barrier(0);                                          \
  const unsigned long long t = __builtin_readcyclecounter();                  \
  __builtin_amdgcn_sched_barrier(0)
#define H3D_SEC_END(k, t)                                                     \
  do {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                        \
    const unsigned long long t_end_ = __builtin_readcyclecounter();           \
    __builtin_amdgcn_sched_barrier(0);                                        \
    if ((int)__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1)     \
      atomicAdd(&g_h3d_secprof[(k)], t_end_ - (t));                           \
  } while (0)
#else
#define H3D_SEC_BEGIN(t) ((void)0)
#define H3D_SEC_END(k, t) ((void)0)
#endif

namespace h3d {

constexpr double kMachEp = 1.11022302462515654042e-16;  // 2^-53
constexpr double kMaxLog = 7.09782712893383996843e2;
constexpr double kBig = 4.503599627370496e15;
constexpr double kBigInv = 2.22044604925031308085e-16;
constexpr double kEuler = 0.577215664901532860606512090082402431;
constexpr double kLogSqrt2Pi = 0.91893853320467274178;
constexpr double kSqrt1_2 = 0.70710678118654752440;
constexpr double kSqrt2Pi = 2.50662827463100050242;
constexpr double kTwoPi = 6.28318530717958647692;
constexpr int kMaxIter = 2000;

H3D_HD bool is_inf(double v) { return fabs(v) == INFINITY; }

H3D_HD double polevl(double x, const double* c, int n) {
  double ans = c[0];
  for (int i = 1; i <= n; ++i) ans = ans * x + c[i];
  return ans;
}

H3D_HD double p1evl(double x, const double* c, int n) {
  double ans = x + c[0];
  for (int i = 1; i < n; ++i) ans = ans * x + c[i];
  return ans;
}

// log Gamma(x) for x > 0 (cephes lgam; reference gammaln).
H3D_HD double lgam(double x) {
  const double A[] = {8.11614167470508450300E-4, -5.95061904284301438324E-4,
                      7.93650340457716943945E-4, -2.77777777730099687205E-3,
                      8.33333333333331927722E-2};
  const double B[] = {-1.37825152569120859100E3, -3.88016315134637840924E4,
                      -3.31612992738871184744E5, -1.16237097492762307383E6,
                      -1.72173700820839662146E6, -8.53555664245765465627E5};
  const double C[] = {-3.51815701436523470549E2, -1.70642106651881159223E4,
                      -2.20528590553854454839E5, -1.13933444367982507207E6,
                      -2.53252307177582951285E6, -2.01889141433532773231E6};
  H3D_STAT(lgam, 1);
  if (!(x > 0.0)) return (x == 0.0) ? INFINITY : NAN;
  if (x < 13.0) {
    H3D_STAT(lgam_small, 1);
    double z = 1.0, p = 0.0, u = x;
    while (u >= 3.0) {
      H3D_STAT(lgam_it, 1);
      p -= 1.0;
      u = x + p;
      z *= u;
    }
    while (u < 2.0) {
      H3D_STAT(lgam_it, 1);
      z /= u;
      p += 1.0;
      u = x + p;
    }
    if (u == 2.0) return log(z);
    p -= 2.0;
    x = x + p;
    p = x * polevl(x, B, 5) / p1evl(x, C, 6);
    return log(z) + p;
  }
  if (x > 2.556348e305) return INFINITY;
  double q = (x - 0.5) * log(x) - x + kLogSqrt2Pi;
  if (x > 1.0e8) return q;
  double p = 1.0 / (x * x);
  if (x >= 1000.0)
    q += ((7.9365079365079365079365e-4 * p - 2.7777777777777777777778e-3) * p +
          0.0833333333333333333333) /
         x;
  else
    q += polevl(p, A, 4) / x;
  return q;
}

// 1/y for the NLL lgamma (absolute accuracy): on gfx950 v_rcp_f64 + one
// Newton step (~1 ulp) instead of the IEEE division sequence; the host
// build divides.
H3D_HD double recip_nll(double y) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double r0 = __builtin_amdgcn_rcp(y);
  return fma(fma(-y, r0, 1.0), r0, r0);
#else
  return 1.0 / y;
#endif
}

// 1/y wherever ~1 ulp is enough (Newton iterates of the mean MLE, series
// terms): recip_nll on gfx950, the division on the host.
H3D_HD double recip_fast(double y) { return recip_nll(y); }
// a / b to ~1 ulp by recip_fast (the equalize pass's quantile-map and
// Halley-step quotients, whose rounding is far below their tests' bars)
H3D_HD double div_fast(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return a * recip_nll(b);
#else
  return a / b;
#endif
}

// Horner step p x + c of the NLL polynomials. On gfx950 an explicit
// three-address v_fma_f64 with the constant addend in an SGPR pair: with the
// constant as the tied accumulator the compiler emitted v_fmac_f64 plus a
// v_mov_b64 copy of the constant per step (84 of the 410 VALU instructions of
// k_brent's loop). Measured (tools/ab_lib.sh, cfg2): k_brent 3.57 -> 3.07 ms
// per step; with a VGPR constraint on c the compiler copied the constants
// from SGPRs instead (3.29 ms). The result is the same fused value the
// contracted `p * x + c` gave. Operands here never come straight from a
// transcendental instruction (s^2, r^2, a Horner value), so the asm needs no
// forwarding wait state. Host: `p * x + c` as before.
#ifndef H3D_EXP11
#define H3D_EXP11 1
#endif
#ifndef H3D_HFMA_ASM
#define H3D_HFMA_ASM 1
#endif
H3D_HD double hfma(double p, double x, double c) {
#if defined(__HIP_DEVICE_COMPILE__) && H3D_HFMA_ASM
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(p), "v"(x), "s"(c));
  return r;
#else
  return p * x + c;
#endif
}

// ln(m) for the NLL log: kLogTabLen = 513 buckets m_i = 1/2 + i/1024 over
// frexp's mantissa range [1/2, 1], c_i = 1/m_i rounded, l_i = ln(1/c_i) --
// plus ln 2 for the buckets below sqrt(1/2) (i <= kLogTabShifted = 212),
// whose exponent is taken one lower, so ln x never cancels e ln 2 against
// ln m near x = 1 (x = 2^k lands on c_0 = 2 exactly and returns (k - 1) ln 2
// + 0). Entries: l_i correctly rounded from 80-bit ln; generated into
// h3d_logtab.h by tools/log_table.py. 8 KB: k_brent / k_lrt keep a copy in
// LDS.
struct LogTab {
  double c, l;
};
#include "h3d_logtab.h"

// Natural log for finite x > 0, straight-line and table-driven:
//   x = m 2^e, i = round(1024 (m - 1/2)), t = m c_i - 1 (one fma, |t| <=
//   2^-10), ln x = e' ln 2 + l_i + log1p(t), log1p by its degree-5 Taylor
//   polynomial (truncation t^6 / 6 < 2^-62).
// Max error 1.9e-16 absolute, 2.3e-16 relative (80-bit reference over
// [1e-300, 1e300] (absolute 5.7e-14 there: |ln x| <= 690), [0.3, 3] and
// [1, 1e4]). The 1024-step table (round 4; 256 steps and degree 7 before)
// takes two fma off every log. Used by the NLL sums (finite x > 0 by
// construction) and, through log_fast_checked, the incomplete-gamma
// prefactor.
// (tab: the table's copy to read -- kLogTab, or a kernel's copy in LDS)
H3D_HD double log_fast(double x, const LogTab* tab = kLogTab) {
  int e;
  const double m = frexp(x, &e);  // [0.5, 1)
  const int i = (int)((m - 0.5) * (double)kLogTabSteps + 0.5);  // 0..512
  const LogTab tb = tab[i];
  const double t = fma(m, tb.c, -1.0);
  double q = 1.0 / 5.0;
  q = hfma(q, t, -1.0 / 4.0);
  q = hfma(q, t, 1.0 / 3.0);
  q = hfma(q, t, -1.0 / 2.0);
  const double lp = fma(q, t * t, t);
  const double de = (double)(e - (i <= kLogTabShifted ? 1 : 0));
  return de * 6.93147180369123816490e-01 + (de * 1.90821492927058770002e-10 + (tb.l + lp));
}

// log_fast for any x: frexp of 0 / inf would index outside the table, so x
// is first replaced by 1 there and libm's values (-inf, inf, NaN) are
// selected afterwards (the k_brent NLL keeps the unchecked form: the checks
// cost it 8 %, r03 PMC)
H3D_HD double log_fast_checked(double x, const LogTab* tab = kLogTab) {
  const bool ok = x > 0.0 && x < INFINITY;
  const double v = log_fast(ok ? x : 1.0, tab);
  if (ok) return v;
  return (x == INFINITY) ? INFINITY : (x == 0.0) ? -INFINITY : NAN;
}

// Stirling series of the NLL lgamma in r2 = 1/y^2 (8 Bernoulli terms),
// Horner from the innermost term: the same fused steps as the nested form
H3D_HD double stirling_nll(double r2) {
  double q = -3617.0 / 122400.0;
  q = hfma(q, r2, 1.0 / 156.0);
  q = hfma(q, r2, -691.0 / 360360.0);
  q = hfma(q, r2, 1.0 / 1188.0);
  q = hfma(q, r2, -1.0 / 1680.0);
  q = hfma(q, r2, 1.0 / 1260.0);
  q = hfma(q, r2, -1.0 / 360.0);
  return hfma(q, r2, 1.0 / 12.0);
}

// e^x on gfx950, straight-line: x = k ln2 + r (|r| <= ln2 / 2, Cody-Waite
// with fdlibm's split ln2), e^r by its degree-13 Taylor polynomial
// (truncation < 5e-18 relative) in hfma steps with the coefficients in
// SGPRs, scaled by ldexp; overflow / underflow / NaN as libm. ~1 ulp. OCML's
// exp carried a v_mov_b64 copy of its constant per Horner step. Host: exp.
H3D_HD double exp_fast(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double kd = rint(x * 1.44269504088896338700e+00);
  double r = fma(kd, -6.93147180369123816490e-01, x);
  r = fma(kd, -1.90821492927058770002e-10, r);
#if H3D_EXP11
  // degree-11 near-minimax (Chebyshev fit, mpmath: 3.2e-18 on |r| <=
  // ln2 / 2; <= 1.01 ulp with the fused Horner steps against 0.98 for the
  // Taylor form below), two steps and two SGPR constants fewer
  double p = 2.5110037605963777e-08;
  p = hfma(p, r, 2.763263963904103e-07);
  p = hfma(p, r, 2.755724091857897e-06);
  p = hfma(p, r, 2.4801485482328494e-05);
  p = hfma(p, r, 0.00019841269890047113);
  p = hfma(p, r, 0.0013888888952314775);
  p = hfma(p, r, 0.008333333333319601);
  p = hfma(p, r, 0.0416666666664881);
  p = hfma(p, r, 0.1666666666666668);
  p = hfma(p, r, 0.5000000000000019);
  p = hfma(p, r, 1.0);
  p = hfma(p, r, 1.0);
#else
  double p = 1.0 / 6227020800.0;              // 1/13!
  p = hfma(p, r, 1.0 / 479001600.0);
  p = hfma(p, r, 1.0 / 39916800.0);
  p = hfma(p, r, 1.0 / 3628800.0);
  p = hfma(p, r, 1.0 / 362880.0);
  p = hfma(p, r, 1.0 / 40320.0);
  p = hfma(p, r, 1.0 / 5040.0);
  p = hfma(p, r, 1.0 / 720.0);
  p = hfma(p, r, 1.0 / 120.0);
  p = hfma(p, r, 1.0 / 24.0);
  p = hfma(p, r, 1.0 / 6.0);
  p = hfma(p, r, 0.5);
  p = hfma(p, r, 1.0);
  p = hfma(p, r, 1.0);
#endif
  const int k = (int)fmax(fmin(kd, 1100.0), -1100.0);
  double v = ldexp(p, k);
  v = (x > 7.09782712893383996843e2) ? INFINITY : v;
  v = (x < -7.45133219101941108420e2) ? 0.0 : v;
  return (x != x) ? x : v;
#else
  return exp(x);
#endif
}

// degree-5 rising factorial x (x+1) (x+2) (x+3) (x+4)
H3D_HD double rise5(double x) {
  return hfma(hfma(hfma(x + 10.0, x, 35.0), x, 50.0), x, 24.0) * x;
}

// log Gamma(x), x > 0 finite, for the NLL sums (dispersion.py:67-70), where
// only the ABSOLUTE error matters (each term joins a sum of thousands of
// O(10..1e4) terms). Branch-light: shift x up to y >= 10 through the
// product P = x (x+1) ... (y-1) (at most 10 multiplies), then Stirling's
// series with 8 Bernoulli terms (truncation < 2e-18 at y = 10):
//   lgam(x) = (y - 1/2) ln y - y + ln sqrt(2 pi) + sum_n B2n/(2n(2n-1)y^(2n-1))
//             - ln P.
// Absolute error <= ~5e-15 for x < 10 (cancellation between lgam(y) and
// ln P), relative ~1e-15 above. cephes lgam (scipy gammaln) instead runs a
// data-dependent recurrence with a division per step below 13, which
// serialises across a wave.
//
// The shift below 10 is a fixed 5 or 10 steps (no data-dependent loop, which
// serialised the lanes of a wave): P is built from the degree-5 rising
// factorial x (x+1) (x+2) (x+3) (x+4) = ((((x + 10) x + 35) x + 50) x + 24) x
// (positive coefficients: no cancellation for x > 0), y lands in [10, 15).
// FMA contraction is on here: only the absolute error matters (see above).
H3D_HD double lgam_nll(double x, const LogTab* tab = kLogTab) {
#if defined(__clang__)
#pragma clang fp contract(fast)
#endif
  if (!(x > 0.0)) return (x == 0.0) ? INFINITY : NAN;  // as cephes
  if (is_inf(x)) return x;
  double y = x, P = 1.0;
  if (x < 10.0) {
    const bool two = x < 5.0;
    const double u = two ? x + 5.0 : x;
    const double pu = rise5(u);
    const double px = rise5(x);
    P = two ? px * pu : pu;
    y = u + 5.0;
  }
  const double r = recip_nll(y), r2 = r * r;
  const double corr = r * stirling_nll(r2);
  double v = (y - 0.5) * log_fast(y, tab) - y + kLogSqrt2Pi + corr;
  if (x < 10.0) v -= log_fast(P, tab);
  return v;
}

// Stirling series of the NLL lgamma with the first 5 Bernoulli terms, for y
// >= 20: the first omitted term, B12 / (12 11 y^11), is < 1e-17 there (the
// 8-term series of stirling_nll is needed down to y = 10)
H3D_HD double stirling_nll5(double r2) {
  double q = 1.0 / 1188.0;
  q = hfma(q, r2, -1.0 / 1680.0);
  q = hfma(q, r2, 1.0 / 1260.0);
  q = hfma(q, r2, -1.0 / 360.0);
  return hfma(q, r2, 1.0 / 12.0);
}

// lgam_nll_parts for x >= 20 (the caller knows it for every lane: the NLL
// arguments d + r with r >= 20, pseudodata d >= 0): no shift product (*P is
// 1), the 5-term Stirling series. Same accuracy as lgam_nll_parts there.
H3D_HD double lgam_nll_large(double x, const LogTab* tab = kLogTab) {
#if defined(__clang__)
#pragma clang fp contract(fast)
#endif
  const double r = recip_nll(x), r2 = r * r;
  const double corr = r * stirling_nll5(r2);
  return (x - 0.5) * log_fast(x, tab) - x + kLogSqrt2Pi + corr;
}

// lgam_nll_parts for x >= 10 (the caller knows it for every lane: the NLL
// arguments d + r with r >= 10): no shift product, the 8-term series -- the
// same terms lgam_nll_parts evaluates there, without the product's bookkeeping
H3D_HD double lgam_nll_mid(double x, const LogTab* tab = kLogTab) {
#if defined(__clang__)
#pragma clang fp contract(fast)
#endif
  const double r = recip_nll(x), r2 = r * r;
  const double corr = r * stirling_nll(r2);
  return (x - 0.5) * log_fast(x, tab) - x + kLogSqrt2Pi + corr;
}

// lgam_nll split for batching: returns lgam(x) + ln P and sets *P, the
// shift product (1 for x >= 10), so a caller summing several lgammas takes
// ONE log of the combined product (nll_pixel: per pixel R_c + 1 lgammas, one
// ln P instead of up to R_c + 1).
H3D_HD double lgam_nll_parts(double x, double* P, const LogTab* tab = kLogTab) {
#if defined(__clang__)
#pragma clang fp contract(fast)
#endif
  double y = x, p = 1.0;
  if (x < 10.0) {
    const bool two = x < 5.0;
    const double u = two ? x + 5.0 : x;
    const double pu = rise5(u);
    const double px = rise5(x);
    p = two ? px * pu : pu;
    y = u + 5.0;
  }
  *P = p;
  const double r = recip_nll(y), r2 = r * r;
  const double corr = r * stirling_nll(r2);
  return (y - 0.5) * log_fast(y, tab) - y + kLogSqrt2Pi + corr;
}

// log(1 + x) - x (cephes log1pmx). For |x| < 0.5 cephes sums the Taylor
// series until it converges (up to ~50 terms, a data-dependent loop that
// diverges across a wave); here it is the fixed-length atanh form
//   log1p(x) - x = -x^2 / (2 + x) + 2 u^3 sum_k u^2k / (2k + 3),
//   u = x / (2 + x), |u| <= 1/3,
// whose 16 terms reach the same ~1 ulp accuracy (the sum is <= 1/12 of the
// leading term and its truncation error < 9^-16).
// The |x| < 0.5 form alone (no libm fallback: the igam prefactor's only call
// has |x| <= 0.4, and the inlined OCML log1p of the other branch, never
// taken there, carried spill code into the equalize kernel).
H3D_HD double log1pmx_small(double x) {
  H3D_STAT(l1_it, 1);
  // (|x| < 0.5: 2 + x in [1.5, 2.5], so the ~1-ulp reciprocal serves both
  // quotients)
  const double r2x = recip_fast(2.0 + x);
  const double u = x * r2x, v = u * u;
  double s = 1.0 / 33.0;
#pragma unroll
  for (int k = 14; k >= 0; --k) s = s * v + 1.0 / (2 * k + 3);
  return 2.0 * u * v * s - x * x * r2x;
}

H3D_HD double log1pmx(double x) {
  if (fabs(x) < 0.5) return log1pmx_small(x);
  return log1p(x) - x;
}

// log Gamma(1 + x) accurate near x = 0 (cephes lgam1p).
H3D_HD double lgam1p_taylor(double x) {
  const double zeta[] = {
      1.64493406684822663e+00, 1.20205690315959401e+00, 1.08232323371113814e+00,
      1.03692775514337043e+00, 1.01734306198444879e+00, 1.00834927738192293e+00,
      1.00407735619794458e+00, 1.00200839282608256e+00, 1.00099457512781820e+00,
      1.00049418860411943e+00, 1.00024608655330782e+00, 1.00012271334757852e+00,
      1.00006124813505859e+00, 1.00003058823630719e+00, 1.00001528225940839e+00,
      1.00000763719763763e+00, 1.00000381729326504e+00, 1.00000190821271628e+00,
      1.00000095396203381e+00, 1.00000047693298666e+00, 1.00000023845050268e+00,
      1.00000011921992593e+00, 1.00000005960818905e+00, 1.00000002980350344e+00,
      1.00000001490155488e+00, 1.00000000745071183e+00, 1.00000000372533404e+00,
      1.00000000186265980e+00, 1.00000000093132746e+00, 1.00000000046566284e+00,
      1.00000000023283109e+00, 1.00000000011641554e+00, 1.00000000005820766e+00,
      1.00000000002910383e+00, 1.00000000001455192e+00, 1.00000000000727596e+00,
      1.00000000000363798e+00, 1.00000000000181899e+00, 1.00000000000090949e+00,
      1.00000000000045475e+00};
  if (x == 0.0) return 0.0;
  double res = -kEuler * x;
  double xfac = -x;
  for (int n = 2; n < 42; ++n) {
    xfac *= -x;
    double coeff = zeta[n - 2] * xfac / n;
    res += coeff;
    if (fabs(coeff) < kMachEp * fabs(res)) break;
  }
  return res;
}

H3D_HD double lgam1p(double x) {
  if (fabs(x) <= 0.5) return lgam1p_taylor(x);
  if (fabs(x - 1.0) < 0.5) return log(x) + lgam1p_taylor(x - 1.0);
  return lgam(x + 1.0);
}

// lgamma(a) - Stirling's leading terms, a >= 10.
H3D_HD double stirling_corr(double a) {
  const double r = recip_fast(a), r2 = r * r;  // a >= 10
  return r * (1.0 / 12.0 +
              r2 * (-1.0 / 360.0 +
                    r2 * (1.0 / 1260.0 +
                          r2 * (-1.0 / 1680.0 +
                                r2 * (1.0 / 1188.0 +
                                      r2 * (-691.0 / 360360.0 +
                                            r2 * (1.0 / 156.0)))))));
}

// x^a e^-x / Gamma(a), given lga = lgam(a).
// (table-driven log_fast / straight-line exp_fast: the exponent's own
// conditioning, a few ulp of |a ln x|, dominates their <= 1 ulp)
H3D_HD double igam_fac_l(double a, double x, double lga, const LogTab* tab = kLogTab) {
  // the plain exponent below a = 50, a deliberate speed-for-accuracy trade:
  // near x ~ a the exponent a ln x - x - lgamma(a) cancels (its derivatives
  // in a and x vanish at the mode, so the prefactor itself is well
  // conditioned there) and its rounding, ~2e-16 x |a ln x|, becomes relative
  // error of the prefactor -- measured up to 8e-14 at a in [10, 50) against
  // 2.8e-14 for cephes' log1pmx form above 50 (test_special_host.py::
  // test_igam_plain_prefactor_near_the_mode pins both). It stays far inside
  // the equalize pass' 1e-10 bar, and the wave no longer splits over the two
  // forms at a ~ 10..20, the equalize pass' common shapes (r05s: -1 %).
  if (fabs(a - x) > 0.4 * fabs(a) || a < 50.0) {
    double ax = a * log_fast_checked(x, tab) - x - lga;
    if (ax < -kMaxLog) return 0.0;
    return exp_fast(ax);
  }
  H3D_STAT(fac_l1, 1);
  double s = div_fast(x - a, a);  // a >= 10; |s| <= 0.4 here
  return exp_fast(a * log1pmx_small(s) + 0.5 * log_fast_checked(a / kTwoPi, tab) -
                  stirling_corr(a));
}

H3D_HD double igam_fac(double a, double x) { return igam_fac_l(a, x, lgam(a)); }

// power series sum of P(a, x) = fac / a * sum (DLMF 8.11.4):
//   sum_n x^n / ((a+1) ... (a+n)),
// four terms per trip from ONE reciprocal: with D = (r+1)(r+2)(r+3)(r+4) and
// the last term c,
//   c1 = c x (r+2)(r+3)(r+4) / D, c2 = c x^2 (r+3)(r+4) / D,
//   c3 = c x^3 (r+4) / D,        c4 = c x^4 / D,
// (x^2, x^3, x^4 hoisted out of the loop) and one stopping test per trip:
// the sum stops once a trip's last term is <= eps * sum (cephes igam_series
// tests every term; the up to three further terms it adds are each below
// eps * sum, so the value moves by an ulp at most). On gfx950 the reciprocal
// is v_rcp_f64 + one Newton step (~1 ulp; the IEEE division sequence was 40%
// of a trip); the host build divides. Measured on gfx950 r03: the two-term
// form with a per-term test spent ~11.5 VALU per term plus an exec-mask
// branch per term; this form ~7.
// The trip's four terms join the sum as ONE Horner group,
//   c1 + c2 + c3 + c4 = cd x (q + x (p34 + x (r4 + x))),  q = r2 p34,
// (den = (r+1) q shares q): ~19 VALU per trip instead of ~30 (r03 form: the
// terms one by one, ~11 multiplies). All terms are positive, so the group
// is accurate to an ulp of itself; the sum moves by rounding only.
H3D_HD double igam_series_sum(double a, double x) {
#if defined(__clang__)
#pragma clang fp contract(fast)
#endif
  const double x4 = (x * x) * (x * x);
  double r = a, c = 1.0, ans = 1.0;
  for (int i = 0; i < kMaxIter / 4; ++i) {
    H3D_STAT(ser_it, 4);
    const double r2 = r + 2.0, r3 = r + 3.0, r4 = r + 4.0;
    const double p34 = r3 * r4;
    const double q = r2 * p34;
    const double den = (r + 1.0) * q;
#if defined(__HIP_DEVICE_COMPILE__)
    const double cd = c * recip_nll(den);
#else
    const double cd = c / den;
#endif
    const double h = (x * ((x * (r4 + x)) + p34) + q) * x;
    ans += h * cd;
    const double c4 = cd * x4;
    c = c4;
    if (c4 <= kMachEp * ans) break;
    r = r4;
  }
  return ans;
}

// P(a, x) by its power series.
H3D_HD double igam_series(double a, double x) {
  double ax = igam_fac(a, x);
  if (ax == 0.0) return 0.0;
  return igam_series_sum(a, x) * ax / a;
}

// Q(a, x) for small x without cancellation (DLMF 8.7.3), given lga. Out of
// line: taken by < 1% of the equalize lanes, but inlined its lgam1p Taylor
// table doubled the equalize kernel's spills (224 -> 112 B/lane at W=4).
H3D_HD_COLD double igamc_series_l(double a, double x, double lga) {
  double fac = 1.0, sum = 0.0;
  for (int n = 1; n < kMaxIter; ++n) {
    H3D_STAT(su_it, 1);
    fac *= -x / n;
    double term = fac / (a + n);
    sum += term;
    if (fabs(term) <= kMachEp * fabs(sum)) break;
  }
  double logx = log(x);
  double term = -expm1(a * logx - lgam1p(a));
  return term - exp(a * logx - lga) * sum;
}

H3D_HD double igamc_series(double a, double x) {
  return igamc_series_l(a, x, lgam(a));
}

// continued-fraction value of Q(a, x) / fac (DLMF 8.9.2), cephes igamc's
// recurrence without the two divisions per step: consecutive convergents
// p_{k-1}/q_{k-1}, p_k/q_k are compared by cross-multiplication,
//   |p_k q_{k-1} - p_{k-1} q_k| <= tol |p_k q_{k-1}|,
// and the quotient is formed once, after the loop. tol = 4 eps: the fused
// cross product is exact to ~1 eps of |p_k q_{k-1}|, so the test is met once
// the convergents agree to ~3 eps (cephes: once they round to the same
// double). Four steps per trip (two of each register pair, so no moves
// between steps), one test and one overflow rescale per trip: the up to
// three steps past the first converged one only refine the value further.
// The rescale multiplies all four terms by 2^-64 once |p| exceeds 2^64
// (exact: changes neither the test nor the quotient; |p0| ~ |p1|, and four
// steps grow them by ~z^4, far inside the double range for the q2qnbinom
// arguments).
// Measured on gfx950 r03: with a test per step and the quotient inside the
// loop, the compiler emitted the IEEE division in a masked block executed
// every time any lane of the wave converged, and ~12 exec-mask instructions
// per step.
H3D_HD double igamc_cf_ratio(double a, double x) {
#if defined(__clang__)
  // contraction (the convergents' products fuse into FMAs) -- the ratio
  // agrees with the uncontracted recurrence to ~1 ulp
#pragma clang fp contract(fast)
#endif
  const double y0 = 1.0 - a;
  double z = x + y0 + 1.0;
  // y c of step k = k (y0 + k) by its forward difference y0 + 2k + 1 (two
  // additions per step instead of the three counters and a product); exact
  // for integer-spaced terms up to rounding, which the 4-eps test absorbs
  double yc = 0.0, dyc = y0 + 1.0;
  // (p1, q1): the latest convergent, (p0, q0): the one before
  double p0 = 1.0, q0 = x, p1 = x + 1.0, q1 = z * x;
  for (int i = 0; i < kMaxIter / 4; ++i) {
    H3D_STAT(cf_it, 4);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      yc += dyc;
      dyc += 2.0;
      z += 2.0;
      p0 = p1 * z - p0 * yc;  // step A: new latest in (p0, q0)
      q0 = q1 * z - q0 * yc;
      yc += dyc;
      dyc += 2.0;
      z += 2.0;
      p1 = p0 * z - p1 * yc;  // step B: new latest in (p1, q1)
      q1 = q0 * z - q1 * yc;
    }
    const double lead = p1 * q0;
    if ((q1 != 0.0) && fabs(lead - p0 * q1) <= 4.0 * kMachEp * fabs(lead)) break;
    // the rescale only where a lane needs it (rare): the four multiplies
    // by 1 every trip were ~15% of the trip
    if (fabs(p1) > 0x1p64) {
      p0 *= 0x1p-64;
      q0 *= 0x1p-64;
      p1 *= 0x1p-64;
      q1 *= 0x1p-64;
    }
  }
  return div_fast(p1, q1);  // (q1 normal: the rescale keeps it in range)
}

// Q(a, x) by the continued fraction.
H3D_HD double igamc_cf(double a, double x) {
  double ax = igam_fac(a, x);
  if (ax == 0.0) return 0.0;
  return igamc_cf_ratio(a, x) * ax;
}

// P(a, x), Q(a, x) and fac = x^a e^-x / Gamma(a) in one evaluation, given
// lga = lgam(a) (a > 0, x > 0 finite). The branch structure follows cephes
// igam/igamc: the tail that is computed directly is the accurate one, the
// other is 1 - it.
// tail = 1 / 0: the caller needs Q / P accurately. Then the method that
// converges fastest for that tail is used -- the power series (Q = 1 - P)
// for Q within 3 sqrt(a) of the mean at shapes a < 8, else the continued
// fraction for Q whenever x > 1; the power series for P up to x < 1.5 a + 5
// -- instead of cephes' x-vs-a switch, so lanes of a wave that want the same
// tail mostly take the same branch. tail = -1: the cephes rule.
H3D_HD void igam_pq(double a, double x, double lga, double* P, double* Q,
                    double* fac, int tail = -1, const LogTab* tab = kLogTab,
                    int sec = 0) {
  H3D_STAT(pq, 1);
  H3D_SEC_BEGIN(t_fac);
  const double f = igam_fac_l(a, x, lga, tab);
  *fac = f;
  H3D_SEC_END(sec, t_fac);
  H3D_SEC_BEGIN(t_loop);
  // v = the directly computed tail, is_q = whether it is Q; P and Q are then
  // written once, by selects (per-branch stores through P / Q made the
  // compiler keep them in a dynamically indexed scratch pair)
  double v;
  bool is_q;
#if defined(H3D_INSTRUMENT) && !defined(__HIP_DEVICE_COMPILE__)
  const long it0 = g_stats ? g_stats->cf_it + g_stats->su_it + g_stats->ser_it : 0;
#endif
  // Which method computes the directly evaluated tail. Trip counts (gfx950
  // ISA: ~21 VALU per four series terms, ~40 per four continued-fraction
  // steps): for shapes a < 8 near the mean the series converges in far
  // fewer VALU than the fraction (a = 2.7, x = a: 6 trips against 8 of the
  // fraction's twice-as-dear ones; a = 1.3: 5 against 15), so Q is taken as
  // 1 - P there -- (x - a)^2 < 9 a keeps Q >= ~1e-3, i.e. its relative
  // rounding <= ~2e-13 -- and the fraction only for the far upper tail and
  // the larger shapes (census, tools/q2q_stats.py: the equalize pass' loop
  // cost per wave -26 .. -34 %, modelled lane utilisation 0.77 -> 0.81)
  const double xa = x - a;
  const bool use_cf = (tail == 1)   ? (x > 1.0 && !(a < 8.0 && xa * xa < 9.0 * a))
                     : (tail == 0) ? (x > 1.0 && x > a && !(x < 1.5 * a + 5.0))
                                   : (x > 1.0 && x > a);
  if (use_cf) {  // continued fraction for the upper tail
    H3D_STAT(cf, 1);
    v = (f == 0.0) ? 0.0 : igamc_cf_ratio(a, x) * f;
    is_q = true;
  } else if ((x <= 1.1) &&
             ((x <= 0.5) ? !(a * log_fast(x, tab) < -0.4) : !(x * 1.1 < a))) {
    // (cephes' -0.4 / ln x < a as a ln x < -0.4 -- ln x < 0 here -- with the
    // table log: the libm log and IEEE division were inlined into every
    // incomplete-gamma evaluation of the inverse's Halley loop, ~110 VALU of
    // its ~250 per trip, for the waves with a lane at x <= 0.5. A rounding-
    // level tie only picks the other, equally accurate method.)
    // Q without cancellation when P is close to 1
    H3D_STAT(su, 1);
    v = igamc_series_l(a, x, lga);
    is_q = true;
  } else {
    H3D_STAT(ser, 1);
    v = (f == 0.0) ? 0.0 : div_fast(igam_series_sum(a, x) * f, a);
    is_q = false;
  }
#if defined(H3D_INSTRUMENT) && !defined(__HIP_DEVICE_COMPILE__)
  if (g_stats)
    H3D_PQ_LOG(a, x, g_stats->cf_it + g_stats->su_it + g_stats->ser_it - it0,
               use_cf ? 0 : is_q ? 1 : 2);
#endif
  const double w = 1.0 - v;
  *P = is_q ? w : v;
  *Q = is_q ? v : w;
  H3D_SEC_END(sec + 1, t_loop);
}

H3D_HD double igamc(double a, double x);

// Regularised lower incomplete gamma P(a, x) (scipy gammainc).
H3D_HD double igam(double a, double x) {
  if (x < 0.0 || a < 0.0 || a != a || x != x) return NAN;
  if (a == 0.0) return (x > 0.0) ? 1.0 : NAN;
  if (x == 0.0) return 0.0;
  if (is_inf(a)) return is_inf(x) ? NAN : 0.0;
  if (is_inf(x)) return 1.0;
  if (x > 1.0 && x > a) return 1.0 - igamc(a, x);
  return igam_series(a, x);
}

// Regularised upper incomplete gamma Q(a, x) (scipy gammaincc).
H3D_HD double igamc(double a, double x) {
  if (x < 0.0 || a < 0.0 || a != a || x != x) return NAN;
  if (a == 0.0) return (x > 0.0) ? 0.0 : NAN;
  if (x == 0.0) return 1.0;
  if (is_inf(a)) return is_inf(x) ? NAN : 1.0;
  if (is_inf(x)) return 0.0;
  if (x > 1.1) {
    if (x < a) return 1.0 - igam_series(a, x);
    return igamc_cf(a, x);
  } else if (x <= 0.5) {
    if (-0.4 / log(x) < a) return 1.0 - igam_series(a, x);
    return igamc_series(a, x);
  } else {
    if (x * 1.1 < a) return 1.0 - igam_series(a, x);
    return igamc_series(a, x);
  }
}

// ---------------------------------------------------------------------------
// normal distribution
// ---------------------------------------------------------------------------

// Standard normal CDF (cephes ndtr).
H3D_HD double ndtr(double a) {
  if (a != a) return NAN;
  double x = a * kSqrt1_2, z = fabs(x), y;
  if (z < kSqrt1_2) {
    y = 0.5 + 0.5 * erf(x);
  } else {
    // cephes erfc underflows to exactly 0 once z^2 > MAXLOG (the reference
    // then maps sf = 0 to isf = inf); libm would return a subnormal instead
    y = (z * z > kMaxLog) ? 0.0 : 0.5 * erfc(z);
    if (x > 0.0) y = 1.0 - y;
  }
  return y;
}

// Lower-tail quantile for q in (0, 0.5]: Acklam's rational guess refined by
// two Halley steps on Phi(x) = erfc(-x/sqrt2)/2 (relative-accurate for x<=0).
H3D_HD double ndtri_lower(double q) {
  const double a[] = {-3.969683028665376e+01, 2.209460984245205e+02,
                      -2.759285104469687e+02, 1.383577518672690e+02,
                      -3.066479806614716e+01, 2.506628277459239e+00};
  const double b[] = {-5.447609879822406e+01, 1.615858368580409e+02,
                      -1.556989798598866e+02, 6.680131188771972e+01,
                      -1.328068155288572e+01};
  const double c[] = {-7.784894002430293e-03, -3.223964580411365e-01,
                      -2.400758277161838e+00, -2.549732539343734e+00,
                      4.374664141464968e+00, 2.938163982698783e+00};
  const double d[] = {7.784695709041462e-03, 3.224671290700398e-01,
                      2.445134137142996e+00, 3.754408661907416e+00};
  double x;
  if (q < 0.02425) {
    double t = sqrt(-2.0 * log(q));
    x = (((((c[0] * t + c[1]) * t + c[2]) * t + c[3]) * t + c[4]) * t + c[5]) /
        ((((d[0] * t + d[1]) * t + d[2]) * t + d[3]) * t + 1.0);
  } else {
    double t = q - 0.5, r = t * t;
    x = (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) *
        t /
        (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1.0);
  }
  // Acklam's guess is good to 1.2e-9 relative: one Halley step is enough
  for (int it = 0; it < 1; ++it) {
    // residual Phi(x) - q; near the centre via erf (q - 0.5 exact there)
    double e = (q > 0.25) ? 0.5 * erf(x * kSqrt1_2) - (q - 0.5)
                          : 0.5 * erfc(-x * kSqrt1_2) - q;
    // u = e * sqrt(2 pi) * exp(x^2/2), split to stay finite deep in the tail
    double h = exp(0.25 * x * x);
    double u = (e * h) * h * kSqrt2Pi;
    x = x - u / (1.0 + 0.5 * x * u);
  }
  return x;
}

// Standard normal quantile (scipy ndtri).
H3D_HD double ndtri(double p) {
  if (p != p) return NAN;
  if (p <= 0.0) return (p == 0.0) ? -INFINITY : NAN;
  if (p >= 1.0) return (p == 1.0) ? INFINITY : NAN;
  if (p > 0.5) return -ndtri_lower(1.0 - p);  // 1 - p exact (Sterbenz)
  return ndtri_lower(p);
}

// ---------------------------------------------------------------------------
// inverse incomplete gamma (scipy gammaincinv / gammainccinv)
// ---------------------------------------------------------------------------

H3D_HD double dm_eq25(double a, double y) {
  double c1 = (a - 1) * log(y);
  double c1_2 = c1 * c1, c1_3 = c1_2 * c1, c1_4 = c1_2 * c1_2;
  double a_2 = a * a, a_3 = a_2 * a;
  double c2 = (a - 1) * (1 + c1);
  double c3 = (a - 1) * (-(c1_2 / 2) + (a - 2) * c1 + (3 * a - 5) / 2);
  double c4 = (a - 1) * ((c1_3 / 3) - (3 * a - 5) * c1_2 / 2 +
                         (a_2 - 6 * a + 7) * c1 + (11 * a_2 - 46 * a + 47) / 6);
  double c5 = (a - 1) * (-(c1_4 / 4) + (11 * a - 17) * c1_3 / 6 +
                         (-3 * a_2 + 13 * a - 13) * c1_2 +
                         (2 * a_3 - 25 * a_2 + 72 * a - 61) * c1 / 2 +
                         (25 * a_3 - 195 * a_2 + 477 * a - 379) / 12);
  double y_2 = y * y, y_3 = y_2 * y, y_4 = y_2 * y_2;
  return y + c1 + (c2 / y) + (c3 / y_2) + (c4 / y_3) + (c5 / y_4);
}

H3D_HD double dm_find_s(double p, double q) {
  // DiDonato & Morris eq. 32, coefficients in descending powers of t
  const double a[] = {0.213623493715853, 4.28342155967104, 11.6616720288968,
                      3.31125922108741};
  const double b[] = {0.3611708101884203e-1, 1.27364489782223,
                      6.40691597760039, 6.61053765625462, 1.0};
  double t = (p < 0.5) ? sqrt(-2 * log(p)) : sqrt(-2 * log(q));
  double s = t - polevl(t, a, 3) / polevl(t, b, 4);
  return (p < 0.5) ? -s : s;
}

H3D_HD double dm_sn(double a, double x, int N, double tol) {
  double sum = 1.0;
  if (N >= 1) {
    double partial = x / (a + 1);
    sum += partial;
    for (int i = 2; i <= N; ++i) {
      partial *= x / (a + i);
      sum += partial;
      if (partial < tol) break;
    }
  }
  return sum;
}

// DiDonato & Morris (1986) initial guess for the inverse of P(a, .) = p,
// Q(a, .) = q (p + q = 1), given lga = lgam(a).
H3D_HD double find_inverse_gamma(double a, double p, double q, double lga) {
  double result;
  if (a == 1.0) {
    result = (q > 0.9) ? -log1p(-p) : -log(q);
  } else if (a < 1.0) {
    double g = exp(lga);
    double b = q * g;
    if ((b > 0.6) || ((b >= 0.45) && (a >= 0.3))) {
      double u;
      if ((b * q > 1e-8) && (q > 1e-5))
        u = pow(p * g * a, 1 / a);
      else
        u = exp((-q / a) - kEuler);
      result = u / (1 - (u / (a + 1)));
    } else if ((a < 0.3) && (b >= 0.35)) {
      double t = exp(-kEuler - b);
      double u = t * exp(t);
      result = t * exp(u);
    } else if ((b > 0.15) || (a >= 0.3)) {
      double y = -log(b);
      double u = y - (1 - a) * log(y);
      result = y - (1 - a) * log(u) - log(1 + (1 - a) / (1 + u));
    } else if (b > 0.1) {
      double y = -log(b);
      double u = y - (1 - a) * log(y);
      result = y - (1 - a) * log(u) -
               log((u * u + 2 * (3 - a) * u + (2 - a) * (3 - a)) /
                   (u * u + (5 - a) * u + 2));
    } else {
      result = dm_eq25(a, -log(b));
    }
  } else {
    double s = dm_find_s(p, q);
    double s_2 = s * s, s_3 = s_2 * s, s_4 = s_2 * s_2, s_5 = s_4 * s;
    double ra = sqrt(a);
    double w = a + s * ra + (s_2 - 1) / 3;
    w += (s_3 - 7 * s) / (36 * ra);
    w -= (3 * s_4 + 7 * s_2 - 16) / (810 * a);
    w += (9 * s_5 + 256 * s_3 - 433 * s) / (38880 * a * ra);
    if ((a >= 500) && (fabs(1 - w / a) < 1e-6)) {
      result = w;
    } else if (p > 0.5) {
      if (w < 3 * a) {
        result = w;
      } else {
        double D = fmax(2.0, a * (a - 1));
        double lb = log(q) + lga;
        if (lb < -D * 2.3) {
          result = dm_eq25(a, -lb);
        } else {
          double u = -lb + (a - 1) * log(w) - log(1 + (1 - a) / (1 + w));
          result = -lb + (a - 1) * log(u) - log(1 + (1 - a) / (1 + u));
        }
      }
    } else {
      double z = w;
      double ap1 = a + 1, ap2 = a + 2;
      const double lg_ap1 = lga + log(a);  // lgam(a + 1)
      if (w < 0.15 * ap1) {
        double v = log(p) + lg_ap1;
        z = exp((v + w) / a);
        s = log1p(z / ap1 * (1 + z / ap2));
        z = exp((v + z - s) / a);
        s = log1p(z / ap1 * (1 + z / ap2));
        z = exp((v + z - s) / a);
        s = log1p(z / ap1 * (1 + z / ap2 * (1 + z / (a + 3))));
        z = exp((v + z - s) / a);
      }
      if ((z <= 0.01 * ap1) || (z > 0.7 * ap1)) {
        result = z;
      } else {
        double ls = log(dm_sn(a, z, 100, 1e-4));
        double v = log(p) + lg_ap1;
        z = exp((v + z - ls) / a);
        result = z * (1 - (a * log(z) - z - v + ls) / (a - z));
      }
    }
  }
  return result;
}

// P(a, xe + h) - P(a, xe) and P'(xe + h) / P'(xe) from P'(xe) alone, for a
// step h: P'(x) = x^(a-1) e^-x / Gamma(a), so
//   P'(xe + s) / P'(xe) = exp(g(s)),  g(s) = (a-1) ln(1 + s/xe) - s,
// and exp(g) = sum e_k s^k by the power-series exponential recurrence
// e_k = (1/k) sum_j j g_j e_(k-j) on g's Taylor coefficients
// g_j = (a-1) (-1)^(j+1) / (j xe^j) (- 1 for j = 1). K = 12 terms, fixed
// length (no lane divergence). Used inside the window igam_taylor_ok, where
// the dropped terms are below (|g_1 h|)^13 / 13! and |a-1| (h/xe)^13 / 13,
// i.e. < 2e-15 x/h of the increment -- the root it leads to moves < 1e-16
// relative.
constexpr int kTaylorK = 12;

// (one ~1-ulp reciprocal of xe for both quotients: a window test, and a
// subnormal xe -- 1/xe flushed to inf on gfx950 -- fails it safely)
H3D_HD bool igam_taylor_ok(double a, double xe, double h) {
  const double rx = recip_fast(xe);
  const double u = h * rx;
  return xe > 0.0 && fabs(u) <= 0.05 &&
         fabs(((a - 1.0) * rx - 1.0) * h) <= 0.4 &&
         fabs(a - 1.0) * u * u <= 0.25;
}

// The coefficients follow from the ODE y' = g'(s) y, g'(s) = b / (xe + s) - 1
// (b = a - 1): (xe + s) y' = (b - xe - s) y gives the three-term recurrence
//   e_(k+1) = ((b - xe - k) e_k - e_(k-1)) / (xe (k + 1)),  e_(-1) = 0,
// i.e. in the scaled E_k = e_k h^k (s = h t, t in [0, 1])
//   E_(k+1) = u ((b - xe - k) E_k - h E_(k-1)) / (k + 1),  u = h / xe.
// Both terms decay (ratios ~ -u and ~ -h / k), so the forward recursion is
// stable; only two coefficients are live at a time (the convolution form of
// the power-series exponential kept all 2K + 1 in registers).
H3D_HD void igam_step_taylor(double a, double xe, double h, double* dint,
                             double* ratio) {
#if defined(__clang__)
#pragma clang fp contract(fast)
#endif
  constexpr int K = kTaylorK;
  const double b = a - 1.0;
  const double u = h * recip_fast(xe);  // xe normal: igam_taylor_ok held
  const double c0 = b - xe;
  double em1 = 0.0, e = 1.0;
  // integral_0^h = h sum E_k / (k+1); exp(g(h)) = sum E_k
  double in = 1.0, ex = 1.0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double en = u * ((c0 - k) * e - h * em1) * (1.0 / (k + 1));
    em1 = e;
    e = en;
    in += e * (1.0 / (k + 2));
    ex += e;
  }
  *dint = in * h;
  *ratio = ex;
}

// Inverse incomplete gamma on either tail: solves P(a, x) = t (upper=false)
// or Q(a, x) = t (upper=true), t in (0, 1), given lga = lgam(a). As scipy's
// igami/igamci it always works on the tail that is <= 0.9 and refines the
// DiDonato & Morris guess with Halley steps (f''/f' = (a-1)/x - 1). It stops
// once a step moved x by <= 1e-6 relative: Halley converges cubically, so the
// error left is ~1e-18 (scipy always takes 3).
// Residual evaluation: a full igam_pq where x moved far from the last full
// evaluation xe; otherwise the residual is continued from xe by the Taylor
// increment of P (igam_step_taylor), which is exact to ~1e-17 of the step and
// costs ~40 flops instead of a series / continued fraction. A good guess
// (~1e-4 relative) thus takes ONE incomplete-gamma evaluation: the confirming
// Halley step runs on the continuation.
H3D_HD double igam_inv(double a, double t, bool upper, double lga,
                       double guess = -1.0, const LogTab* tab = kLogTab) {
  H3D_STAT(inv, 1);
  H3D_STAT(wh, guess > 0.0);
  if (t > 0.9) {
    t = 1.0 - t;
    upper = !upper;
  }
  H3D_SEC_BEGIN(t_dm);
  double x = (guess > 0.0) ? guess
                           : upper ? find_inverse_gamma(a, 1.0 - t, t, lga)
                                   : find_inverse_gamma(a, t, 1.0 - t, lga);
  H3D_SEC_END(10, t_dm);
  // last full evaluation: point, residual F = tail(x) - t, slope P'(x)
  double xe = -1.0, Fe = 0.0, dPe = 0.0;
  for (int i = 0; i < 8; ++i) {
    H3D_STAT(halley, 1);
    double F, dP;
    const double h = x - xe;
    H3D_SEC_BEGIN(t_tay);
    const bool tay = igam_taylor_ok(a, xe, h);
    if (tay) {
      double dint, ratio;
      igam_step_taylor(a, xe, h, &dint, &ratio);
      const double dPint = dPe * dint;  // P(x) - P(xe)
      F = upper ? Fe - dPint : Fe + dPint;
      dP = dPe * ratio;
    }
    H3D_SEC_END(11, t_tay);
    if (!tay) {
      double P, Q, fac;
      igam_pq(a, x, lga, &P, &Q, &fac, upper ? 1 : 0, tab, 8);
      if (fac == 0.0) return x;
      F = (upper ? Q : P) - t;
      dP = fac / x;
      xe = x;
      Fe = F;
      dPe = dP;
    }
    // Newton ratio f / f' (f' = -P' on the upper tail), Halley correction
    // f / f' and (a - 1) / x: ~1-ulp quotients where the divisor is a
    // normal number, IEEE divisions where it is not -- P' and x reach the
    // subnormal range deep in the tails, where v_rcp_f64 flushes (found by
    // the gfx950 unit grids); only a wave with such a lane takes that
    // branch. The Halley denominator ~1 takes the ~1-ulp quotient.
    H3D_SEC_BEGIN(t_hal);
    const bool nrm = fabs(dP) >= 0x1p-1000 && x >= 0x1p-1000;
    double f_fp, fpp_fp;
    if (nrm) {
      f_fp = div_fast(upper ? -F : F, dP);
      fpp_fp = -1.0 + div_fast(a - 1, x);
    } else {
      f_fp = upper ? -F / dP : F / dP;
      fpp_fp = -1.0 + (a - 1) / x;
    }
    double xn = is_inf(fpp_fp) ? x - f_fp
                               : x - div_fast(f_fp, 1.0 - 0.5 * f_fp * fpp_fp);
    if (!(xn > 0.0)) xn = 0.5 * x;  // safeguard: stay in the support
    const double dx = fabs(xn - x);
    x = xn;
    H3D_SEC_END(12, t_hal);
    if (dx <= 1e-6 * x) break;
  }
  return x;
}

// Inverse of P(a, .) (scipy gammaincinv).
H3D_HD double igami(double a, double p) {
  if (a != a || p != p) return NAN;
  if (a < 0.0 || p < 0.0 || p > 1.0) return NAN;
  if (p == 0.0) return 0.0;
  if (p == 1.0) return INFINITY;
  return igam_inv(a, p, false, lgam(a));
}

// Inverse of Q(a, .) (scipy gammainccinv).
H3D_HD double igamci(double a, double q) {
  if (a != a || q != q) return NAN;
  if (a < 0.0 || q < 0.0 || q > 1.0) return NAN;
  if (q == 0.0) return INFINITY;
  if (q == 1.0) return 0.0;
  return igam_inv(a, q, true, lgam(a));
}

// chi2(df).sf(x) as scipy.stats: support lower bound -> 1 (cephes chdtrc).
// df = 1 and 2 (the LRT with 2 and 3 conditions) use the closed forms
// Q(1/2, y) = erfc(sqrt(y)) and Q(1, y) = exp(-y) instead of the series /
// continued fraction (same values to a few ulp).
H3D_HD double chi2_sf(double df, double x);

// chi2_sf out of line: the LRT kernels' general-df fallback (designs of
// four or more conditions), kept from inflating the register budget of the
// closed-form paths they take otherwise
H3D_HD_COLD double chi2_sf_cold(double df, double x) { return chi2_sf(df, x); }

H3D_HD double chi2_sf(double df, double x) {
  if (x != x) return NAN;
  if (x <= 0.0) return 1.0;
  if (df == 1.0) return erfc(sqrt(x / 2.0));
  if (df == 2.0) return exp(-x / 2.0);
  return igamc(df / 2.0, x / 2.0);
}

}  // namespace h3d
