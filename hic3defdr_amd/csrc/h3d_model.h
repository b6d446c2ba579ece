// Scaled negative-binomial model pieces shared by the gfx950 kernels and the
// host unit-test build. Each function cites the reference code it restates
// (reference = thomasgilgenast/hic3defdr 0.2.1).
//
// Register discipline: per-pixel replicate vectors live in fixed-size local
// arrays of M slots (M a template constant >= the runtime count n), and every
// loop runs over all M slots with an `k < n` (or mask) predicate. After
// inlining and unrolling, every array index is a compile-time constant, so
// the arrays stay in VGPRs on gfx950 instead of spilling to scratch.
#pragma once

#include <cmath>

#include "h3d_special.h"

namespace h3d {

constexpr int kMaxReps = 32;  // replicates per pixel (R)
constexpr int kMaxConds = 8;  // conditions (C)

// status flags (OR-ed per pixel / per segment, reported by the C ABI)
constexpr int kFlagNoRoot = 1;     // all-zero counts: no MLE (ref: ValueError)
constexpr int kFlagNoConv = 2;     // MLE solver did not converge
constexpr int kFlagBrentFail = 4;  // bounded Brent not successful (ref: assert)
constexpr int kFlagQcmlGuard = 8;  // qcml exceeded 1000 iterations
constexpr int kFlagBadInput = 16;  // alpha/b not positive finite (ref: assert)

// numpy's row-sum association for a short contiguous row of n <= M values
// (pairwise_sum with n <= 128: sequential below 8, eight accumulators from 8).
template <int M>
H3D_HD double np_sum(const double* v, int n) {
  if (n < 8) {
    double res = 0.0;
#pragma unroll
    for (int i = 0; i < (M < 8 ? M : 8); ++i)
      if (i < n) res += v[i];
    return res;
  }
  if constexpr (M >= 8) {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = v[j];
    const int blk = n - (n % 8);
#pragma unroll
    for (int i = 8; i < M; ++i)
      if (i < blk) r[i % 8] += v[i];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int i = 8; i < M; ++i)
      if (i >= blk && i < n) res += v[i];
    return res;
  }
  return NAN;
}

// np_sum's association fed one value at a time, in index order k = 0..n-1
// (the same additions in the same order, so the same bits): the caller needs
// no array of the n values -- 8 accumulators instead of M registers.
struct NpSumStream {
  double r[8];
  double res;
  int n, blk;
  H3D_HD explicit NpSumStream(int n_) : res(0.0), n(n_), blk(n_ - n_ % 8) {}
  H3D_HD void add(int k, double v) {
    if (n < 8) {
      res += v;
    } else if (k < 8) {
      r[k] = v;
    } else if (k < blk) {
      r[k % 8] += v;
    } else {
      if (k == blk) res = combine();
      res += v;
    }
  }
  // the same with a runtime position j (compacted subsets): register
  // selects instead of an indexed accumulator array (no scratch)
  H3D_HD void add_dyn(int j, double v) {
    if (n < 8 || j >= blk) {
      if (n >= 8 && j == blk) res = combine();
      res += v;
      return;
    }
#pragma unroll
    for (int t = 0; t < 8; ++t)
      if (t == (j & 7)) r[t] = (j < 8) ? v : r[t] + v;
  }
  H3D_HD double combine() const {
    return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  }
  H3D_HD double sum() const { return (n >= 8 && blk == n) ? combine() : res; }
};

// MLE of mu under fixed per-replicate dispersion: root of
//   S(mu) = sum_k (x_k - mu b_k) / (mu + a_k mu^2 b_k)      (scaled_nb.py:143-147)
// over the replicates k < n with bit k of `mask` set.
// The reference finds it with scipy's array secant + a brentq fallback
// (scaled_nb.py:149-181). The log-likelihood is strictly concave in
// theta = log(mu), so the root is unique; here it is found per lane by
// Halley steps on g(theta) = mu S(mu) inside a shrinking bracket (bisection
// safeguard), to full double precision.
template <int M, typename TX>
H3D_HD double fit_mu(const TX* x, const double* b, const double* a, int n,
                     unsigned mask, int* status, const LogTab* tab = kLogTab) {
#if defined(__clang__)
  // contraction: the per-replicate score terms and the Halley quotients fuse
  // into FMAs (18 -> 14 FP64 instructions per replicate and step on gfx950);
  // the root is converged to full precision either way (the host build's
  // g++ keeps -ffp-contract=off)
#pragma clang fp contract(fast)
#endif
  double sx = 0.0, sb = 0.0;
  bool bad = false;
#pragma unroll
  for (int k = 0; k < M; ++k)
    if (k < n && ((mask >> k) & 1u)) {
      bad |= !(a[k] > 0.0) || !(b[k] > 0.0) || is_inf(a[k]) || is_inf(b[k]) ||
             !(x[k] >= 0.0);
      sx += x[k];
      sb += b[k];
    }
  if (bad) {
    *status |= kFlagBadInput;
    return NAN;
  }
  if (!(sx > 0.0)) {
    *status |= kFlagNoRoot;
    return NAN;
  }
  H3D_STAT(fit, 1);
  // start at sum(x) / sum(b), the MLE of the Poisson limit (alpha -> 0),
  // instead of the reference's secant start mean(x / b) (scaled_nb.py:150):
  // the root is unique and converged to full precision either way, and this
  // start is closer to it (wave of 64 pixels: 2.37 against 2.62 steps)
  // (the table log and straight-line exp of h3d_special.h: ~1 ulp, the
  // OCML forms carried constant copies; the MLE is Newton-converged anyway)
  const double q0 = div_fast(sx, sb);
  double th = log_fast_checked(q0, tab);
  double lo = -INFINITY, hi = INFINITY;
  for (int it = 0; it < 200; ++it) {
    H3D_STAT(fit_it, 1);
    // (the start's mu is the quotient itself, exp(log q0) to an ulp: one exp
    // fewer per fit)
    const double mu = (it == 0) ? q0 : exp_fast(th);
    double g = 0.0, gp = 0.0, gpp = 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k)
      if (k < n && ((mask >> k) & 1u)) {
        const double mb = mu * b[k];
        const double am = a[k] * mb;
        // v_rcp_f64 + one Newton step on gfx950 (the IEEE division sequence
        // was ~12 VALU per replicate and iteration)
        const double den = recip_fast(1.0 + am);
        g += (x[k] - mb) * den;
        // g' and g'' in theta: d(mb)/dtheta = mb, d(den)/dtheta = -am den^2
        const double t = mb * (1.0 + a[k] * x[k]) * den * den;
        gp -= t;
        gpp -= t * (1.0 - 2.0 * am * den);
      }
    if (g > 0.0)
      lo = th;
    else if (g < 0.0)
      hi = th;
    else
      return mu;
    // Halley's step g / (g' - g g'' / (2 g')), the Newton step where the
    // correction factor is far from 1 (away from the root; the bracket below
    // catches what is left). Near the root it converges cubically: once a
    // step is <= 1e-5 the error after it is ~1e-15, so take it and stop
    // (2.0 steps per fit on average, 2.4 per wave of 64 pixels against 3.5
    // for Newton with its 1e-8 exit, tools census r04). (Without an exit of
    // this kind, a final step below one ulp left th on the bracket edge and
    // fell through to ~50 bisections.)
    const double nt = g * recip_fast(gp);
    const double hf = 1.0 - 0.5 * nt * gpp * recip_fast(gp);
    const double dn = (hf >= 0.5 && hf <= 2.0) ? nt * recip_fast(hf) : nt;
    // the last step: exp(th - dn) = mu exp(-dn), |dn| <= 1e-5 max(1, |th|),
    // exp(-dn) by its cubic Taylor polynomial where |dn| <= 1e-4 (truncation
    // dn^4 / 24 < 5e-18) -- the final exp of every fit without its range
    // reduction
    if (fabs(dn) <= 1e-5 * fmax(1.0, fabs(th)))
      return (fabs(dn) <= 1e-4)
                 ? mu + mu * (-dn * (1.0 + -dn * (0.5 + -dn * (1.0 / 6.0))))
                 : exp_fast(th - dn);
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

// ---- scipy.stats frozen-distribution methods as the reference calls them
// (rv_continuous.sf/cdf/isf/ppf edge handling of scipy 1.7.1) ------------

H3D_HD double norm_sf(double x, double loc, double scale) {
  return ndtr(-((x - loc) / scale));
}
H3D_HD double norm_cdf(double x, double loc, double scale) {
  return ndtr((x - loc) / scale);
}
H3D_HD double norm_isf(double q, double loc, double scale) {
  if (q != q) return NAN;
  if (q == 0.0) return INFINITY;
  if (q == 1.0) return -INFINITY;
  return -ndtri(q) * scale + loc;
}
H3D_HD double norm_ppf(double q, double loc, double scale) {
  if (q != q) return NAN;
  if (q == 0.0) return -INFINITY;
  if (q == 1.0) return INFINITY;
  return ndtri(q) * scale + loc;
}
H3D_HD double gamma_sf(double x, double shape, double scale) {
  const double xs = x / scale;
  if (xs <= 0.0) return 1.0;
  return igamc(shape, xs);
}
H3D_HD double gamma_cdf(double x, double shape, double scale) {
  const double xs = x / scale;
  if (xs <= 0.0) return 0.0;
  return igam(shape, xs);
}
H3D_HD double gamma_isf(double q, double shape, double scale) {
  if (q != q) return NAN;
  if (q == 0.0) return INFINITY;
  if (q == 1.0) return 0.0;
  return igamci(shape, q) * scale;
}
H3D_HD double gamma_ppf(double q, double shape, double scale) {
  if (q != q) return NAN;
  if (q == 0.0) return 0.0;
  if (q == 1.0) return INFINITY;
  return igami(shape, q) * scale;
}

// q2qnbinom for one value (scaled_nb.py:217-275). mu_in / mu_out are
// clamped IN PLACE exactly as the reference does (:240-242) so the caller can
// carry the mu_out clamp into the next replicate (equalize, :209-213).
// lgamma of the output shape, reused across the replicates of a pixel (they
// share mu_out unless a clamp changes it)
struct LgamCache {
  double a = -1.0, lga = 0.0;
};

// log Gamma of the q2qnbinom gamma shapes (a = mu / r > 0 finite): the
// branch-light Stirling form of the NLL (lgam_nll: fixed 5- or 10-step shift,
// no data-dependent loop or division; absolute error <= ~5e-15, which moves
// the incomplete-gamma prefactor by the same relative amount). cephes lgam's
// shift loop below 13 with an IEEE division per step serialised the lanes of
// a wave (gfx950 r03 asm: two divergent loops per call).
H3D_HD double lgam_q2q(double a, const LogTab* tab = kLogTab) { return lgam_nll(a, tab); }

H3D_HD double lgam_cached(double a, LgamCache* c, const LogTab* tab = kLogTab) {
  if (!c) return lgam_q2q(a, tab);
  if (a != c->a) {
    c->a = a;
    c->lga = lgam_q2q(a, tab);
  }
  return c->lga;
}

// q2qnbinom's arithmetic on already clamped means (mi, mo), with lgam of the
// output gamma shape either given (lga_out) or taken from `cache` (lga_out
// NaN).
H3D_HD double q2q_core(double x, double mi, double mo, double alpha,
                       double lga_out, LgamCache* cache, const LogTab* tab = kLogTab);

H3D_HD double q2q(double x, double* mu_in, double* mu_out, double alpha,
                  LgamCache* cache = nullptr, const LogTab* tab = kLogTab) {
  if (!((*mu_in >= 0.25) && (*mu_out >= 0.25))) {
    *mu_in = 0.25;
    *mu_out = 0.25;
  }
  return q2q_core(x, *mu_in, *mu_out, alpha, NAN, cache, tab);
}

H3D_HD double q2q_core(double x, double mi, double mo, double alpha,
                       double lga_out, LgamCache* cache, const LogTab* tab) {
  // (the quotients here by div_fast: ~1 ulp on gfx950 instead of the IEEE
  // division sequence; the q2q values move by rounding only, test bar 1e-10)
  H3D_SEC_BEGIN(t_setup);
  const double r_in = 1 + alpha * mi, r_out = 1 + alpha * mo;
  const double v_in = mi * r_in, v_out = mo * r_out;
  const double rr_in = recip_fast(r_in);
  const double a_in = mi * rr_in, a_out = div_fast(mo, r_out);
  // right tail: isf(sf(x)); left tail: ppf(cdf(x)). Both tails go through
  // the same code with a per-lane tail flag (no divergent duplicate paths).
  const bool right = x >= mi;
  // normal: isf(sf(x)) = ppf(cdf(x)) = mo + sd_out (x - mi) / sd_in exactly;
  // the reference's ndtr/ndtri round trip only adds rounding (<= 1e-16 of
  // the result) -- except where its ndtr underflows to 0 (|z| > 37.68), and
  // then isf(0) / ppf(0) are the +-inf support bounds
  // (one square root: sd_out / sd_in = sqrt(v_out / v_in), and the
  // underflow test on zh^2 = (x - mi)^2 / (2 v_in) without either root --
  // the two correctly rounded FP64 roots and the quotient by sd_in were ~50
  // VALU per call; the map moves by rounding only)
  const double dxm = x - mi;
  const double rv_in = recip_fast(v_in);  // v_in >= 0.25: normal
  const double zh2 = dxm * dxm * rv_in * 0.5;  // the erfc argument of ndtr, squared
  const bool under = zh2 > kMaxLog;
  double qn;
  if (dxm != dxm || rv_in != rv_in)
    qn = NAN;
  else if (right && dxm > 0.0 && under)
    qn = INFINITY;
  else if (!right && dxm < 0.0 && under)
    qn = -INFINITY;
  else
    qn = dxm * sqrt(v_out * rv_in) + mo;
  // gamma(a, scale r): sf = Q(a, x/r), cdf = P(a, x/r); isf / ppf invert the
  // same tail; x/r <= 0 is the support bound (sf 1, cdf 0)
  const double xs = x * rr_in;
  H3D_SEC_END(1, t_setup);
  double tg;
  if (xs <= 0.0) {
    tg = right ? 1.0 : 0.0;
  } else {
    double P, Q, fac;
    H3D_SEC_BEGIN(t_lg);
    const double lga_in = lgam_q2q(a_in, tab);
    H3D_SEC_END(2, t_lg);
    igam_pq(a_in, xs, lga_in, &P, &Q, &fac, right ? 1 : 0, tab, 3);
    tg = right ? Q : P;
  }
  double qg;
  if (tg != tg) {
    qg = NAN;
  } else if (tg == 0.0) {
    qg = right ? INFINITY : 0.0;
  } else if (tg == 1.0) {
    qg = right ? 0.0 : INFINITY;
  } else {
    // initial guess: carry x through the Wilson-Hilferty cube-root normal
    // approximation of gamma(a_in) into gamma(a_out) -- the approximation
    // errors of the two shapes largely cancel, so Halley usually needs one
    // step; DiDonato-Morris below shape 1, where Wilson-Hilferty is poor
    double guess = -1.0;
    H3D_SEC_BEGIN(t_wh);
    if (a_in >= 1.0 && a_out >= 1.0) {
      const double m_in = 1.0 - recip_fast(9.0 * a_in);
      const double m_out = 1.0 - recip_fast(9.0 * a_out);
#if defined(__HIP_DEVICE_COMPILE__)
      // single precision on gfx950 (v_log_f32 / v_exp_f32 / v_rsq_f32): the
      // guess carries the approximation's own ~1e-4 error, 1e-7 more is
      // nothing to Halley; the FP64 cbrt and sqrts were ~60 VALU
      const float zz = (cbrtf((float)div_fast(xs, a_in)) - (float)m_in) *
                       sqrtf((float)(9.0 * a_in));
      const double y = m_out + (double)(zz * rsqrtf((float)(9.0 * a_out)));
#else
      const double zz = (cbrt(div_fast(xs, a_in)) - m_in) * sqrt(9.0 * a_in);
      const double y = m_out + div_fast(zz, sqrt(9.0 * a_out));
#endif
      if (y > 0.0) guess = a_out * y * y * y;
    }
    H3D_SEC_END(5, t_wh);
    H3D_SEC_BEGIN(t_lgo);
    const double lga = (lga_out == lga_out) ? lga_out : lgam_cached(a_out, cache, tab);
    H3D_SEC_END(6, t_lgo);
    H3D_SEC_BEGIN(t_inv);
    qg = igam_inv(a_out, tg, right, lga, guess, tab) * r_out;
    H3D_SEC_END(7, t_inv);
  }
  double pc = (qn + qg) / 2;
  if (!(pc >= 0.0)) pc = 0.0;
  return pc;
}

// equalize for one pixel (scaled_nb.py:186-214) with a scalar dispersion;
// x, f: the condition's n replicates (compacted, in design order).
// Forced inline: k_disp_work<8>'s >= 8-replicate branch calls it, and when
// the inliner left it out of line (round 5, after the prefactor's log1pmx
// shrank) cfg4's equalize -- which never takes that branch -- went 52 -> 67
// ms per step (r05ao).
template <int M>
H3D_HD_INLINE int equalize_pixel(const double* x, const double* f, int n, double alpha,
                          double* out, const LogTab* tab = kLogTab) {
  double lf[M], as[M];
#pragma unroll
  for (int k = 0; k < M; ++k) {
    lf[k] = (k < n) ? log_fast_checked(f[k], tab) : 0.0;
    as[k] = alpha;
  }
  // gmean(f, pseudocount=0, axis=1) = exp(nanmean(log f)) - 0
  const double f_mean = exp_fast(np_sum<M>(lf, n) / n) - 0.0;
  int st = 0;
  const double mu = fit_mu<M>(x, f, as, n, ~0u, &st, tab);
  double mu_out = mu * f_mean;
  LgamCache cache;
#pragma unroll
  for (int k = 0; k < M; ++k)
    if (k < n) {
      double mu_in = mu * f[k];
      out[k] = q2q(x[k], &mu_in, &mu_out, alpha, &cache, tab);
    }
  return st;
}

// NB log pmf, mean/dispersion parameterisation (scaled_nb.py:12-33).
H3D_HD double logpmf(double k, double m, double phi) {
  const double r = 1.0 / phi;
  return lgam(r + k) - lgam(k + 1) - lgam(r) + r * log(r) - r * log(r + m) +
         k * log(m) - k * log(r + m);
}

// Per-pixel LRT (lrt.py:7-50). a[k] = disp_wide[k] = disp[cond[k]]; CM is a
// compile-time bound on the number of conditions C.
template <int M, int CM, typename TX>
H3D_HD int lrt_pixel(const TX* x, const double* f, const double* a,
                     const int* cond, int R, int C, bool refit, double* p,
                     double* llr, double* mu0, double* mu1,
                     const LogTab* tab = kLogTab) {
  int st = 0;
  // fit 0 is the null (every replicate), fit t = c + 1 condition c's
  // replicates: ONE runtime loop, so fit_mu is inlined once rather than CM + 1
  // times (code size and register pressure of the wide-R instantiations)
#pragma unroll 1
  for (int t = 0; t <= C; ++t) {
    unsigned mask = 0u;
#pragma unroll
    for (int k = 0; k < M; ++k)
      if (k < R && (t == 0 || cond[k] == t - 1)) mask |= (1u << k);
    double mu;
    if (refit) {
      mu = fit_mu<M>(x, f, a, R, mask, &st);
    } else {
      // np.mean(raw / f) over the fit's replicates (lrt.py:36-40)
      int cnt = 0;
#pragma unroll
      for (int k = 0; k < M; ++k) cnt += (k < R && ((mask >> k) & 1u)) ? 1 : 0;
      NpSumStream q(cnt);
      int j = 0;
#pragma unroll
      for (int k = 0; k < M; ++k)
        if (k < R && ((mask >> k) & 1u)) q.add_dyn(j++, (double)x[k] / f[k]);
      mu = q.sum() / cnt;
    }
    if (t == 0) *mu0 = mu;
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c == t - 1) mu1[c] = mu;
  }
  // llr = sum(null logpmf row) - sum(alt logpmf row) (lrt.py:42-48) per
  // replicate k, with m0 = mu0 f_k, m1 = mu1[c(k)] f_k, r = 1 / disp_k
  // (scaled_nb.py:31-33):
  //   gammaln(r + x) - gammaln(x + 1) - gammaln(r) + r log r  cancels,
  //   x log m0 - x log m1 = x log(mu0 / mu1)                (f_k cancels),
  //   -(r + x) log(r + m0) + (r + x) log(r + m1) = -(r + x) log((r + m0) / (r + m1)),
  // so one log per replicate and one per condition instead of four per
  // replicate -- and without the cancellation of two O(1e3) row sums that
  // leaves the reference's llr ~1e-13 of noise (the rows' rounding; the
  // p-values move by that only).
  double lq[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c)
    lq[c] = (c < C) ? log_fast_checked(div_fast(*mu0, mu1[c]), tab) : 0.0;
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < M; ++k) {
    if (k < R) {
      double m1 = 0.0, l = 0.0;
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c == cond[k]) {
          m1 = mu1[c];
          l = lq[c];
        }
      const double xk = (double)x[k];
      const double r = 1.0 / a[k];
      const double lr = log_fast_checked(div_fast(r + *mu0 * f[k], r + m1 * f[k]), tab);
      acc += xk * l - (r + xk) * lr;
    }
  }
  *llr = acc;
  if constexpr (CM == 2) {
    // C <= 2: chi2 with df = C - 1 <= 1 -- chi2_sf's closed form for df = 1
    // (erfc) and its df = 0 value (igamc(0, .) = 0 above the support bound),
    // so the general incomplete-gamma code (and its registers) is not part of
    // the two-condition kernels
    const double x2 = -2 * acc;
    *p = (x2 != x2) ? NAN : (x2 <= 0.0) ? 1.0 : (C == 2) ? erfc(sqrt(x2 / 2.0)) : 0.0;
  } else {
    *p = chi2_sf((double)(C - 1), -2 * *llr);
  }
  return st;
}

// ---- cml negative log likelihood (dispersion.py:67-70) -------------------

struct NllConst {
  double r, nr, lg_nr, n_lg_r;
};

H3D_HD NllConst nll_const(double delta, int n) {
  NllConst k;
  k.r = 1. / delta - 1;
  k.nr = n * k.r;
  k.lg_nr = lgam(k.nr);
  k.n_lg_r = n * lgam(k.r);
  return k;
}

// one pixel's term sum_k gammaln(d_k + r) + gammaln(n r) - gammaln(z + n r)
// - n gammaln(r); nll(delta) = -(sum over pixels). The per-pixel gammaln
// terms use lgam_nll (absolute error ~1e-15, far below the rounding of the
// segment sum), the per-segment constants cephes lgam.
//
// The shift products of the R_c + 1 lgammas are folded into one logarithm
// per 8 replicates (lgam_nll_parts): ln(prod P_j / P_z) -- the products stay
// far inside the double range (P < 15^10 per factor, >= ~1e-2) -- which
// halves the transcendental work of the NLL passes. Arguments: d_j + r >=
// 1/101 - ... > 0 (r = 1/delta - 1 >= 1/0.99 - 1, pseudodata >= 0).
// nll_pixel where every lgamma argument is >= 20 (r = 1/delta - 1 >= 20,
// pseudodata >= 0, z + n r >= 2 r): no shift products, the 5-term Stirling
// series (lgam_nll_large). The Brent kernels take it for the evaluations
// whose r is that large -- the searches' trial points near the optimum at
// the usual dispersions ~0.01..0.05 -- with a branch that is uniform across
// the segment.
template <int M>
H3D_HD double nll_pixel_large(const double* d, int n, const NllConst& k,
                              const LogTab* tab = kLogTab) {
  double lg[M];
#pragma unroll
  for (int j = 0; j < M; ++j) lg[j] = (j < n) ? lgam_nll_large(d[j] + k.r, tab) : 0.0;
  const double z = np_sum<M>(d, n);
  const double lz = lgam_nll_large(z + k.nr, tab);
  return np_sum<M>(lg, n) + k.lg_nr - lz - k.n_lg_r;
}

constexpr double kNllLargeR = 20.0;

// nll_pixel where every lgamma argument is >= 10 (r >= 10): nll_pixel's
// terms without its shift products (all 1 there, so its ln of their product
// is 0) -- the Brent kernels take it for 10 <= r < kNllLargeR, the usual
// optimum region of the searches
template <int M>
H3D_HD double nll_pixel_mid(const double* d, int n, const NllConst& k,
                            const LogTab* tab = kLogTab) {
  double lg[M];
#pragma unroll
  for (int j = 0; j < M; ++j) lg[j] = (j < n) ? lgam_nll_mid(d[j] + k.r, tab) : 0.0;
  const double z = np_sum<M>(d, n);
  const double lz = lgam_nll_mid(z + k.nr, tab);
  return np_sum<M>(lg, n) + k.lg_nr - lz - k.n_lg_r;
}
constexpr double kNllMidR = 10.0;

template <int M>
H3D_HD double nll_pixel(const double* d, int n, const NllConst& k,
                        const LogTab* tab = kLogTab) {
  double lg[M];
  double lnp = 0.0, prod = 1.0;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    double pj = 1.0;
    lg[j] = (j < n) ? lgam_nll_parts(d[j] + k.r, &pj, tab) : 0.0;
    prod *= pj;
    if ((j & 7) == 7 && j + 1 < M) {  // keep 8 factors per logarithm
      lnp += log_fast(prod, tab);
      prod = 1.0;
    }
  }
  const double z = np_sum<M>(d, n);
  double pz = 1.0;
  const double lz = lgam_nll_parts(z + k.nr, &pz, tab);
  lnp += log_fast(prod * recip_nll(pz), tab);
  return np_sum<M>(lg, n) - lnp + k.lg_nr - lz - k.n_lg_r;
}

// ---- qcml + bounded Brent as a resumable state machine --------------------
// qcml (dispersion.py:10-43): disp = 0.01; repeat { equalize; cml } until
// |disp - new| <= 1e-4 (``it`` is never incremented in the reference; a
// 1000-iteration guard raises instead of spinning).
// cml (dispersion.py:46-80): minimize_scalar(nll, bounds=(1e-4, 100/101),
// method='bounded') = scipy 1.7.1 _minimize_scalar_bounded
// (optimize.py:1982-2125, xatol=1e-5, maxiter=500), restated op for op.
// Every NLL evaluation is one data pass; seg_step consumes its result.

constexpr int kEqualize = 0;  // next pass: equalize at disp, then NLL at x0
constexpr int kNll = 1;       // next pass: NLL at x
constexpr int kDone = 2;

constexpr double kBrentA = 1e-4;
constexpr double kBrentB = 100. / (100 + 1);
constexpr double kXatol = 1e-5;
constexpr int kMaxFun = 500;
constexpr double kQcmlTol = 1e-4;  // qcml's default tol (dispersion.py:10)

struct SegState {
  int phase;
  int flags;
  int num;
  int qiter;
  int evals;  // NLL evaluations over every Brent search of the segment
  int last_evals;  // ... of its latest search (k_brent's queue order)
  double disp;    // current qcml dispersion (used by the equalize pass)
  double x;       // delta at which the next NLL is evaluated
  double result;  // final qcml dispersion (NaN for an empty segment)
  NllConst k;     // nll constants at x for n = replicates of the condition
  double a, b, xf, fx, nfc, fnfc, fulc, ffulc, e, rat, xm, tol1, tol2, fu;
  double tol;     // qcml's convergence tolerance on |disp - new disp|
};

H3D_HD double brent_sqrt_eps() { return sqrt(2.2e-16); }
H3D_HD double brent_golden() { return 0.5 * (3.0 - sqrt(5.0)); }
H3D_HD double brent_x0() {
  return kBrentA + brent_golden() * (kBrentB - kBrentA);
}

H3D_HD void seg_init(SegState* s, long long n_px, int n_reps, double tol = kQcmlTol) {
  s->tol = tol;
  s->flags = 0;
  s->num = 0;
  s->qiter = 0;
  s->evals = 0;
  s->last_evals = 0;
  s->disp = 0.01;
  s->x = brent_x0();
  s->k = nll_const(s->x, n_reps);
  s->result = NAN;
  s->phase = (n_px > 0) ? kEqualize : kDone;
}

H3D_HD double sgn(double v) { return (double)((v > 0) - (v < 0)); }

// Advance with the NLL pixel-term total evaluated at s->x.
H3D_HD void seg_step(SegState* s, double total, int n_reps) {
#if defined(__clang__)
  // scipy's Brent arithmetic op for op (no fused multiply-adds): the trial
  // points follow the reference bit for bit given the same NLL values
#pragma clang fp contract(off)
#endif
  const double sqrt_eps = brent_sqrt_eps();
  const double golden_mean = brent_golden();
  const double fval = -total;
  bool finished = false;
  s->evals += 1;
  if (s->phase == kEqualize) {
    s->a = kBrentA;
    s->b = kBrentB;
    s->fulc = s->a + golden_mean * (s->b - s->a);
    s->nfc = s->xf = s->fulc;
    s->rat = s->e = 0.0;
    s->fx = fval;
    s->num = 1;
    s->fu = INFINITY;
    s->ffulc = s->fnfc = s->fx;
    s->xm = 0.5 * (s->a + s->b);
    s->tol1 = sqrt_eps * fabs(s->xf) + kXatol / 3.0;
    s->tol2 = 2.0 * s->tol1;
  } else {
    const double x = s->x, fu = fval;
    s->fu = fu;
    s->num += 1;
    if (fu <= s->fx) {
      if (x >= s->xf)
        s->a = s->xf;
      else
        s->b = s->xf;
      s->fulc = s->nfc;
      s->ffulc = s->fnfc;
      s->nfc = s->xf;
      s->fnfc = s->fx;
      s->xf = x;
      s->fx = fu;
    } else {
      if (x < s->xf)
        s->a = x;
      else
        s->b = x;
      if ((fu <= s->fnfc) || (s->nfc == s->xf)) {
        s->fulc = s->nfc;
        s->ffulc = s->fnfc;
        s->nfc = x;
        s->fnfc = fu;
      } else if ((fu <= s->ffulc) || (s->fulc == s->xf) ||
                 (s->fulc == s->nfc)) {
        s->fulc = x;
        s->ffulc = fu;
      }
    }
    s->xm = 0.5 * (s->a + s->b);
    s->tol1 = sqrt_eps * fabs(s->xf) + kXatol / 3.0;
    s->tol2 = 2.0 * s->tol1;
    if (s->num >= kMaxFun) {
      s->flags |= kFlagBrentFail;  // scipy flag 1 -> res.success False
      finished = true;
    }
  }
  if (!finished && (fabs(s->xf - s->xm) > (s->tol2 - 0.5 * (s->b - s->a)))) {
    // next trial point (loop body up to ``fu = func(x)``)
    int golden = 1;
    double x = s->xf;
    if (fabs(s->e) > s->tol1) {
      golden = 0;
      double r = (s->xf - s->nfc) * (s->fx - s->ffulc);
      double q = (s->xf - s->fulc) * (s->fx - s->fnfc);
      double p = (s->xf - s->fulc) * q - (s->xf - s->nfc) * r;
      q = 2.0 * (q - r);
      if (q > 0.0) p = -p;
      q = fabs(q);
      r = s->e;
      s->e = s->rat;
      if ((fabs(p) < fabs(0.5 * q * r)) && (p > q * (s->a - s->xf)) &&
          (p < q * (s->b - s->xf))) {
        s->rat = (p + 0.0) / q;
        x = s->xf + s->rat;
        if (((x - s->a) < s->tol2) || ((s->b - x) < s->tol2)) {
          const double si = sgn(s->xm - s->xf) + ((s->xm - s->xf) == 0);
          s->rat = s->tol1 * si;
        }
      } else {
        golden = 1;
      }
    }
    if (golden) {
      if (s->xf >= s->xm)
        s->e = s->a - s->xf;
      else
        s->e = s->b - s->xf;
      s->rat = golden_mean * s->e;
    }
    const double si = sgn(s->rat) + (s->rat == 0);
    s->x = s->xf + si * fmax(fabs(s->rat), s->tol1);
    s->k = nll_const(s->x, n_reps);
    s->phase = kNll;
    return;
  }
  // Brent finished: qcml update
  if (s->xf != s->xf || s->fx != s->fx || s->fu != s->fu)
    s->flags |= kFlagBrentFail;
  const double new_disp = s->xf / (1 - s->xf);
  const double delta = fabs(s->disp - new_disp);
  s->disp = new_disp;
  s->qiter += 1;
  if (delta > s->tol && s->qiter < 1000 && !(s->flags & kFlagBrentFail)) {
    s->phase = kEqualize;
    s->x = brent_x0();
    s->k = nll_const(s->x, n_reps);
  } else {
    if (s->qiter >= 1000 && delta > s->tol) s->flags |= kFlagQcmlGuard;
    s->phase = kDone;
    s->result = s->disp;
  }
}

}  // namespace h3d
