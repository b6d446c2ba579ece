// Work census of the equalize pass (host build, H3D_INSTRUMENT): runs the
// device numerics on the CPU over one segment-sorted workload and records,
// per pixel-replicate, how much work each special function did. The wave
// divergence estimate (per-64-lane max vs mean) is computed in
// tools/q2q_stats.py. Measurement tool only; never part of the product.
#define H3D_INSTRUMENT 1
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../hic3defdr_amd/csrc/h3d_model.h"

extern "C" {

constexpr int kFields = sizeof(h3d::Stats) / sizeof(long);
int q2qs_fields() { return kFields; }

// raw (n, R) int32, f (n, R), alpha (n) per pixel, reps of the condition in
// rep_idx[0..nr). rec out: (n, nr, kFields) longs.
void q2qs_equalize(int64_t n, int R, const int32_t* raw, const double* f,
                   const double* alpha, int nr, const int32_t* rep_idx,
                   long* rec, double* out) {
  constexpr int M = 8;
  for (int64_t i = 0; i < n; ++i) {
    double x[M], fs[M], as[M], lf[M];
    for (int k = 0; k < M; ++k) {
      const bool on = k < nr;
      x[k] = on ? raw[i * R + rep_idx[k]] : 0.0;
      fs[k] = on ? f[i * R + rep_idx[k]] : 1.0;
      lf[k] = on ? log(fs[k]) : 0.0;
      as[k] = alpha[i];
    }
    h3d::Stats s0;
    memset(&s0, 0, sizeof s0);
    h3d::g_stats = &s0;
    int fl = 0;
    const double f_mean = exp(h3d::np_sum<M>(lf, nr) / nr);
    const double mu = h3d::fit_mu<M>(x, fs, as, nr, ~0u, &fl);
    double mu_out = mu * f_mean;
    h3d::LgamCache cache;
    for (int k = 0; k < nr; ++k) {
      h3d::Stats s;
      memset(&s, 0, sizeof s);
      if (k == 0) s = s0;  // the per-pixel mean fit is charged to slot 0
      h3d::g_stats = &s;
      double mu_in = mu * fs[k];
      const double dk = h3d::q2q(x[k], &mu_in, &mu_out, alpha[i], &cache);
      out[i * nr + k] = dk;
      (void)h3d::lgam(dk + 1.0 / alpha[i]);
      memcpy(rec + (i * nr + k) * kFields, &s, sizeof s);
    }
    h3d::g_stats = nullptr;
  }
}
}

extern "C" {
// Halley probe: for each pixel-replicate of the equalize pass, the relative
// move of 4 unconditional Halley steps from the q2q initial guess, and the
// relative error left after step 1 / step 2 (vs step 4). out: (n, nr, 6).
void q2qs_halley(int64_t n, int R, const int32_t* raw, const double* f,
                 const double* alpha, int nr, const int32_t* rep_idx,
                 double* out) {
  using namespace h3d;
  constexpr int M = 8;
  for (int64_t i = 0; i < n; ++i) {
    double x[M], fs[M], as[M], lf[M];
    for (int k = 0; k < M; ++k) {
      const bool on = k < nr;
      x[k] = on ? raw[i * R + rep_idx[k]] : 0.0;
      fs[k] = on ? f[i * R + rep_idx[k]] : 1.0;
      lf[k] = on ? log(fs[k]) : 0.0;
      as[k] = alpha[i];
    }
    int fl = 0;
    const double f_mean = exp(np_sum<M>(lf, nr) / nr);
    const double mu = fit_mu<M>(x, fs, as, nr, ~0u, &fl);
    double mu_out = mu * f_mean;
    for (int k = 0; k < nr; ++k) {
      double* o = out + (i * nr + k) * 6;
      for (int j = 0; j < 6; ++j) o[j] = NAN;
      double mu_in = mu * fs[k];
      const double al = alpha[i];
      if (!((mu_in >= 0.25) && (mu_out >= 0.25))) mu_in = mu_out = 0.25;
      const double r_in = 1 + al * mu_in, r_out = 1 + al * mu_out;
      const double a_in = mu_in / r_in, a_out = mu_out / r_out;
      const bool right0 = x[k] >= mu_in;
      const double xs = x[k] / r_in;
      if (!(xs > 0.0)) continue;
      double P, Q, fac;
      igam_pq(a_in, xs, lgam(a_in), &P, &Q, &fac);
      double t = right0 ? Q : P;
      if (!(t > 0.0 && t < 1.0)) continue;
      bool upper = right0;
      double guess = -1.0;
      if (a_in >= 1.0 && a_out >= 1.0) {
        const double m_in = 1.0 - 1.0 / (9.0 * a_in);
        const double m_out = 1.0 - 1.0 / (9.0 * a_out);
        const double zz = (cbrt(xs / a_in) - m_in) * sqrt(9.0 * a_in);
        const double y = m_out + zz / sqrt(9.0 * a_out);
        if (y > 0.0) guess = a_out * y * y * y;
      }
      const double lga = lgam(a_out);
      if (t > 0.9) {
        t = 1.0 - t;
        upper = !upper;
      }
      double xx = (guess > 0.0) ? guess
                  : upper ? find_inverse_gamma(a_out, 1.0 - t, t, lga)
                          : find_inverse_gamma(a_out, t, 1.0 - t, lga);
      double xs_[5];
      xs_[0] = xx;
      for (int s = 0; s < 4; ++s) {
        igam_pq(a_out, xx, lga, &P, &Q, &fac);
        if (fac == 0.0) break;
        const double f_fp = upper ? (Q - t) * xx / (-fac) : (P - t) * xx / fac;
        const double fpp_fp = -1.0 + (a_out - 1) / xx;
        double xn = xx - f_fp / (1.0 - 0.5 * f_fp * fpp_fp);
        if (!(xn > 0.0)) xn = 0.5 * xx;
        xx = xn;
        xs_[s + 1] = xx;
        if (s < 3) o[s] = fabs(xs_[s + 1] - xs_[s]) / xx;
      }
      o[3] = fabs(xs_[1] - xs_[4]) / xs_[4];
      o[4] = fabs(xs_[2] - xs_[4]) / xs_[4];
      o[5] = a_out;
    }
  }
}
}

extern "C" {
// fit_mu trace of one pixel (printf), for slow-convergence diagnosis
void q2qs_fit_trace(int n, const double* x, const double* b, double a) {
  double init = 0.0;
  for (int k = 0; k < n; ++k) init += x[k] / b[k];
  double th = log(init / n), lo = -INFINITY, hi = INFINITY;
  for (int it = 0; it < 40; ++it) {
    const double mu = exp(th);
    double g = 0.0, gp = 0.0;
    for (int k = 0; k < n; ++k) {
      const double mb = mu * b[k];
      const double den = 1.0 / (1.0 + a * mb);
      g += (x[k] - mb) * den;
      gp -= mb * (1.0 + a * x[k]) * den * den;
    }
    if (g > 0.0) lo = th; else if (g < 0.0) hi = th; else break;
    double tn = th - g / gp;
    const bool newton = tn > lo && tn < hi;
    if (!newton) tn = std::isinf(lo) ? hi - 2.0 : std::isinf(hi) ? lo + 2.0 : 0.5 * (lo + hi);
    printf("it %2d th %.17g g %.3e gp %.3e step %.3e %s\n", it, th, g, gp,
           tn - th, newton ? "" : "BISECT");
    const double step = fabs(tn - th);
    th = tn;
    if (step <= 1e-15 * fmax(1.0, fabs(th))) break;
    if (!std::isinf(lo) && !std::isinf(hi) && (hi - lo) <= 4e-16 * fmax(1.0, fabs(th))) break;
  }
  fflush(stdout);
}
}

extern "C" {
// per igam_pq call log for one equalize sweep: (a, x, iterations, path)
// path 0 = CF, 1 = small-x upper series, 2 = power series. Returns count.
int64_t q2qs_pq_log(int64_t n, int R, const int32_t* raw, const double* f,
                    const double* alpha, int nr, const int32_t* rep_idx,
                    double* out /* (cap, 4) */, int64_t cap) {
  using namespace h3d;
  constexpr int M = 8;
  int64_t cnt = 0;
  for (int64_t i = 0; i < n && cnt + 64 < cap; ++i) {
    double x[M], fs[M], as[M], lf[M];
    for (int k = 0; k < M; ++k) {
      const bool on = k < nr;
      x[k] = on ? raw[i * R + rep_idx[k]] : 0.0;
      fs[k] = on ? f[i * R + rep_idx[k]] : 1.0;
      lf[k] = on ? log(fs[k]) : 0.0;
      as[k] = alpha[i];
    }
    if (!(alpha[i] > 0)) continue;
    int fl = 0;
    const double f_mean = exp(np_sum<M>(lf, nr) / nr);
    const double mu = fit_mu<M>(x, fs, as, nr, ~0u, &fl);
    double mu_out = mu * f_mean;
    LgamCache cache;
    for (int k = 0; k < nr; ++k) {
      double mu_in = mu * fs[k];
      Stats st;
      memset(&st, 0, sizeof st);
      g_stats = &st;
      g_pq_log = out + cnt * 4;
      g_pq_cap = cap - cnt;
      g_pq_n = 0;
      (void)q2q(x[k], &mu_in, &mu_out, alpha[i], &cache);
      cnt += g_pq_n;
      g_pq_log = nullptr;
      g_stats = nullptr;
    }
  }
  return cnt;
}
}

extern "C" {
// Per pixel and replicate slot, in the kernel's visiting order (upper tail
// first): the igam_pq calls of q2qnbinom -- count, then (iterations, path)
// of up to 5 calls; plus fit_mu iterations per pixel. rec: (n, nr, 11),
// fit: (n).
void q2qs_wave_log(int64_t n, int R, const int32_t* raw, const double* f,
                   const double* alpha, int nr, const int32_t* rep_idx,
                   double* rec, double* fit) {
  using namespace h3d;
  constexpr int M = 8;
  double buf[4 * 16];
  for (int64_t i = 0; i < n; ++i) {
    double x[M], fs[M], as[M], lf[M];
    for (int k = 0; k < M; ++k) {
      const bool on = k < nr;
      x[k] = on ? raw[i * R + rep_idx[k]] : 0.0;
      fs[k] = on ? f[i * R + rep_idx[k]] : 1.0;
      lf[k] = on ? log(fs[k]) : 0.0;
      as[k] = alpha[i];
    }
    for (int j = 0; j < nr * 11; ++j) rec[i * nr * 11 + j] = 0.0;
    fit[i] = 0.0;
    if (!(alpha[i] > 0)) continue;
    Stats st;
    memset(&st, 0, sizeof st);
    g_stats = &st;
    int fl = 0;
    const double f_mean = exp(np_sum<M>(lf, nr) / nr);
    const double mu = fit_mu<M>(x, fs, as, nr, ~0u, &fl);
    fit[i] = (double)st.fit_it;
    const double mu_out0 = mu * f_mean;
    int fc = nr;
    unsigned up = 0u, lo = 0u;
    for (int k = nr - 1; k >= 0; --k) {
      const double mi = mu * fs[k];
      if (!(mi >= 0.25 && mu_out0 >= 0.25)) fc = k;
      if (x[k] >= mi) up |= 1u << k; else lo |= 1u << k;
    }
    LgamCache cache;
    for (int j = 0; j < nr; ++j) {
      int k;
      if (up) { k = __builtin_ctz(up); up &= up - 1u; }
      else { k = __builtin_ctz(lo); lo &= lo - 1u; }
      double mu_in = mu * fs[k];
      double mu_out = (k > fc) ? 0.25 : mu_out0;
      memset(&st, 0, sizeof st);
      g_pq_log = buf;
      g_pq_cap = 16;
      g_pq_n = 0;
      (void)q2q(x[k], &mu_in, &mu_out, alpha[i], &cache);
      double* o = rec + (i * nr + j) * 11;
      o[0] = (double)g_pq_n;
      for (int c = 0; c < 5 && c < g_pq_n; ++c) {
        o[1 + 2 * c] = buf[4 * c + 2];
        o[2 + 2 * c] = buf[4 * c + 3];
      }
      g_pq_log = nullptr;
    }
    g_stats = nullptr;
  }
}
}
