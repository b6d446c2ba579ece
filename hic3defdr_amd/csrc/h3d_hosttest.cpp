// Host build of the device numerics, for CPU unit tests ONLY.
//
// The same headers the gfx950 kernels include (h3d_special.h, h3d_model.h)
// compiled with g++ and exported over a flat C ABI so tests/ can check them
// against scipy / the oracle without a GPU. The product never loads this
// library (hic3defdr_amd loads libh3d.so and fails loudly without it).
#include <cstdint>
#include <vector>

#include "h3d_model.h"
#include "h3d_special.h"

namespace {
constexpr int M = h3d::kMaxReps;
}

extern "C" {

#define H3DT_UNARY(name, fn)                                   \
  void h3dt_##name(int64_t n, const double* x, double* out) { \
    for (int64_t i = 0; i < n; ++i) out[i] = h3d::fn(x[i]);   \
  }
#define H3DT_BINARY(name, fn)                                     \
  void h3dt_##name(int64_t n, const double* a, const double* x,  \
                   double* out) {                                 \
    for (int64_t i = 0; i < n; ++i) out[i] = h3d::fn(a[i], x[i]); \
  }

H3DT_UNARY(lgam, lgam)
H3DT_UNARY(lgam_nll, lgam_nll)
H3DT_UNARY(log_fast, log_fast)
H3DT_UNARY(ndtr, ndtr)
H3DT_UNARY(ndtri, ndtri)
H3DT_UNARY(log1pmx, log1pmx)
H3DT_UNARY(lgam1p, lgam1p)
H3DT_BINARY(igam, igam)
H3DT_BINARY(igamc, igamc)
H3DT_BINARY(igami, igami)
H3DT_BINARY(igamci, igamci)
H3DT_BINARY(chi2_sf, chi2_sf)

// fit_mu_hat per pixel: x (n, r) int32, b (n, r), alpha (n, r) -> mu (n)
int h3dt_fit_mu(int64_t n, int r, const int32_t* x, const double* b,
                const double* alpha, double* mu) {
  int bad = 0;
  for (int64_t i = 0; i < n; ++i) {
    double xs[M], bs[M], as[M];
    for (int k = 0; k < r; ++k) {
      xs[k] = x[i * r + k];
      bs[k] = b[i * r + k];
      as[k] = alpha[i * r + k];
    }
    int st = 0;
    mu[i] = h3d::fit_mu<M>(xs, bs, as, r, ~0u, &st);
    bad |= st;
  }
  return bad;
}

// q2qnbinom elementwise (single replicate, no clamp carry)
void h3dt_q2q(int64_t n, const double* x, const double* mu_in,
              const double* mu_out, const double* alpha, double* out) {
  for (int64_t i = 0; i < n; ++i) {
    double mi = mu_in[i], mo = mu_out[i];
    out[i] = h3d::q2q(x[i], &mi, &mo, alpha[i]);
  }
}

// equalize one segment: data (n, r) int32, f (n, r), scalar alpha
int h3dt_equalize(int64_t n, int r, const int32_t* x, const double* f,
                  double alpha, double* out) {
  int bad = 0;
  for (int64_t i = 0; i < n; ++i) {
    double xs[M], fs[M], ps[M];
    for (int k = 0; k < r; ++k) {
      xs[k] = x[i * r + k];
      fs[k] = f[i * r + k];
    }
    bad |= h3d::equalize_pixel<M>(xs, fs, r, alpha, ps);
    for (int k = 0; k < r; ++k) out[i * r + k] = ps[k];
  }
  return bad;
}

// per-pixel NLL terms at delta by the general / mid (r >= 10) / large
// (r >= 20) forms of the Brent kernels (mode 0 / 1 / 2)
int h3dt_nll_terms(int64_t n, int r, const double* pseudo, double delta, int mode,
                   double* out) {
  if (r < 1 || r > M || mode < 0 || mode > 2) return -1;
  const h3d::NllConst kc = h3d::nll_const(delta, r);
  for (int64_t i = 0; i < n; ++i) {
    double ps[M];
    for (int k = 0; k < M; ++k) ps[k] = k < r ? pseudo[i * r + k] : 0.0;
    out[i] = mode == 2   ? h3d::nll_pixel_large<M>(ps, r, kc)
             : mode == 1 ? h3d::nll_pixel_mid<M>(ps, r, kc)
                         : h3d::nll_pixel<M>(ps, r, kc);
  }
  return 0;
}

// per-pixel LRT with per-replicate dispersions (lrt.py:7-50)
int h3dt_lrt(int64_t n, int R, int C, const int32_t* raw, const double* f,
             const double* disp_wide, const int32_t* cond_of_rep, int refit,
             double* p, double* llr, double* mu0, double* mu1) {
  int bad = 0;
  int cond[M];
  for (int k = 0; k < R; ++k) cond[k] = cond_of_rep[k];
  for (int64_t i = 0; i < n; ++i) {
    double xs[M], fs[M], as[M];
    for (int k = 0; k < R; ++k) {
      xs[k] = raw[i * R + k];
      fs[k] = f[i * R + k];
      as[k] = disp_wide[i * R + k];
    }
    double m1[h3d::kMaxConds];
    bad |= h3d::lrt_pixel<M, h3d::kMaxConds>(xs, fs, as, cond, R, C,
                                             refit != 0, &p[i], &llr[i],
                                             &mu0[i], m1);
    for (int c = 0; c < C; ++c) mu1[i * C + c] = m1[c];
  }
  return bad;
}

// full qcml on one segment, driven by the same state machine as the kernels
double h3dt_qcml(int64_t n, int r, const int32_t* x, const double* f,
                 int* status) {
  std::vector<double> pseudo(n * r);
  h3d::SegState st;
  h3d::seg_init(&st, n, r);
  int guard = 0;
  while (st.phase != h3d::kDone && guard++ < 100000) {
    double total = 0.0;
    if (st.phase == h3d::kEqualize) {
      for (int64_t i = 0; i < n; ++i) {
        double xs[M], fs[M];
        for (int k = 0; k < r; ++k) {
          xs[k] = x[i * r + k];
          fs[k] = f[i * r + k];
        }
        st.flags |= h3d::equalize_pixel<M>(xs, fs, r, st.disp, &pseudo[i * r]);
      }
    }
    for (int64_t i = 0; i < n; ++i)
      total += h3d::nll_pixel<M>(&pseudo[i * r], r, st.k);
    h3d::seg_step(&st, total, r);
  }
  *status = st.flags;
  return st.result;
}

// Host emulation of the multi-rank estimate_disp driver (h3d_disp_per_dist_dev
// with an all-reduce hook): this rank's pixels, stable-ordered by distance;
// per data pass every active segment's local NLL total, summed across ranks
// by `reduce`, then the shared qcml/Brent state machines advance. Used by the
// gloo world_size-2 tests to check the sharded algorithm on CPU.
typedef int (*h3dt_reduce_fn)(double* buf, int64_t count, void* user);

int h3dt_disp_rounds(int64_t n, int R, int C, const int32_t* raw,
                     const double* f, const int32_t* dist,
                     const int32_t* cond_of_rep, int D, h3dt_reduce_fn reduce,
                     void* user, double* out, int32_t* flags_out) {
  const int S = D * C;
  std::vector<int> nrep(C, 0), rep_idx(C * M, 0);
  for (int r = 0; r < R; ++r) rep_idx[cond_of_rep[r] * M + nrep[cond_of_rep[r]]++] = r;
  std::vector<std::vector<int64_t>> px(D);
  for (int64_t i = 0; i < n; ++i) px[dist[i]].push_back(i);
  std::vector<double> cnt(S, 0.0), tot(S, 0.0);
  for (int d = 0; d < D; ++d)
    for (int c = 0; c < C; ++c) cnt[d * C + c] = (double)px[d].size();
  if (reduce && reduce(cnt.data(), S, user)) return -2;
  std::vector<h3d::SegState> st(S);
  for (int s = 0; s < S; ++s) h3d::seg_init(&st[s], (long long)cnt[s], nrep[s % C]);
  std::vector<double> pd((size_t)n * R, 0.0);
  for (int guard = 0; guard < 200000; ++guard) {
    bool any = false;
    for (int s = 0; s < S; ++s) any |= st[s].phase != h3d::kDone;
    if (!any) break;
    for (int s = 0; s < S; ++s) {
      tot[s] = 0.0;
      if (st[s].phase == h3d::kDone) continue;
      const int d = s / C, c = s % C, nr = nrep[c];
      for (int64_t i : px[d]) {
        double x[M], fv[M], dd[M];
        for (int k = 0; k < nr; ++k) {
          const int r = rep_idx[c * M + k];
          x[k] = raw[i * R + r];
          fv[k] = f[i * R + r];
          dd[k] = pd[i * R + r];
        }
        if (st[s].phase == h3d::kEqualize) {
          st[s].flags |= h3d::equalize_pixel<M>(x, fv, nr, st[s].disp, dd);
          for (int k = 0; k < nr; ++k) pd[i * R + rep_idx[c * M + k]] = dd[k];
        }
        tot[s] += h3d::nll_pixel<M>(dd, nr, st[s].k);
      }
    }
    if (reduce && reduce(tot.data(), S, user)) return -2;
    for (int s = 0; s < S; ++s)
      if (st[s].phase != h3d::kDone) h3d::seg_step(&st[s], tot[s], nrep[s % C]);
  }
  for (int s = 0; s < S; ++s) {
    out[s] = st[s].result;
    if (flags_out) flags_out[s] = st[s].flags;
  }
  return 0;
}

}  // extern "C"
