// gfx950 build of the device numerics, for GPU unit tests ONLY.
//
// libh3d_selftest.so exports the same flat C ABI as the host build
// (h3d_hosttest.cpp: h3dt_*), but every entry point runs the device code of
// h3d_special.h / h3d_model.h in a gfx950 kernel -- OCML exp/log, the
// contracted NLL lgamma, device-side branch structure -- so tests/ can hold
// the kernels' numerics to the reference's unit goldens at the same
// tolerances as the host build (tests/test_special_host.py, parametrized
// over both libraries). The product never loads this library.
//
// Host pointers in, host pointers out: each call stages its arrays through
// device buffers (synchronous; sizes are unit-test sized).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "h3d_model.h"
#include "h3d_special.h"

namespace {

constexpr int M = h3d::kMaxReps;
constexpr int kBlock = 256;

enum Op {
  kLgam, kLgamNll, kLogFast, kNdtr, kNdtri, kLog1pmx, kLgam1p,
  kIgam, kIgamc, kIgami, kIgamci, kChi2Sf
};

template <int OP>
__device__ double unary_op(double x) {
  if constexpr (OP == kLgam) return h3d::lgam(x);
  else if constexpr (OP == kLgamNll) return h3d::lgam_nll(x);
  else if constexpr (OP == kLogFast) return h3d::log_fast(x);
  else if constexpr (OP == kNdtr) return h3d::ndtr(x);
  else if constexpr (OP == kNdtri) return h3d::ndtri(x);
  else if constexpr (OP == kLog1pmx) return h3d::log1pmx(x);
  else return h3d::lgam1p(x);
}

template <int OP>
__device__ double binary_op(double a, double x) {
  if constexpr (OP == kIgam) return h3d::igam(a, x);
  else if constexpr (OP == kIgamc) return h3d::igamc(a, x);
  else if constexpr (OP == kIgami) return h3d::igami(a, x);
  else if constexpr (OP == kIgamci) return h3d::igamci(a, x);
  else return h3d::chi2_sf(a, x);
}

template <int OP>
__global__ void k_unary(int64_t n, const double* __restrict__ x,
                        double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = unary_op<OP>(x[i]);
}

template <int OP>
__global__ void k_binary(int64_t n, const double* __restrict__ a,
                         const double* __restrict__ x, double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = binary_op<OP>(a[i], x[i]);
}

__global__ void k_fit_mu(int64_t n, int r, const int32_t* __restrict__ x,
                         const double* __restrict__ b,
                         const double* __restrict__ alpha, double* __restrict__ mu,
                         int* __restrict__ status) {
  int st_all = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double xs[M], bs[M], as[M];
#pragma unroll
    for (int k = 0; k < M; ++k) {
      const bool on = k < r;
      xs[k] = on ? (double)x[i * r + k] : 0.0;
      bs[k] = on ? b[i * r + k] : 1.0;
      as[k] = on ? alpha[i * r + k] : 1.0;
    }
    int st = 0;
    mu[i] = h3d::fit_mu<M>(xs, bs, as, r, ~0u, &st);
    st_all |= st;
  }
  if (st_all) atomicOr(status, st_all);
}

__global__ void k_q2q(int64_t n, const double* __restrict__ x,
                      const double* __restrict__ mu_in,
                      const double* __restrict__ mu_out,
                      const double* __restrict__ alpha, double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double mi = mu_in[i], mo = mu_out[i];
    out[i] = h3d::q2q(x[i], &mi, &mo, alpha[i]);
  }
}

// equalize (scalar alpha) and, when `nll` is set, the per-pixel NLL term at
// the constants `kc` over the pseudodata just produced
__global__ void k_equalize_nll(int64_t n, int r, const int32_t* __restrict__ x,
                               const double* __restrict__ f, double alpha,
                               int do_equalize, double* __restrict__ pseudo,
                               h3d::NllConst kc, double* __restrict__ term,
                               int* __restrict__ status) {
  int st_all = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double ps[M];
    if (do_equalize) {
      double xs[M], fs[M];
#pragma unroll
      for (int k = 0; k < M; ++k) {
        const bool on = k < r;
        xs[k] = on ? (double)x[i * r + k] : 0.0;
        fs[k] = on ? f[i * r + k] : 1.0;
      }
      st_all |= h3d::equalize_pixel<M>(xs, fs, r, alpha, ps);
#pragma unroll
      for (int k = 0; k < M; ++k)
        if (k < r) pseudo[i * r + k] = ps[k];
    } else {
#pragma unroll
      for (int k = 0; k < M; ++k) ps[k] = (k < r) ? pseudo[i * r + k] : 0.0;
    }
    if (term) term[i] = h3d::nll_pixel<M>(ps, r, kc);
  }
  if (st_all) atomicOr(status, st_all);
}

__global__ void k_nll_terms(int64_t n, int r, const double* __restrict__ pseudo,
                            h3d::NllConst kc, int mode, double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double ps[M];
#pragma unroll
    for (int k = 0; k < M; ++k) ps[k] = (k < r) ? pseudo[i * r + k] : 0.0;
    out[i] = mode == 2   ? h3d::nll_pixel_large<M>(ps, r, kc)
             : mode == 1 ? h3d::nll_pixel_mid<M>(ps, r, kc)
                         : h3d::nll_pixel<M>(ps, r, kc);
  }
}

__global__ void k_lrt(int64_t n, int R, int C, const int32_t* __restrict__ raw,
                      const double* __restrict__ f,
                      const double* __restrict__ disp_wide,
                      const int32_t* __restrict__ cond_of_rep, int refit,
                      double* __restrict__ p, double* __restrict__ llr,
                      double* __restrict__ mu0, double* __restrict__ mu1,
                      int* __restrict__ status) {
  int cond[M];
#pragma unroll
  for (int k = 0; k < M; ++k) cond[k] = (k < R) ? cond_of_rep[k] : -1;
  int st_all = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double xs[M], fs[M], as[M];
#pragma unroll
    for (int k = 0; k < M; ++k) {
      const bool on = k < R;
      xs[k] = on ? (double)raw[i * R + k] : 0.0;
      fs[k] = on ? f[i * R + k] : 1.0;
      as[k] = on ? disp_wide[i * R + k] : 1.0;
    }
    double pv, lv, m0, m1[h3d::kMaxConds];
    st_all |= h3d::lrt_pixel<M, h3d::kMaxConds>(xs, fs, as, cond, R, C,
                                                refit != 0, &pv, &lv, &m0, m1);
    p[i] = pv;
    llr[i] = lv;
    mu0[i] = m0;
    for (int c = 0; c < C; ++c) mu1[i * C + c] = m1[c];
  }
  if (st_all) atomicOr(status, st_all);
}

// --- host staging --------------------------------------------------------

bool g_failed = false;

bool ok(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "[h3d_selftest] %s: %s\n", what, hipGetErrorString(e));
    g_failed = true;
    return false;
  }
  return true;
}

// device copy of a host array (freed by the destructor)
template <typename T>
struct Dev {
  T* p = nullptr;
  size_t n = 0;
  Dev(const T* host, size_t count) : n(count) {
    if (!ok(hipMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T)), "hipMalloc"))
      return;
    if (host && count)
      ok(hipMemcpy(p, host, count * sizeof(T), hipMemcpyHostToDevice), "H2D");
    else
      ok(hipMemset(p, 0, std::max<size_t>(count, 1) * sizeof(T)), "memset");
  }
  void to_host(T* host) const {
    if (host && n) ok(hipMemcpy(host, p, n * sizeof(T), hipMemcpyDeviceToHost), "D2H");
  }
  ~Dev() {
    if (p) (void)hipFree(p);
  }
};

int grid_of(int64_t n) {
  int64_t g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  return (int)g;
}

bool sync_ok() {
  return ok(hipGetLastError(), "launch") && ok(hipDeviceSynchronize(), "sync");
}

template <int OP>
void run_unary(int64_t n, const double* x, double* out) {
  Dev<double> dx(x, n), dout(nullptr, n);
  hipLaunchKernelGGL(k_unary<OP>, dim3(grid_of(n)), dim3(kBlock), 0, 0, n, dx.p, dout.p);
  if (sync_ok()) dout.to_host(out);
  if (g_failed)
    for (int64_t i = 0; i < n; ++i) out[i] = NAN;
}

template <int OP>
void run_binary(int64_t n, const double* a, const double* x, double* out) {
  Dev<double> da(a, n), dx(x, n), dout(nullptr, n);
  hipLaunchKernelGGL(k_binary<OP>, dim3(grid_of(n)), dim3(kBlock), 0, 0, n, da.p, dx.p,
                     dout.p);
  if (sync_ok()) dout.to_host(out);
  if (g_failed)
    for (int64_t i = 0; i < n; ++i) out[i] = NAN;
}

}  // namespace

extern "C" {

// 1 when a device is visible and every call so far succeeded
int h3dt_device_ok(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return 0;
  return g_failed ? 0 : 1;
}

#define H3DT_UNARY(name, op) \
  void h3dt_##name(int64_t n, const double* x, double* out) { run_unary<op>(n, x, out); }
#define H3DT_BINARY(name, op)                                               \
  void h3dt_##name(int64_t n, const double* a, const double* x, double* out) { \
    run_binary<op>(n, a, x, out);                                           \
  }

H3DT_UNARY(lgam, kLgam)
H3DT_UNARY(lgam_nll, kLgamNll)
H3DT_UNARY(log_fast, kLogFast)
H3DT_UNARY(ndtr, kNdtr)
H3DT_UNARY(ndtri, kNdtri)
H3DT_UNARY(log1pmx, kLog1pmx)
H3DT_UNARY(lgam1p, kLgam1p)
H3DT_BINARY(igam, kIgam)
H3DT_BINARY(igamc, kIgamc)
H3DT_BINARY(igami, kIgami)
H3DT_BINARY(igamci, kIgamci)
H3DT_BINARY(chi2_sf, kChi2Sf)

int h3dt_fit_mu(int64_t n, int r, const int32_t* x, const double* b,
                const double* alpha, double* mu) {
  if (r < 1 || r > M) return -1;
  Dev<int32_t> dx(x, n * r);
  Dev<double> db(b, n * r), da(alpha, n * r), dmu(nullptr, n);
  Dev<int> dst(nullptr, 1);
  hipLaunchKernelGGL(k_fit_mu, dim3(grid_of(n)), dim3(kBlock), 0, 0, n, r, dx.p, db.p,
                     da.p, dmu.p, dst.p);
  int st = 0;
  if (!sync_ok()) return -2;
  dmu.to_host(mu);
  dst.to_host(&st);
  return g_failed ? -2 : st;
}

void h3dt_q2q(int64_t n, const double* x, const double* mu_in,
              const double* mu_out, const double* alpha, double* out) {
  Dev<double> dx(x, n), di(mu_in, n), dout_(mu_out, n), dal(alpha, n), d(nullptr, n);
  hipLaunchKernelGGL(k_q2q, dim3(grid_of(n)), dim3(kBlock), 0, 0, n, dx.p, di.p, dout_.p,
                     dal.p, d.p);
  if (sync_ok()) d.to_host(out);
  if (g_failed)
    for (int64_t i = 0; i < n; ++i) out[i] = NAN;
}

int h3dt_equalize(int64_t n, int r, const int32_t* x, const double* f,
                  double alpha, double* out) {
  if (r < 1 || r > M) return -1;
  Dev<int32_t> dx(x, n * r);
  Dev<double> df(f, n * r), dp(nullptr, n * r);
  Dev<int> dst(nullptr, 1);
  hipLaunchKernelGGL(k_equalize_nll, dim3(grid_of(n)), dim3(kBlock), 0, 0, n, r, dx.p,
                     df.p, alpha, 1, dp.p, h3d::NllConst{}, (double*)nullptr, dst.p);
  int st = 0;
  if (!sync_ok()) return -2;
  dp.to_host(out);
  dst.to_host(&st);
  return g_failed ? -2 : st;
}

int h3dt_nll_terms(int64_t n, int r, const double* pseudo, double delta, int mode,
                   double* out) {
  if (r < 1 || r > M || mode < 0 || mode > 2) return -1;
  Dev<double> dp(pseudo, n * r), dout_(nullptr, n);
  const h3d::NllConst kc = h3d::nll_const(delta, r);
  hipLaunchKernelGGL(k_nll_terms, dim3(grid_of(n)), dim3(kBlock), 0, 0, n, r, dp.p, kc, mode,
                     dout_.p);
  if (!sync_ok()) return -2;
  dout_.to_host(out);
  return g_failed ? -2 : 0;
}

int h3dt_lrt(int64_t n, int R, int C, const int32_t* raw, const double* f,
             const double* disp_wide, const int32_t* cond_of_rep, int refit,
             double* p, double* llr, double* mu0, double* mu1) {
  if (R < 1 || R > M || C < 1 || C > h3d::kMaxConds) return -1;
  Dev<int32_t> dr(raw, n * R), dc(cond_of_rep, R);
  Dev<double> df(f, n * R), dd(disp_wide, n * R), dp(nullptr, n), dl(nullptr, n),
      d0(nullptr, n), d1(nullptr, n * C);
  Dev<int> dst(nullptr, 1);
  hipLaunchKernelGGL(k_lrt, dim3(grid_of(n)), dim3(kBlock), 0, 0, n, R, C, dr.p, df.p,
                     dd.p, dc.p, refit, dp.p, dl.p, d0.p, d1.p, dst.p);
  int st = 0;
  if (!sync_ok()) return -2;
  dp.to_host(p);
  dl.to_host(llr);
  d0.to_host(mu0);
  d1.to_host(mu1);
  dst.to_host(&st);
  return g_failed ? -2 : st;
}

// full qcml on one segment: the data passes (equalize, NLL terms) run on the
// device, the bounded-Brent / qcml state machine (h3d_model.h seg_step) and
// the pixel-term sum on the host
double h3dt_qcml(int64_t n, int r, const int32_t* x, const double* f,
                 int* status) {
  if (r < 1 || r > M) {
    *status = -1;
    return NAN;
  }
  Dev<int32_t> dx(x, n * r);
  Dev<double> df(f, n * r), dp(nullptr, n * r), dt(nullptr, n);
  Dev<int> dst(nullptr, 1);
  std::vector<double> term(n);
  h3d::SegState st;
  h3d::seg_init(&st, n, r);
  int guard = 0;
  while (st.phase != h3d::kDone && guard++ < 100000) {
    hipLaunchKernelGGL(k_equalize_nll, dim3(grid_of(n)), dim3(kBlock), 0, 0, n, r, dx.p,
                       df.p, st.disp, st.phase == h3d::kEqualize ? 1 : 0, dp.p, st.k,
                       dt.p, dst.p);
    if (!sync_ok()) {
      *status = -2;
      return NAN;
    }
    dt.to_host(term.data());
    double total = 0.0;
    for (int64_t i = 0; i < n; ++i) total += term[i];
    h3d::seg_step(&st, total, r);
  }
  int fl = 0;
  dst.to_host(&fl);
  *status = st.flags | fl | (g_failed ? -2 : 0);
  return st.result;
}

}  // extern "C"
