// Measured roofline denominators for bench.py (achieved
// FP64 rate and HBM bandwidth against MEASURED peaks, beside the spec ones).
//
// libh3d_peak.so -- measurement only; the product never loads it.
//   h3d_peak_fp64: independent v_fma_f64 chains, 8 per lane, at 8 waves per
//                  SIMD over every CU: the chip's sustained vector-FP64 FMA
//                  issue rate (2 flops per lane per FMA).
//   h3d_peak_copy: a 16-byte-per-lane streaming copy (double2 nontemporal
//                  loads and stores, four in flight per lane, grid-stride,
//                  every CU), read + write bytes over the kernel time: the
//                  sustained HBM rate.
// Each runs `reps` timed launches after one warm-up launch on its own stream
// and reports the best (the least disturbed) and the median launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

namespace {

constexpr int kChains = 8;
constexpr int kUnroll = 16;
constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void k_fma_chains(double* __restrict__ sink,
                                                       double a, double b,
                                                       int iters) {
  double x[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c)
    x[c] = 1.0 + 1e-9 * (threadIdx.x + c * 977 + blockIdx.x);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
      for (int c = 0; c < kChains; ++c) x[c] = __builtin_fma(x[c], a, b);
    }
  }
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s += x[c];
  // never true for the arguments the host passes; keeps the chains live
  if (s == -1.0) sink[blockIdx.x * kBlock + threadIdx.x] = s;
}

// four independent 16-byte loads in flight per lane before their stores
// (one load per trip measured 4.8 TB/s: too few bytes in flight per CU)
constexpr int kCopyUnroll = 4;

__global__ __launch_bounds__(kBlock) void k_copy16(const double2* __restrict__ src,
                                                   double2* __restrict__ dst,
                                                   int64_t n) {
  constexpr int U = kCopyUnroll;
  const int64_t stride = (int64_t)gridDim.x * kBlock * U;
  int64_t i = blockIdx.x * (int64_t)kBlock * U + threadIdx.x;
  for (; i + (U - 1) * kBlock < n; i += stride) {
    // (as a two-double vector type: the nontemporal builtins take native
    // vectors, not HIP's double2 struct)
    typedef double v2d __attribute__((ext_vector_type(2)));
    const v2d* s2 = reinterpret_cast<const v2d*>(src);
    v2d* d2 = reinterpret_cast<v2d*>(dst);
    v2d v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(s2 + i + u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], d2 + i + u * kBlock);
  }
  for (; i < n; i += kBlock) dst[i] = src[i];  // the ragged end
}

struct Timing {
  double best_ms = 0, median_ms = 0;
};

template <class Launch>
int time_launches(hipStream_t s, int reps, Launch launch, Timing* t) {
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess)
    return -1;
  launch();  // warm-up
  std::vector<double> ms;
  for (int r = 0; r < reps; ++r) {
    (void)hipEventRecord(a, s);
    launch();
    (void)hipEventRecord(b, s);
    if (hipEventSynchronize(b) != hipSuccess) return -2;
    float v = 0.f;
    (void)hipEventElapsedTime(&v, a, b);
    ms.push_back(v);
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  if (hipGetLastError() != hipSuccess) return -3;
  std::sort(ms.begin(), ms.end());
  t->best_ms = ms.front();
  t->median_ms = ms[ms.size() / 2];
  return 0;
}

int cu_count(int device) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount,
                            device) != hipSuccess)
    return 0;
  return cus;
}

}  // namespace

extern "C" {

// out[0] best TFLOP/s, out[1] median TFLOP/s, out[2] flops per launch,
// out[3] best ms. Returns 0 or a negative HIP failure code.
int h3d_peak_fp64(int device, int reps, double* out) {
  if (hipSetDevice(device) != hipSuccess || reps < 1) return -10;
  const int cus = cu_count(device);
  if (cus <= 0) return -11;
  // 8 waves per SIMD: 4 SIMDs x 8 waves x 64 lanes = 8 blocks of 256 per CU
  const int blocks = cus * 8;
  const int iters = 2048;
  double* sink = nullptr;
  if (hipMalloc(&sink, (size_t)blocks * kBlock * sizeof(double)) != hipSuccess)
    return -12;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
    (void)hipFree(sink);
    return -13;
  }
  Timing t;
  const int st = time_launches(s, reps, [&] {
    k_fma_chains<<<blocks, kBlock, 0, s>>>(sink, 0.999999999, 1e-9, iters);
  }, &t);
  (void)hipStreamDestroy(s);
  (void)hipFree(sink);
  if (st) return st;
  const double flops = 2.0 * kChains * kUnroll * (double)iters * blocks * kBlock;
  out[0] = flops / (t.best_ms * 1e-3) / 1e12;
  out[1] = flops / (t.median_ms * 1e-3) / 1e12;
  out[2] = flops;
  out[3] = t.best_ms;
  return 0;
}

// out[0] best GB/s, out[1] median GB/s (read + write bytes), out[2] bytes per
// launch, out[3] best ms. `bytes` per buffer (rounded down to 16 B).
int h3d_peak_copy(int device, int64_t bytes, int reps, double* out) {
  if (hipSetDevice(device) != hipSuccess || reps < 1 || bytes < 16) return -10;
  const int cus = cu_count(device);
  if (cus <= 0) return -11;
  const int64_t n = bytes / 16;
  double2 *src = nullptr, *dst = nullptr;
  if (hipMalloc(&src, n * 16) != hipSuccess) return -12;
  if (hipMalloc(&dst, n * 16) != hipSuccess) {
    (void)hipFree(src);
    return -12;
  }
  (void)hipMemset(src, 0, n * 16);
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
    (void)hipFree(src);
    (void)hipFree(dst);
    return -13;
  }
  // 8 blocks of 256 per CU (8 waves per SIMD), each block a contiguous run
  // of U x 256 elements per trip
  const int blocks = cus * 8;
  Timing t;
  const int st = time_launches(s, reps, [&] {
    k_copy16<<<blocks, kBlock, 0, s>>>(src, dst, n);
  }, &t);
  (void)hipStreamDestroy(s);
  (void)hipFree(src);
  (void)hipFree(dst);
  if (st) return st;
  const double moved = 2.0 * 16.0 * (double)n;
  out[0] = moved / (t.best_ms * 1e-3) / 1e9;
  out[1] = moved / (t.median_ms * 1e-3) / 1e9;
  out[2] = moved;
  out[3] = t.best_ms;
  return 0;
}

}  // extern "C"
