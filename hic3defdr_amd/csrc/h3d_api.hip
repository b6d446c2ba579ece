// libh3d.so: C ABI (include/h3d.h) + orchestration of the gfx950 kernels:
// context, profiling, the estimate_disp driver, cml, bh. The lrt entries live
// in h3d_lrt.hip, prepare_data's in h3d_prepare_api.hip (separate TUs,
// compiled in parallel).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "h3d.h"
#include "h3d_ctx.h"
#include "h3d_errors.h"
#include "h3d_host.h"
#include "h3d_kernels.h"

using namespace h3d;
using namespace h3dint;
using h3derr::fail;

namespace h3dint {

void* scratch(h3d_ctx* ctx, const char* slot, size_t bytes) {
  auto& b = ctx->bufs[slot];
  if (b.second >= bytes && b.first) return b.first;
  if (b.first) (void)hipFree(b.first);
  b.first = nullptr;
  b.second = 0;
  void* p = nullptr;
  if (hipMalloc(&p, std::max<size_t>(bytes, 256)) != hipSuccess) return nullptr;
  b.first = p;
  b.second = std::max<size_t>(bytes, 256);
  return p;
}

void* scratch_keep(h3d_ctx* ctx, const char* slot, size_t bytes, size_t keep) {
  auto& b = ctx->bufs[slot];
  if (b.first && b.second >= bytes) return b.first;
  const size_t cap = std::max<size_t>(std::max(bytes, 2 * b.second), 256);
  void* p = nullptr;
  if (hipMalloc(&p, cap) != hipSuccess) return nullptr;
  if (b.first) {
    if (keep) (void)hipMemcpyAsync(p, b.first, std::min(keep, b.second),
                                   hipMemcpyDeviceToDevice, ctx->stream);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(b.first);
  }
  b.first = p;
  b.second = cap;
  return p;
}

int h2d_pinned(h3d_ctx* ctx, void* d_dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return 0;
  const size_t need = (bytes + 255) & ~(size_t)255;
  if (!ctx->bounce_ev) HIP_TRY(hipEventCreateWithFlags(&ctx->bounce_ev, hipEventDisableTiming));
  // the buffer is rewritten only after every earlier copy out of it has
  // read it: wrap-around, growth and a change of stream wait on the last one
  const bool wrap = ctx->bounce_off + need > ctx->bounce_cap;
  if ((wrap || (ctx->bounce_stream && ctx->bounce_stream != s)) && ctx->bounce_stream) {
    HIP_TRY(hipEventSynchronize(ctx->bounce_ev));
    ctx->bounce_off = 0;
    ctx->bounce_stream = nullptr;
  }
  if (need > ctx->bounce_cap) {
    if (ctx->bounce) (void)hipHostFree(ctx->bounce);
    ctx->bounce = nullptr;
    ctx->bounce_cap = 0;
    const size_t cap = std::max<size_t>(need, (size_t)1 << 20);
    HIP_TRY(hipHostMalloc(&ctx->bounce, cap, hipHostMallocDefault));
    ctx->bounce_cap = cap;
    ctx->bounce_off = 0;
  }
  char* b = (char*)ctx->bounce + ctx->bounce_off;
  std::memcpy(b, src, bytes);
  HIP_TRY(hipMemcpyAsync(d_dst, b, bytes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipEventRecord(ctx->bounce_ev, s));
  ctx->bounce_stream = s;
  ctx->bounce_off += need;
  return 0;
}

void* pinned_rd(h3d_ctx* ctx, size_t bytes) {
  if (bytes > ctx->land_cap) {
    if (ctx->land) (void)hipHostFree(ctx->land);
    ctx->land = nullptr;
    ctx->land_cap = 0;
    const size_t cap = std::max<size_t>(bytes, 4096);
    if (hipHostMalloc(&ctx->land, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
    ctx->land_cap = cap;
  }
  return ctx->land;
}

int d2h_sync(h3d_ctx* ctx, void* dst, const void* d_src, size_t bytes, hipStream_t s) {
  void* l = pinned_rd(ctx, bytes);
  if (!l) return fail(H3D_ENOMEM, "pinned landing zone");
  HIP_TRY(hipMemcpyAsync(l, d_src, bytes, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  std::memcpy(dst, l, bytes);
  return 0;
}

hipEvent_t ev_get(h3d_ctx* ctx) {
  if (!ctx->event_pool.empty()) {
    hipEvent_t e = ctx->event_pool.back();
    ctx->event_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}

void prof_collect(h3d_ctx* ctx) {
  if (ctx->pending.empty()) return;
  (void)hipStreamSynchronize(ctx->stream);
  for (size_t i = 0; i < ctx->pending.size(); ++i) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, ctx->pending[i].second.first,
                              ctx->pending[i].second.second);
    auto& e = ctx->stats[ctx->pending[i].first];
    e.ms += ms;
    e.launches += 1;
    e.units += ctx->pending_units[i];
    ctx->event_pool.push_back(ctx->pending[i].second.first);
    ctx->event_pool.push_back(ctx->pending[i].second.second);
  }
  ctx->pending.clear();
  ctx->pending_units.clear();
}

int grid_for(h3d_ctx* ctx, int64_t n, int per_cu) {
  int64_t g = (n + kBlock - 1) / kBlock;
  g = std::min<int64_t>(g, (int64_t)ctx->n_cu * per_cu);
  return (int)std::max<int64_t>(g, 1);
}

int check_cond(const int32_t* cond_of_rep, int R, int C, std::vector<int>* nrep,
               std::vector<int32_t>* rep_idx) {
  if (R < 1 || R > kMaxReps) return fail(H3D_EARG, "R=%d outside [1, %d]", R, kMaxReps);
  if (C < 1 || C > kMaxConds) return fail(H3D_EARG, "C=%d outside [1, %d]", C, kMaxConds);
  nrep->assign(C, 0);
  rep_idx->assign((size_t)C * kMaxReps, 0);
  for (int r = 0; r < R; ++r) {
    const int c = cond_of_rep[r];
    if (c < 0 || c >= C) return fail(H3D_EARG, "cond_of_rep[%d]=%d", r, c);
    (*rep_idx)[(size_t)c * kMaxReps + (*nrep)[c]] = r;
    (*nrep)[c] += 1;
  }
  for (int c = 0; c < C; ++c)
    if ((*nrep)[c] == 0) return fail(H3D_EARG, "condition %d has no replicates", c);
  return 0;
}

int flags_to_code(int fl) {
  if (fl & kFlagBadInput) return fail(H3D_EINPUT, "non-positive or non-finite dispersion / scaling factor (status %d)", fl);
  if (fl & (kFlagNoRoot | kFlagNoConv)) return fail(H3D_ENOCONV, "mean MLE failed (status %d)", fl);
  if (fl & (kFlagBrentFail | kFlagQcmlGuard)) return fail(H3D_ENOCONV, "dispersion optimisation failed (status %d)", fl);
  return 0;
}

}  // namespace h3dint

namespace {

// H3D_TIMING=1: host-side stage stamps of the estimate_disp driver (stderr)
struct HostStamps {
  bool on = std::getenv("H3D_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  void operator()(const char* what) const {
    if (on)
      fprintf(stderr, "[h3d timing] %8.1f us %s\n",
              std::chrono::duration<double, std::micro>(
                  std::chrono::steady_clock::now() - t0).count(), what);
  }
};

// workgroups of `kernel` that fit on one CU at once (queried once per kernel;
// every device of a process is a gfx950)
template <typename K>
int resident_blocks(K kernel) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, kBlock, 0) != hipSuccess ||
      nb < 1)
    nb = 1;
  return nb;
}

// grid = one full wave of resident workgroups (the kernels grid-stride over
// the work list), at most one workgroup per item
template <typename K>
int work_grid(h3d_ctx* ctx, K kernel, size_t max_items) {
  int& nb = ctx->resident[(const void*)kernel];
  if (nb == 0) nb = resident_blocks(kernel);
  return (int)std::max<size_t>(1, std::min<size_t>(max_items, (size_t)ctx->n_cu * nb));
}

template <int M, bool NLL>
void launch_disp_work(h3d_ctx* ctx, size_t max_items, const int32_t* raw_s,
                      const double* f_s, double* pd, int64_t n,
                      const int64_t* cs, const int32_t* cl, const int32_t* cd,
                      int C, const int32_t* rep_idx, const int32_t* n_rep,
                      const SegState* st, int* seg_flags, const int32_t* list,
                      int32_t* meta, double* partial) {
  // equalize pass (heavy: q2qnbinom), then (multi-rank driver) the NLL-only
  // pass (light)
  {
    ProfScope ps(ctx, "disp_work", 0, 1);
#define H3D_EQ(WW)                                                                  \
  do {                                                                              \
    auto k = k_disp_work<M, WW, kEqualize, NLL>;                                    \
    hipLaunchKernelGGL(k, dim3(work_grid(ctx, k, max_items)), dim3(kBlock), 0,      \
                       ctx->stream, raw_s, f_s, pd, n, cs, cl, cd, C, rep_idx, n_rep, \
                       st, seg_flags, list, meta, partial, ctx->eq_static8);        \
  } while (0)
    if constexpr (M == 2 && NLL) {
      H3D_EQ(4);
    } else if constexpr (M == 2) {
      // H3D_DISP_W2: the R_c <= 2 path (cfg2's 2 + 2 design)
      if (ctx->disp_w2 == 8) H3D_EQ(8);
      else if (ctx->disp_w2 == 6) H3D_EQ(6);
      else if (ctx->disp_w2 == 5) H3D_EQ(5);
      else H3D_EQ(4);
    } else if constexpr (M == 4) {
      if (ctx->disp_w == 4) H3D_EQ(4);
      else if (ctx->disp_w == 3) H3D_EQ(3);
      else if (ctx->disp_w == 2) H3D_EQ(2);
      else H3D_EQ(1);
    } else if constexpr (M == 8) {
      // H3D_DISP_W8: register budget of the M = 8 path (R_c <= 8, cfg4;
      // W 1/2/3/4 measured 214/214/199/197 ms per cfg4 step, r02)
      if (ctx->disp_w8 == 4) H3D_EQ(4);
      else H3D_EQ(1);
    } else {
      H3D_EQ(1);
    }
#undef H3D_EQ
  }
  if constexpr (NLL) {
    ProfScope ps(ctx, "disp_nll", 0);
    auto k = k_disp_work<M, 1, kNll>;
    if constexpr (M == 4) {
      if (ctx->nll_w == 2) k = k_disp_work<M, 2, kNll>;
      else if (ctx->nll_w == 4) k = k_disp_work<M, 4, kNll>;
    }
    hipLaunchKernelGGL(k, dim3(work_grid(ctx, k, max_items)), dim3(kBlock), 0,
                       ctx->stream, raw_s, f_s, pd, n, cs, cl, cd, C, rep_idx, n_rep,
                       st, seg_flags, list, meta, partial, ctx->eq_static8);
  }
}

// the whole Brent search of every freshly equalized segment (single rank)
template <int M>
void launch_brent(h3d_ctx* ctx, const double* pd, int64_t n, const int64_t* seg_start,
                  int S, int C, const int32_t* rep_idx, const int32_t* n_rep,
                  SegState* st, const int* seg_flags, double* result, int* queue,
                  const int32_t* gate_meta = nullptr, int live_min = 0,
                  const int* gang_abort = nullptr, bool queue_zeroed = false) {
  ProfScope ps(ctx, "disp_nll", 0);
  auto k = k_brent<M>;
  constexpr int kBrentBlock = brent_block<M>();
  const size_t lds_max = M <= 8 ? (size_t)ctx->brent_lds_kb * 1024 : 0;
  int& nb = ctx->resident[(const void*)k];
  if (nb == 0) {
    if (lds_max)
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds_max);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kBrentBlock, lds_max) !=
            hipSuccess ||
        nb < 1)
      nb = 1;
  }
  const int grid = std::max(1, std::min(S, ctx->n_cu * nb));
  // LDS staging of each segment's head: the workgroup's whole share of the
  // CU's LDS (one 1024-thread workgroup per CU), minus the static part
  // (M >= 16: 512-thread workgroups, two per CU -- staging would halve that)
  const size_t lds_bytes = M <= 8 ? (size_t)ctx->brent_lds_kb * 1024 : 0;
  const int64_t lds_px = (int64_t)(lds_bytes / (8 * (size_t)M));
  if (!queue_zeroed) (void)hipMemsetAsync(queue, 0, sizeof(int), ctx->stream);
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBrentBlock), lds_px ? lds_px * 8 * M : 0,
                     ctx->stream, pd, n, seg_start, S, C, rep_idx, n_rep, st, seg_flags,
                     result, queue, ctx->work_count, lds_px, gate_meta, live_min, gang_abort);
#ifdef H3D_BRENT_CLOCK
  unsigned long long clk[38];
  (void)hipMemcpyFromSymbolAsync(clk, HIP_SYMBOL(g_brent_clk), sizeof(clk), 0,
                                 hipMemcpyDeviceToHost, ctx->stream);
  (void)hipStreamSynchronize(ctx->stream);
  fprintf(stderr, "[brent_clk] sum %llu bar1 %llu step %llu bar2 %llu stage %llu total %llu\n",
          clk[0], clk[1], clk[2], clk[3], clk[4], clk[5]);
  fprintf(stderr, "[brent_clk_wave] sum");
  for (int i = 0; i < 16; ++i) fprintf(stderr, " %llu", clk[6 + i]);
  fprintf(stderr, " bar1");
  for (int i = 0; i < 16; ++i) fprintf(stderr, " %llu", clk[22 + i]);
  fprintf(stderr, "\n");
#endif
}

// the gang variant (k_brent_gang): every live segment's search over the
// co-resident workgroups of its slices.
struct GangTables {
  int32_t* task_seg = nullptr;
  int32_t* task_g = nullptr;
  int T = 0, gmax = 1, grid = 0;
  int64_t P = 0;
  double* part = nullptr;
  int* tag = nullptr;
  int* abort = nullptr;
  long long timeout = 0;
};

// next tag epoch of the gang exchange: the tags are cleared when their
// buffer is new -- another pointer, or the same pointer handed out again by
// a grown allocation (scratch frees and reallocates: the grown tail would
// hold stale device words), i.e. another (pointer, capacity) -- or the epoch
// wraps (tag = epoch << 10 | evaluation + 1). The whole allocation is
// cleared, so a later call with another layout (S, gmax) inside the same
// allocation only ever finds zeros or tags of older epochs.
int gang_next_epoch(h3d_ctx* ctx, const GangTables& g, int S) {
  const size_t cap = ctx->bufs["gang_tag"].second;
  if (ctx->gang_tag_buf != (void*)g.tag || ctx->gang_tag_cap != cap ||
      ctx->gang_epoch >= (1 << 20)) {
    const size_t bytes = std::max(cap, (size_t)2 * S * g.gmax * 4);
    if (hipMemsetAsync(g.tag, 0, bytes, ctx->stream) != hipSuccess) return -1;
    ctx->gang_tag_buf = (void*)g.tag;
    ctx->gang_tag_cap = cap;
    ctx->gang_epoch = 0;
  }
  return ++ctx->gang_epoch;
}

// spin bound of a gang wait: 0.5 s of the constant-rate wall clock
long long gang_timeout(h3d_ctx* ctx) {
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device) !=
          hipSuccess ||
      khz <= 0)
    khz = 100000;
  return (long long)khz * 500;
}

// Returns 1 (nothing set up) when one workgroup per segment already fills
// the chip -- the gang's exchange only pays where CUs would idle -- or when
// a gang would not fit the resident grid.
template <int M>
int gang_setup(h3d_ctx* ctx, const std::vector<int64_t>& seg_start, int D, int C,
               GangTables* g) {
  auto k = k_brent_gang<M>;
  int& nb = ctx->resident[(const void*)k];
  if (nb == 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kGangThreads, 0) != hipSuccess ||
        nb < 1)
      nb = 1;
  }
  g->grid = ctx->n_cu * nb;
  int live = 0;
  int64_t total = 0;
  for (int d = 0; d < D; ++d) {
    const int64_t np = seg_start[d + 1] - seg_start[d];
    if (np) live += C;
    total += np * C;
  }
  // H3D_BRENT=1 (auto): gangs when the segments leave CUs without a
  // workgroup; 2: always
  if (ctx->brent_gang == 1 && live >= ctx->n_cu) return 1;
  // slices: about two resident grids of them over the whole call, at least
  // 1024 pixels (4 per thread)
  int64_t P = (total + 2 * (int64_t)g->grid - 1) / (2 * (int64_t)g->grid);
  P = std::max<int64_t>(1024, (P + kGangThreads - 1) / kGangThreads * kGangThreads);
  std::vector<int32_t> ts, tg;
  int gmax = 1;
  for (int d = 0; d < D; ++d) {
    const int64_t np = seg_start[d + 1] - seg_start[d];
    if (np == 0) continue;
    const int G = (int)((np + P - 1) / P);
    if (G > g->grid) return 1;  // cannot be co-resident: plain k_brent
    gmax = std::max(gmax, G);
    for (int c = 0; c < C; ++c)
      for (int j = 0; j < G; ++j) {
        ts.push_back(d * C + c);
        tg.push_back(j);
      }
  }
  const int S = D * C;
  g->T = (int)ts.size();
  g->gmax = gmax;
  g->P = P;
  g->task_seg = (int32_t*)scratch(ctx, "gang_seg", std::max<size_t>(1, ts.size()) * 4);
  g->task_g = (int32_t*)scratch(ctx, "gang_g", std::max<size_t>(1, tg.size()) * 4);
  g->part = (double*)scratch(ctx, "gang_part", (size_t)2 * S * gmax * 8);
  g->tag = (int*)scratch(ctx, "gang_tag", (size_t)2 * S * gmax * 4);
  g->abort = (int*)scratch(ctx, "gang_abort", 4);
  if (!g->task_seg || !g->task_g || !g->part || !g->tag || !g->abort)
    return fail(H3D_ENOMEM, "gang tables");
  if (g->T) {
    HIP_TRY(hipMemcpyAsync(g->task_seg, ts.data(), ts.size() * 4, hipMemcpyHostToDevice,
                           ctx->stream));
    HIP_TRY(hipMemcpyAsync(g->task_g, tg.data(), tg.size() * 4, hipMemcpyHostToDevice,
                           ctx->stream));
  }
  HIP_TRY(hipMemsetAsync(g->abort, 0, 4, ctx->stream));
  // the host vectors die here: the copies must have read them
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  g->timeout = gang_timeout(ctx);
  return 0;
}

// Device-built gang tables (the dev_tables path, no host sync): the slice
// size from the call's pixel count alone -- about two resident grids of
// slices over all segments, at least 1024 pixels, and few enough slices per
// segment to be co-resident (G <= grid) --, room for the task table
// (k_disp_tables fills it) and the exchange buffers sized for the largest
// possible segment (all n pixels).
template <int M>
int gang_setup_dev(h3d_ctx* ctx, int64_t n, int D, int C, GangTables* g) {
  auto k = k_brent_gang<M>;
  int& nb = ctx->resident[(const void*)k];
  if (nb == 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kGangThreads, 0) != hipSuccess ||
        nb < 1)
      nb = 1;
  }
  g->grid = ctx->n_cu * nb;
  const int64_t total = n * C;
  int64_t P = (total + 2 * (int64_t)g->grid - 1) / (2 * (int64_t)g->grid);
  P = std::max<int64_t>(P, (n + g->grid - 1) / g->grid);
  P = std::max<int64_t>(1024, (P + kGangThreads - 1) / kGangThreads * kGangThreads);
  if (ctx->gang_px > 0)
    P = std::max<int64_t>(std::max<int64_t>(64, ctx->gang_px), (n + g->grid - 1) / g->grid);
  g->P = P;
  g->gmax = (int)std::max<int64_t>(1, (n + P - 1) / P);
  g->T = (int)std::min<int64_t>(INT32_MAX, (int64_t)C * (g->gmax + D));
  const int S = D * C;
  g->task_seg = (int32_t*)scratch(ctx, "gang_seg", (size_t)g->T * 4);
  g->task_g = (int32_t*)scratch(ctx, "gang_g", (size_t)g->T * 4);
  g->part = (double*)scratch(ctx, "gang_part", (size_t)2 * S * g->gmax * 8);
  g->tag = (int*)scratch(ctx, "gang_tag", (size_t)2 * S * g->gmax * 4);
  g->abort = (int*)scratch(ctx, "gang_abort", 4);
  if (!g->task_seg || !g->task_g || !g->part || !g->tag || !g->abort)
    return fail(H3D_ENOMEM, "gang tables");
  // (task_seg's tail and abort are set by k_disp_tables, which fills the
  // table)
  g->timeout = gang_timeout(ctx);
  return 0;
}

template <int M>
void launch_brent_gang(h3d_ctx* ctx, const double* pd, int64_t n, const int64_t* seg_start,
                       int S, int C, const int32_t* rep_idx, const int32_t* n_rep,
                       SegState* st, const int* seg_flags, double* result, int* queue,
                       const GangTables& g, const int32_t* gate_meta = nullptr,
                       int live_max = 0, bool queue_zeroed = false) {
  ProfScope ps(ctx, "disp_nll", 0);
  if (!queue_zeroed) (void)hipMemsetAsync(queue, 0, sizeof(int), ctx->stream);
  const int epoch = gang_next_epoch(ctx, g, S);
  const int grid = std::max(1, std::min(g.T, g.grid));
  hipLaunchKernelGGL(k_brent_gang<M>, dim3(grid), dim3(kGangThreads), 0, ctx->stream, pd,
                     n, seg_start, S, C, rep_idx, n_rep, st, seg_flags, result, queue,
                     g.task_seg, g.task_g, g.T, g.P, g.part, g.tag, g.gmax, g.abort,
                     g.timeout, ctx->work_count, epoch, gate_meta, live_max);
}

// algorithmic HBM bytes of the disp_work launches so far: an equalize
// pixel-replicate reads raw (4 B) + f (8 B) and writes pseudodata (8 B); an
// NLL pixel-replicate reads pseudodata (8 B)
int64_t disp_work_bytes(h3d_ctx* ctx, bool nll) {
  unsigned long long c[2] = {0, 0};
  if (!ctx->work_count) return 0;
  (void)hipMemcpyAsync(c, ctx->work_count, sizeof(c), hipMemcpyDeviceToHost, ctx->stream);
  (void)hipStreamSynchronize(ctx->stream);
  return nll ? (int64_t)(c[1] * 8ull) : (int64_t)(c[0] * 20ull);
}

}  // namespace

extern "C" {

int h3d_version(void) { return 1; }

const char* h3d_last_error(void) { return h3derr::last(); }

int h3d_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

h3d_ctx* h3d_open(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    fail(H3D_ENODEV, "no HIP device visible");
    return nullptr;
  }
  if (device < 0 || device >= n) {
    fail(H3D_EARG, "device %d of %d", device, n);
    return nullptr;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    fail(H3D_EHIP, "hipGetDeviceProperties failed");
    return nullptr;
  }
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    fail(H3D_ENODEV, "device %d is %s, libh3d is built for gfx950", device,
         prop.gcnArchName);
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    fail(H3D_EHIP, "hipSetDevice failed");
    return nullptr;
  }
  h3d_ctx* ctx = new h3d_ctx();
  ctx->device = device;
  ctx->n_cu = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    fail(H3D_EHIP, "stream create failed");
    return nullptr;
  }
  ctx->stream = ctx->own;
  if (const char* e = std::getenv("H3D_DISP_W")) ctx->disp_w = std::atoi(e);
  if (const char* e = std::getenv("H3D_DISP_SORT")) ctx->disp_sort = std::atoi(e);
  if (const char* e = std::getenv("H3D_NLL_W")) ctx->nll_w = std::atoi(e);
  if (const char* e = std::getenv("H3D_DISP_W8")) ctx->disp_w8 = std::atoi(e);
  if (const char* e = std::getenv("H3D_DISP_W2")) ctx->disp_w2 = std::atoi(e);
  if (const char* e = std::getenv("H3D_PACK_GATHER")) ctx->pack_gather = std::atoi(e);
  if (const char* e = std::getenv("H3D_EQ_STATIC8"))
    ctx->eq_static8 = std::max(0, std::min(8, std::atoi(e)));
  if (const char* e = std::getenv("H3D_DISP_M2")) ctx->disp_m2 = std::atoi(e);
  if (const char* e = std::getenv("H3D_BRENT")) ctx->brent_gang = std::atoi(e);
  if (const char* e = std::getenv("H3D_BRENT_LDS_KB")) ctx->brent_lds_kb = std::atoi(e);
  if (const char* e = std::getenv("H3D_GANG_P")) ctx->gang_px = std::atoi(e);
  if (const char* e = std::getenv("H3D_DEV_SEG_TABLES")) ctx->dev_seg_tables = std::atoi(e);
  if (hipMalloc((void**)&ctx->work_count, 2 * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(ctx->work_count, 0, 2 * sizeof(unsigned long long)) != hipSuccess) {
    (void)hipStreamDestroy(ctx->own);
    delete ctx;
    fail(H3D_ENOMEM, "counter allocation failed");
    return nullptr;
  }
  return ctx;
}

void h3d_close(h3d_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  prof_collect(ctx);
  for (auto& kv : ctx->bufs)
    if (kv.second.first) (void)hipFree(kv.second.first);
  for (auto e : ctx->event_pool) (void)hipEventDestroy(e);
  if (ctx->work_count) (void)hipFree(ctx->work_count);
  if (ctx->h_meta) (void)hipHostFree(ctx->h_meta);
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  if (ctx->h_res) (void)hipHostFree(ctx->h_res);
  if (ctx->h_stage_done) (void)hipEventDestroy(ctx->h_stage_done);
  if (ctx->bounce) (void)hipHostFree(ctx->bounce);
  if (ctx->bounce_ev) (void)hipEventDestroy(ctx->bounce_ev);
  if (ctx->land) (void)hipHostFree(ctx->land);
  if (ctx->own) (void)hipStreamDestroy(ctx->own);
  delete ctx;
}

int h3d_set_stream(h3d_ctx* ctx, void* stream) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  ctx->stream = stream ? (hipStream_t)stream : ctx->own;
  return 0;
}

int h3d_set_qcml_tol(h3d_ctx* ctx, double tol) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  if (!(tol >= 0.0) || !(tol < INFINITY)) return fail(H3D_EARG, "qcml tol %g", tol);
  ctx->qcml_tol = tol;
  return 0;
}

int h3d_profile_enable(h3d_ctx* ctx, int on) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  prof_collect(ctx);
  ctx->prof = on < 0 ? 0 : on > 2 ? 2 : on;
  return 0;
}

int h3d_profile_reset(h3d_ctx* ctx) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  prof_collect(ctx);
  ctx->stats.clear();
  HIP_TRY(hipMemsetAsync(ctx->work_count, 0, 2 * sizeof(unsigned long long), ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

// Section clock ticks of the equalize pass (a -DH3D_SECPROF build only,
// h3d_special.h; tools/secprof.py): copies the 32 counters out, then zeroes
// them when reset. Returns -1 (H3D_EARG) in a normal build. Not part of
// include/h3d.h: a measurement hook of profiling builds.
extern "C" int h3d_secprof(int reset, unsigned long long* out32) {
#if defined(H3D_SECPROF)
  if (out32)
    HIP_TRY(hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_h3d_secprof), 32 * 8, 0,
                                hipMemcpyDeviceToHost));
  if (reset) {
    static const unsigned long long zeros[32] = {};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_h3d_secprof), zeros, 32 * 8, 0,
                              hipMemcpyHostToDevice));
  }
  return 0;
#else
  (void)reset;
  (void)out32;
  return fail(H3D_EARG, "not a -DH3D_SECPROF build");
#endif
}

int h3d_profile_read(h3d_ctx* ctx, const char* name, double* total_ms,
                     int64_t* launches, int64_t* units) {
  if (!ctx || !name) return fail(H3D_EARG, "null argument");
  prof_collect(ctx);
  if (std::strcmp(name, "gang_aborts") == 0) {
    // gang Brent waits that hit their wall-clock bound (the searches then
    // finished under k_brent): a count over the ctx's life, not a timing
    if (total_ms) *total_ms = 0.0;
    if (launches) *launches = ctx->gang_aborts;
    if (units) *units = 0;
    return 0;
  }
  auto it = ctx->stats.find(name);
  ProfEntry e = (it == ctx->stats.end()) ? ProfEntry() : it->second;
  if (total_ms) *total_ms = e.ms;
  if (launches) *launches = e.launches;
  // disp_work / disp_nll units = algorithmic bytes; lrt / disp_prep = pixels
  if (units)
    *units = std::strcmp(name, "disp_work") == 0   ? disp_work_bytes(ctx, false)
             : std::strcmp(name, "disp_nll") == 0 ? disp_work_bytes(ctx, true)
                                                   : e.units;
  return 0;
}

// ---------------------------------------------------------------------------
// estimate_disp
// ---------------------------------------------------------------------------

namespace {
// H3D_DEBUG: the first launch error of the estimate_disp driver, by site
void dbg_launch(const char* where) {
  static const bool on = std::getenv("H3D_DEBUG") != nullptr;
  if (!on) return;
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fprintf(stderr, "[h3d] launch error at %s: %s\n", where, hipGetErrorString(e));
}

// h3d_estimate_disp_dev's request: the smoothed tables of the result, on the
// device, enqueued behind the result copies
struct TableReq {
  int weighted;
  double frac, aff;
  double* d_tables;
};

int disp_per_dist_core(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                       const int32_t* d_dist, int64_t n, int R, int C,
                       const int32_t* cond_of_rep, int D, int estimator,
                       double* disp_per_dist, int32_t* seg_flags_out,
                       h3d_allreduce_fn reduce, void* user, const TableReq* treq);
}  // namespace

int h3d_disp_per_dist_dev(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                          const int32_t* d_dist, int64_t n, int R, int C,
                          const int32_t* cond_of_rep, int D, int estimator,
                          double* disp_per_dist, int32_t* seg_flags_out,
                          h3d_allreduce_fn reduce, void* user) {
  return disp_per_dist_core(ctx, d_raw, d_f, d_dist, n, R, C, cond_of_rep, D, estimator,
                            disp_per_dist, seg_flags_out, reduce, user, nullptr);
}

int h3d_estimate_disp_dev(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                          const int32_t* d_dist, int64_t n, int R, int C,
                          const int32_t* cond_of_rep, int D, int weighted, double frac,
                          double auto_frac_factor, double* disp_per_dist,
                          int32_t* seg_flags_out, double* d_tables_out) {
  if (!d_tables_out) return fail(H3D_EARG, "null d_tables_out");
  const TableReq req{weighted, frac, auto_frac_factor, d_tables_out};
  return disp_per_dist_core(ctx, d_raw, d_f, d_dist, n, R, C, cond_of_rep, D, H3D_EST_QCML,
                            disp_per_dist, seg_flags_out, nullptr, nullptr, &req);
}

namespace {
int disp_per_dist_core(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                       const int32_t* d_dist, int64_t n, int R, int C,
                       const int32_t* cond_of_rep, int D, int estimator,
                       double* disp_per_dist, int32_t* seg_flags_out,
                       h3d_allreduce_fn reduce, void* user, const TableReq* treq) {
  if (!ctx || !cond_of_rep || !disp_per_dist) return fail(H3D_EARG, "null argument");
  if (n < 0 || D < 1) return fail(H3D_EARG, "n=%lld D=%d", (long long)n, D);
  if (n > 0 && (!d_raw || !d_f || !d_dist)) return fail(H3D_EARG, "null device input");
  if (n >= (int64_t)1 << 31) return fail(H3D_EARG, "n=%lld exceeds 2^31 pixels per call", (long long)n);
  if (estimator != H3D_EST_QCML)
    return fail(H3D_EARG, "estimator %d: only qcml runs on the GPU path (the reference's cml/mme divide an int64 array in place and raise)", estimator);
  std::vector<int> nrep;
  std::vector<int32_t> rep_idx;
  if (int rc = check_cond(cond_of_rep, R, C, &nrep, &rep_idx)) return rc;
  HIP_TRY(hipSetDevice(ctx->device));
  if (std::getenv("H3D_DEBUG")) {
    const hipError_t pe = hipGetLastError();
    if (pe != hipSuccess)
      fprintf(stderr, "[h3d] estimate_disp entry: pending HIP error %s\n", hipGetErrorString(pe));
  }
  hipStream_t s = ctx->stream;
  const int S = D * C;
  const int maxnr = *std::max_element(nrep.begin(), nrep.end());
  HostStamps stamp;
  // the per-call tables built on the device (k_disp_tables), no host sync
  // before the qcml loop -- single rank, and enough segments that the Brent
  // searches need no gangs (whose task tables the host builds from the
  // segment bounds)
  // (any number of live segments: the Brent mode -- one workgroup per
  // segment or gangs -- is chosen on the device per qcml iteration, so a rank
  // of the distance re-shard, whose ~D / world live segments leave CUs idle,
  // needs no host-built gang tables either; r03z: its N = 8 cfg3 share 13.9
  // ms per step with the host tables, 13.9 with these)
  const bool dev_tables = ctx->dev_seg_tables && !reduce && n > 0 && ctx->brent_gang != 2;

  // 1. stable sort of the pixels by distance, SoA gather
  std::vector<int64_t> seg_start(D + 1, 0);
  int32_t *raw_s = nullptr, *dist_s = nullptr;
  double *f_s = nullptr, *pd = nullptr;
  if (n > 0) {
    ProfScope ps(ctx, "disp_prep", n);
    int32_t* idx_in = (int32_t*)scratch(ctx, "idx_in", n * 4);
    int32_t* idx_out = (int32_t*)scratch(ctx, "idx_out", n * 4);
    dist_s = (int32_t*)scratch(ctx, "dist_s", n * 4);
    raw_s = (int32_t*)scratch(ctx, "raw_s", n * R * 4);
    f_s = (double*)scratch(ctx, "f_s", n * R * 8);
    pd = (double*)scratch(ctx, "pd", n * R * 8);
    int64_t* d_seg = (int64_t*)scratch(ctx, "seg_start", (D + 1) * 8);
    if (!idx_in || !idx_out || !dist_s || !raw_s || !f_s || !pd || !d_seg)
      return fail(H3D_ENOMEM, "device allocation failed (n=%lld)", (long long)n);
    hipLaunchKernelGGL(k_iota, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s, idx_in, n);
    int end_bit = 1;
    while ((1 << end_bit) <= D) ++end_bit;
    size_t tmp_bytes = 0;
    if (ctx->disp_sort == 2) {
      // one (distance, max, min count) order per condition: per condition a
      // key pass over its replicates' counts, a radix sort, and a tiled
      // gather of just those replicates' row slices (k_gather_cond_tile)
      idx_out = (int32_t*)scratch(ctx, "idx_out_c", (size_t)n * 4);
      int32_t* d_reps = (int32_t*)scratch(ctx, "sort_reps", (size_t)C * kMaxReps * 4);
      if (!idx_out || !d_reps) return fail(H3D_ENOMEM, "sort buffers");
      if (int rc = h2d_pinned(ctx, d_reps, rep_idx.data(), (size_t)C * kMaxReps * 4, s))
        return rc;
      const bool k32 = end_bit <= 16;
      // 32-bit keys: (distance, 8-bit min / max count codes), sorted over
      // end_bit + 16 bits (cfg2: 24 bits, three radix passes). (A stable
      // scatter into distance buckets, then each bucket sorted in LDS, gave
      // the same order but measured slower: prep 0.55 -> 1.19 ms per cfg2
      // step, r06aj / r06ak -- the scatter's 4-byte writes to ~250 buckets
      // are uncoalesced (195 us) and the LDS bitonic sorts LDS-bound (555
      // us); the radix passes stage their scatter through LDS.)
      const int cbits = k32 ? 16 : 64 - end_bit;
      const int sort_bits = k32 ? end_bit + 16 : 64;
      // every condition of <= 2 replicates: one key pass for all of them,
      // packed (raw, f) records for the gathers (k_dist_cond_keys_pack2)
      const bool pack = k32 && maxnr <= 2 && ctx->pack_gather;
      int32_t* d_nrep = nullptr;
      CondPack2* packed = nullptr;
      if (pack) {
        d_nrep = (int32_t*)scratch(ctx, "sort_nrep", (size_t)C * 4);
        packed = (CondPack2*)scratch(ctx, "cond_pack2", (size_t)C * n * sizeof(CondPack2));
        if (!d_nrep || !packed) return fail(H3D_ENOMEM, "packed gather rows");
        if (int rc = h2d_pinned(ctx, d_nrep, nrep.data(), (size_t)C * 4, s)) return rc;
      }
      void* keys = scratch(ctx, "dkeys", (pack ? (size_t)C : 1) * n * (k32 ? 4 : 8));
      void* keys_s = scratch(ctx, "dkeys_s", n * (k32 ? 4 : 8));
      if (!keys || !keys_s) return fail(H3D_ENOMEM, "sort keys");
      for (int c = 0; c < C; ++c) {
        const int32_t* reps_c = d_reps + c * kMaxReps;
        uint32_t* keys_c = pack ? (uint32_t*)keys + (size_t)c * n : (uint32_t*)keys;
        if (pack) {
          if (c == 0)
            hipLaunchKernelGGL(k_dist_cond_keys_pack2, dim3(grid_for(ctx, n)), dim3(kBlock),
                               0, s, d_dist, d_raw, d_f, n, R, C, d_reps, d_nrep, keys_c,
                               packed);
        } else if (k32) {
          hipLaunchKernelGGL(k_dist_cond_keys<uint32_t>, dim3(grid_for(ctx, n)),
                             dim3(kBlock), 0, s, d_dist, d_raw, n, R, reps_c, nrep[c],
                             cbits, keys_c);
        }
        if (k32) {
          HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys_c,
                                                     (uint32_t*)keys_s, idx_in, idx_out,
                                                     (int)n, 0, sort_bits, s));
          void* tmp = scratch(ctx, "cub_tmp", tmp_bytes);
          if (!tmp) return fail(H3D_ENOMEM, "sort temp");
          HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys_c,
                                                     (uint32_t*)keys_s, idx_in, idx_out,
                                                     (int)n, 0, sort_bits, s));
          if (c == 0)
            hipLaunchKernelGGL(k_key_dist<uint32_t>, dim3(grid_for(ctx, n)), dim3(kBlock),
                               0, s, (const uint32_t*)keys_s, n, cbits, dist_s);
        } else {
          hipLaunchKernelGGL(k_dist_cond_keys<uint64_t>, dim3(grid_for(ctx, n)),
                             dim3(kBlock), 0, s, d_dist, d_raw, n, R, reps_c, nrep[c],
                             cbits, (uint64_t*)keys);
          HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, (uint64_t*)keys,
                                                     (uint64_t*)keys_s, idx_in, idx_out,
                                                     (int)n, 0, 64, s));
          void* tmp = scratch(ctx, "cub_tmp", tmp_bytes);
          if (!tmp) return fail(H3D_ENOMEM, "sort temp");
          HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, (uint64_t*)keys,
                                                     (uint64_t*)keys_s, idx_in, idx_out,
                                                     (int)n, 0, 64, s));
          if (c == 0)
            hipLaunchKernelGGL(k_key_dist<uint64_t>, dim3(grid_for(ctx, n)), dim3(kBlock),
                               0, s, (const uint64_t*)keys_s, n, cbits, dist_s);
        }
        SoaRows rows;
        for (int j = 0; j < nrep[c]; ++j) {
          const int r = rep_idx[(size_t)c * kMaxReps + j];
          rows.raw[j] = raw_s + (size_t)r * n;
          rows.f[j] = f_s + (size_t)r * n;
        }
        if (pack) {
          hipLaunchKernelGGL(k_gather_pack2, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s,
                             idx_out, packed + (size_t)c * n, n, nrep[c], rows);
          continue;
        }
        const int64_t tiles = (n + kGatherTile - 1) / kGatherTile;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(tiles, (int64_t)ctx->n_cu * 8));
        hipLaunchKernelGGL(k_gather_cond_tile, dim3(grid), dim3(256), 0, s, idx_out, d_raw,
                           d_f, n, R, reps_c, nrep[c], rows);
      }
    } else if (ctx->disp_sort == 1 && end_bit <= 16) {
      // (distance, total count) keys: same segments, less lane divergence;
      // 32-bit keys (16 count bits) whenever the distance fits 16 bits
      constexpr int cbits = 16;
      uint32_t* keys = (uint32_t*)scratch(ctx, "dkeys", n * 4);
      uint32_t* keys_s = (uint32_t*)scratch(ctx, "dkeys_s", n * 4);
      if (!keys || !keys_s) return fail(H3D_ENOMEM, "sort keys");
      hipLaunchKernelGGL(k_dist_count_keys<uint32_t>, dim3(grid_for(ctx, n)), dim3(kBlock),
                         0, s, d_dist, d_raw, n, R, cbits, keys);
      HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys, keys_s,
                                                 idx_in, idx_out, (int)n, 0,
                                                 cbits + end_bit, s));
      void* tmp = scratch(ctx, "cub_tmp", tmp_bytes);
      if (!tmp) return fail(H3D_ENOMEM, "sort temp");
      HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys_s, idx_in,
                                                 idx_out, (int)n, 0, cbits + end_bit, s));
      hipLaunchKernelGGL(k_key_dist<uint32_t>, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s,
                         keys_s, n, cbits, dist_s);
    } else if (ctx->disp_sort == 1) {
      constexpr int cbits = 32;
      uint64_t* keys = (uint64_t*)scratch(ctx, "dkeys", n * 8);
      uint64_t* keys_s = (uint64_t*)scratch(ctx, "dkeys_s", n * 8);
      if (!keys || !keys_s) return fail(H3D_ENOMEM, "sort keys");
      hipLaunchKernelGGL(k_dist_count_keys<uint64_t>, dim3(grid_for(ctx, n)), dim3(kBlock),
                         0, s, d_dist, d_raw, n, R, cbits, keys);
      HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys, keys_s,
                                                 idx_in, idx_out, (int)n, 0,
                                                 cbits + end_bit, s));
      void* tmp = scratch(ctx, "cub_tmp", tmp_bytes);
      if (!tmp) return fail(H3D_ENOMEM, "sort temp");
      HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys_s, idx_in,
                                                 idx_out, (int)n, 0, cbits + end_bit, s));
      hipLaunchKernelGGL(k_key_dist<uint64_t>, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s,
                         keys_s, n, cbits, dist_s);
    } else {
      HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, d_dist, dist_s,
                                                 idx_in, idx_out, (int)n, 0, end_bit, s));
      void* tmp = scratch(ctx, "cub_tmp", tmp_bytes);
      if (!tmp) return fail(H3D_ENOMEM, "sort temp");
      HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, d_dist, dist_s, idx_in,
                                                 idx_out, (int)n, 0, end_bit, s));
    }
    if (ctx->disp_sort != 2) {
      SoaRows rows;
      for (int r = 0; r < R; ++r) {
        rows.raw[r] = raw_s + (size_t)r * n;
        rows.f[r] = f_s + (size_t)r * n;
      }
      hipLaunchKernelGGL(k_gather_soa, dim3(grid_for(ctx, n)), dim3(kBlock), 0, s,
                         idx_out, d_raw, d_f, n, R, rows);
    }
    hipLaunchKernelGGL(k_seg_bounds, dim3((D + 1 + 255) / 256), dim3(256), 0, s,
                       dist_s, n, D, d_seg);
    if (!dev_tables) {
      HIP_TRY(hipMemcpyAsync(seg_start.data(), d_seg, (D + 1) * 8,
                             hipMemcpyDeviceToHost, s));
      stamp("prep launched");
      HIP_TRY(hipStreamSynchronize(s));
      if (seg_start[0] != 0 || seg_start[D] != n) {
        stamp("seg_start synced (dist check failed)");
        // pixels with dist < 0 or >= D
        return fail(H3D_EARG, "dist outside [0, %d)", D);
      }
    } else {
      stamp("prep launched");
    }
  }

  // 2. chunk table
  stamp("seg_start synced");
  std::vector<int64_t> cs;
  std::vector<int32_t> cl, cd, scb(D), sce(D);
  std::vector<SegState> st(S);
  std::vector<int64_t> lpx(S);
  int n_chunks = 0;
  if (dev_tables) {
    n_chunks = (int)std::min<int64_t>(n / kChunk + D + 1, INT32_MAX);  // an upper bound
  } else {
    for (int d = 0; d < D; ++d) {
      scb[d] = (int32_t)cl.size();
      for (int64_t a = seg_start[d]; a < seg_start[d + 1]; a += kChunk) {
        cs.push_back(a);
        cl.push_back((int32_t)std::min<int64_t>(kChunk, seg_start[d + 1] - a));
        cd.push_back(d);
      }
      sce[d] = (int32_t)cl.size();
    }
    n_chunks = (int)cl.size();

    // global pixel counts per segment (all ranks)
    std::vector<double> cnt(S, 0.0);
    for (int d = 0; d < D; ++d)
      for (int c = 0; c < C; ++c) cnt[d * C + c] = (double)(seg_start[d + 1] - seg_start[d]);
    double* d_cnt = (double*)scratch(ctx, "seg_cnt", S * 8);
    if (!d_cnt) return fail(H3D_ENOMEM, "seg_cnt");
    if (reduce) {
      HIP_TRY(hipMemcpyAsync(d_cnt, cnt.data(), S * 8, hipMemcpyHostToDevice, s));
      if (reduce(d_cnt, S, user)) return fail(H3D_EHIP, "allreduce callback failed");
      HIP_TRY(hipMemcpyAsync(cnt.data(), d_cnt, S * 8, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
    }
    for (int sg = 0; sg < S; ++sg)
      seg_init(&st[sg], (long long)cnt[sg], nrep[sg % C], ctx->qcml_tol);
    for (int d = 0; d < D; ++d)
      for (int c = 0; c < C; ++c) lpx[d * C + c] = seg_start[d + 1] - seg_start[d];
  }

  // the per-call tables go up as ONE copy from a pinned staging buffer (nine
  // pageable copies cost ~0.3 ms of host-side gaps per cfg2 step: each
  // staged and launched its own blit)
  std::vector<int32_t> nrep32(nrep.begin(), nrep.end());
  struct Part {
    const void* src;
    size_t bytes, off;
  };
  // (dev_tables: the chunk / segment tables are k_disp_tables' outputs, only
  // their room is reserved and nothing of them is copied)
  const size_t nch = (size_t)std::max(n_chunks, 1);
  Part parts[] = {{cs.data(), nch * 8, 0},               {cl.data(), nch * 4, 0},
                  {cd.data(), nch * 4, 0},               {scb.data(), (size_t)D * 4, 0},
                  {sce.data(), (size_t)D * 4, 0},        {nrep32.data(), (size_t)C * 4, 0},
                  {rep_idx.data(), rep_idx.size() * 4, 0},
                  {st.data(), (size_t)S * sizeof(SegState), 0},
                  {lpx.data(), (size_t)S * 8, 0}};
  size_t blob = 0;
  for (Part& q : parts) {
    q.off = blob;
    blob += (q.bytes + 255) & ~(size_t)255;
  }
  // the bytes that go up: everything, or (dev_tables) nrep + rep_idx only
  const size_t up_lo = dev_tables ? parts[5].off : 0;
  const size_t up_hi = dev_tables ? parts[7].off : blob;
  if (!ctx->h_stage_done)
    HIP_TRY(hipEventCreateWithFlags(&ctx->h_stage_done, hipEventDisableTiming));
  else
    HIP_TRY(hipEventSynchronize(ctx->h_stage_done));  // the previous copy has read it
  if (ctx->h_stage_bytes < blob) {
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    ctx->h_stage = nullptr;
    ctx->h_stage_bytes = 0;
    HIP_TRY(hipHostMalloc(&ctx->h_stage, blob, hipHostMallocDefault));
    ctx->h_stage_bytes = blob;
  }
  char* d_blob = (char*)scratch(ctx, "disp_tables", blob);
  if (!d_blob) return fail(H3D_ENOMEM, "disp tables");
  for (int qi = dev_tables ? 5 : 0; qi < (dev_tables ? 7 : 9); ++qi)
    if (parts[qi].bytes)
      std::memcpy((char*)ctx->h_stage + parts[qi].off, parts[qi].src, parts[qi].bytes);
  HIP_TRY(hipMemcpyAsync(d_blob + up_lo, (char*)ctx->h_stage + up_lo, up_hi - up_lo,
                         hipMemcpyHostToDevice, s));
  HIP_TRY(hipEventRecord(ctx->h_stage_done, s));
  int64_t* d_cs = (int64_t*)(d_blob + parts[0].off);
  int32_t* d_cl = (int32_t*)(d_blob + parts[1].off);
  int32_t* d_cd = (int32_t*)(d_blob + parts[2].off);
  int32_t* d_scb = (int32_t*)(d_blob + parts[3].off);
  int32_t* d_sce = (int32_t*)(d_blob + parts[4].off);
  int32_t* d_nrep = (int32_t*)(d_blob + parts[5].off);
  int32_t* d_repidx = (int32_t*)(d_blob + parts[6].off);
  SegState* d_st = (SegState*)(d_blob + parts[7].off);
  int64_t* d_lpx = (int64_t*)(d_blob + parts[8].off);
  const size_t max_items = (size_t)std::max(n_chunks, 1) * C;
  int32_t* d_list = (int32_t*)scratch(ctx, "work_list", max_items * 4);
  // len, active, eq_len, live; k_disp_work's task heads (kTaskHeadStride apart)
  int32_t* d_meta = (int32_t*)scratch(ctx, "work_meta", kWorkMetaInts * 4);
  int32_t* d_slb = (int32_t*)scratch(ctx, "seg_lb", S * 4);
  int32_t* d_sle = (int32_t*)scratch(ctx, "seg_le", S * 4);
  double* d_partial = (double*)scratch(ctx, "partial", max_items * 8 * kWavesPerBlock);
  double* d_total = (double*)scratch(ctx, "seg_total", S * 8);
  int* d_flags = (int*)scratch(ctx, "seg_flags", S * 4);
  double* d_res = (double*)scratch(ctx, "seg_result", S * 8);
  if (!d_cs || !d_cl || !d_cd || !d_scb || !d_sce || !d_nrep || !d_repidx ||
      !d_st || !d_lpx || !d_list || !d_meta || !d_slb || !d_sle || !d_partial ||
      !d_total || !d_flags || !d_res)
    return fail(H3D_ENOMEM, "disp scratch");
  if (!dev_tables) HIP_TRY(hipMemsetAsync(d_flags, 0, S * 4, s));  // else k_disp_tables
  int* d_bad = (int*)scratch(ctx, "dist_bad", 4);
  if (!d_bad) return fail(H3D_ENOMEM, "dist_bad");
  // (an M = 6 instantiation for cfg4's R_c = 6 measured equal to M = 8:
  // 111.5 vs 110.5 ms equalize per step, profiles/r02/q2)
  const int mslot = (maxnr <= 2 && ctx->disp_m2) ? 2
                    : maxnr <= 4                  ? 4
                    : maxnr <= 8                  ? 8
                    : maxnr <= 16                 ? 16
                                                  : 32;
  // dev_tables, single rank: k_brent and k_brent_gang are both launched every
  // qcml iteration and the DEVICE picks one by the live-segment count (one
  // workgroup per segment while they fill the CUs, gangs for the tail
  // iterations, whose few live segments left most CUs idle: cfg2's fourth
  // iteration ran ~55 searches on 55 CUs for 0.36 ms); the gang task table
  // comes from k_disp_tables
  GangTables gang;
  const bool dual = dev_tables && !reduce && ctx->brent_gang == 1;
  if (dual) {
    const int grc = mslot == 2    ? gang_setup_dev<2>(ctx, n, D, C, &gang)
                    : mslot == 4  ? gang_setup_dev<4>(ctx, n, D, C, &gang)
                    : mslot == 8  ? gang_setup_dev<8>(ctx, n, D, C, &gang)
                    : mslot == 16 ? gang_setup_dev<16>(ctx, n, D, C, &gang)
                                  : gang_setup_dev<32>(ctx, n, D, C, &gang);
    if (grc) return grc;
  }
  if (dev_tables) {
    const int64_t* d_seg0 = (const int64_t*)scratch(ctx, "seg_start", (D + 1) * 8);
    hipLaunchKernelGGL(k_disp_tables, dim3(1), dim3(1024), 0, s, d_seg0, D, C, n, d_nrep,
                       d_cs, d_cl, d_cd, d_scb, d_sce, d_st, d_lpx, d_bad,
                       dual ? gang.P : (int64_t)1, dual ? gang.task_seg : nullptr,
                       dual ? gang.task_g : nullptr, ctx->qcml_tol, dual ? gang.T : 0,
                       d_flags, dual ? gang.abort : nullptr);
    dbg_launch("k_disp_tables");
  }
  stamp("tables uploaded");

  // the single-rank Brent kernels' work queues, zeroed by k_seg_update
  int* d_queue = (int*)scratch(ctx, "brent_queue", 2 * sizeof(int));
  if (!d_queue) return fail(H3D_ENOMEM, "brent queue");
  // initial active list
  hipLaunchKernelGGL(k_seg_update, dim3(1), dim3(1024), 0, s, d_st, d_total,
                     d_flags, S, C, d_nrep, d_scb, d_sce, d_list, d_slb, d_sle,
                     d_res, d_meta, 1, 0, d_lpx, ctx->work_count, d_queue,
                     dual ? gang.P : (int64_t)1, dual ? gang.task_seg : nullptr,
                     dual ? gang.task_g : nullptr);
  if (!ctx->h_meta) HIP_TRY(hipHostMalloc((void**)&ctx->h_meta, 32, hipHostMallocDefault));
  int32_t* h_meta = ctx->h_meta;
  const size_t res_bytes = (size_t)S * 8 + (size_t)S * sizeof(SegState) + 8;
  if (ctx->h_res_bytes < res_bytes) {
    if (ctx->h_res) (void)hipHostFree(ctx->h_res);
    ctx->h_res = nullptr;
    ctx->h_res_bytes = 0;
    HIP_TRY(hipHostMalloc(&ctx->h_res, res_bytes, hipHostMallocDefault));
    ctx->h_res_bytes = res_bytes;
  }
  double* h_resd = (double*)ctx->h_res;
  SegState* h_sst = (SegState*)(h_resd + S);
  int* h_bad = (int*)(h_sst + S);
  *h_bad = 0;
  bool have_res = false;  // the results of the final poll are in h_res
  int rounds = 0, batch = 2, rc = 0;
  if (!reduce) {
    // Single rank: one equalize pass per qcml iteration over every segment
    // that needs one, then k_brent runs each such segment's whole Brent
    // search in-kernel, then k_seg_update rebuilds the equalize list. The
    // host polls the live-segment count every `batch` iterations (an
    // iteration with nothing to do costs three empty launches).
    int64_t* d_seg = (int64_t*)scratch(ctx, "seg_start", (D + 1) * 8);
    if (!d_seg) return fail(H3D_ENOMEM, "brent scratch");
    if (n == 0) HIP_TRY(hipMemsetAsync(d_seg, 0, (D + 1) * 8, s));
    // H3D_BRENT: 1 (default) = gang searches (k_brent_gang) when the
    // segments are fewer than the CUs, 2 = always, 0 = one workgroup per
    // segment (k_brent)
    bool use_gang = ctx->brent_gang != 0 && n > 0 && !dev_tables;
    bool dual_on = dual;
    if (use_gang) {
      int grc = mslot == 2   ? gang_setup<2>(ctx, seg_start, D, C, &gang)
                : mslot == 4 ? gang_setup<4>(ctx, seg_start, D, C, &gang)
                : mslot == 8 ? gang_setup<8>(ctx, seg_start, D, C, &gang)
                : mslot == 16 ? gang_setup<16>(ctx, seg_start, D, C, &gang)
                              : gang_setup<32>(ctx, seg_start, D, C, &gang);
      if (grc == 1) use_gang = false;
      else if (grc) return grc;
    }
    // first poll after 5 iterations (cfg2's searches end after 5; a poll is
    // a host sync plus the relaunch latency, ~50 us of idle GPU -- r03 host
    // stamps), then every 2
    batch = 5;
    while (true) {
      for (int b = 0; b < batch; ++b) {
#define H3D_QCML_ITER(MM)                                                                 \
  launch_disp_work<MM, false>(ctx, max_items, raw_s, f_s, pd, n, d_cs, d_cl, d_cd, C,     \
                              d_repidx, d_nrep, d_st, d_flags, d_list, d_meta, d_partial); \
  dbg_launch("equalize");                                                                 \
  if (dual_on) {                                                                          \
    launch_brent<MM>(ctx, pd, n, d_seg, S, C, d_repidx, d_nrep, d_st, d_flags, d_res,      \
                     d_queue, d_meta, ctx->n_cu, gang.abort, true);                        \
    dbg_launch("k_brent (dual)");                                                         \
    launch_brent_gang<MM>(ctx, pd, n, d_seg, S, C, d_repidx, d_nrep, d_st, d_flags, d_res, \
                          d_queue + 1, gang, d_meta, ctx->n_cu, true);                    \
    dbg_launch("k_brent_gang (dual)");                                                    \
  } else if (use_gang)                                                                    \
    launch_brent_gang<MM>(ctx, pd, n, d_seg, S, C, d_repidx, d_nrep, d_st, d_flags, d_res, \
                          d_queue + 1, gang, nullptr, 0, true);                           \
  else                                                                                    \
    launch_brent<MM>(ctx, pd, n, d_seg, S, C, d_repidx, d_nrep, d_st, d_flags, d_res,      \
                     d_queue, nullptr, 0, nullptr, true)
        dbg_launch("before qcml iteration");
        if (mslot == 2) { H3D_QCML_ITER(2); }
        else if (mslot == 4) { H3D_QCML_ITER(4); }
        else if (mslot == 8) { H3D_QCML_ITER(8); }
        else if (mslot == 16) { H3D_QCML_ITER(16); }
        else { H3D_QCML_ITER(32); }
#undef H3D_QCML_ITER
        {
          ProfScope ps(ctx, "disp_update", 0);
          hipLaunchKernelGGL(k_seg_update, dim3(1), dim3(1024), 0, s, d_st, d_total,
                             d_flags, S, C, d_nrep, d_scb, d_sce, d_list, d_slb, d_sle,
                             d_res, d_meta, 0, 0, d_lpx, ctx->work_count, d_queue,
                             dual_on ? gang.P : (int64_t)1,
                             dual_on ? gang.task_seg : nullptr,
                             dual_on ? gang.task_g : nullptr);
        }
        ++rounds;
      }
      // the poll, and speculatively what follows a final one: the result
      // copies (pinned) and the requested smoother behind them, so a final
      // poll costs one host round trip (r03s trace: ~0.12 ms of host gaps
      // after the fifth iteration); a poll that finds live segments simply
      // runs them, and a later poll redoes both
      hipEvent_t copied = ev_get(ctx);
      if (hipMemcpyAsync(h_meta, d_meta, 16, hipMemcpyDeviceToHost, s) != hipSuccess ||
          ((use_gang || dual_on) &&
           hipMemcpyAsync(h_meta + 4, gang.abort, 4, hipMemcpyDeviceToHost, s) != hipSuccess) ||
          hipMemcpyAsync(h_resd, d_res, (size_t)S * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipMemcpyAsync(h_sst, d_st, (size_t)S * sizeof(SegState), hipMemcpyDeviceToHost, s) !=
              hipSuccess ||
          (dev_tables && hipMemcpyAsync(h_bad, d_bad, 4, hipMemcpyDeviceToHost, s) != hipSuccess) ||
          hipEventRecord(copied, s) != hipSuccess) {
        ctx->event_pool.push_back(copied);
        rc = fail(H3D_EHIP, "disp round copies failed: %s", hipGetErrorString(hipGetLastError()));
        break;
      }
      // (speculatively only where the smoother is the device's, enqueued
      // without a wait; the host smoother of D > kTableMaxD runs once, on
      // the final result, below -- on an intermediate poll it would block
      // and could reject a table that is not final)
      if (treq && D <= kTableMaxD) {
        rc = h3d_disp_tables_dev(ctx, d_res, D, C, treq->weighted, treq->frac, treq->aff,
                                 treq->d_tables);
        if (rc) {
          (void)hipEventSynchronize(copied);
          ctx->event_pool.push_back(copied);
          break;
        }
      }
      const hipError_t ce = hipEventSynchronize(copied);
      ctx->event_pool.push_back(copied);
      if (ce != hipSuccess) {
        rc = fail(H3D_EHIP, "disp round sync failed: %s", hipGetErrorString(ce));
        break;
      }
      have_res = true;
      stamp("poll");
      if (std::getenv("H3D_DEBUG"))
        fprintf(stderr, "[h3d] qcml iterations=%d live_segments=%d gang=%d abort=%d\n",
                rounds, h_meta[3], use_gang ? 1 : dual_on ? 2 : 0,
                (use_gang || dual_on) ? h_meta[4] : 0);
      if (dual_on && h_meta[4]) {
        // a gang aborted: k_brent (gated on the same flag) already took over
        // the following iterations on the device; launch it alone from here
        dual_on = false;
        ctx->gang_aborts += 1;
      }
      if (use_gang && h_meta[4]) {
        // a gang's wait timed out (CUs held elsewhere): its segments stayed
        // in kEqualize and repeat their iteration; finish with k_brent
        use_gang = false;
        ctx->gang_aborts += 1;
        continue;
      }
      if (h_meta[3] == 0) break;
      if (rounds > 2000) {
        rc = fail(H3D_ENOCONV, "estimate_disp did not terminate");
        break;
      }
      batch = 2;
    }
  }
  while (reduce && !rc) {
    for (int b = 0; b < batch; ++b) {
      {
        // every width the single-rank driver picks (mslot 2 fell through to
        // the M = 32 instantiation here: 13.1 vs 5.5 ms of equalize per cfg2
        // step, bench --noop-reduce)
        switch (mslot) {
          case 2:
            launch_disp_work<2, true>(ctx, max_items, raw_s, f_s, pd, n, d_cs, d_cl, d_cd, C, d_repidx, d_nrep, d_st, d_flags, d_list, d_meta, d_partial);
            break;
          case 4:
            launch_disp_work<4, true>(ctx, max_items, raw_s, f_s, pd, n, d_cs, d_cl, d_cd, C, d_repidx, d_nrep, d_st, d_flags, d_list, d_meta, d_partial);
            break;
          case 8:
            launch_disp_work<8, true>(ctx, max_items, raw_s, f_s, pd, n, d_cs, d_cl, d_cd, C, d_repidx, d_nrep, d_st, d_flags, d_list, d_meta, d_partial);
            break;
          case 16:
            launch_disp_work<16, true>(ctx, max_items, raw_s, f_s, pd, n, d_cs, d_cl, d_cd, C, d_repidx, d_nrep, d_st, d_flags, d_list, d_meta, d_partial);
            break;
          default:
            launch_disp_work<32, true>(ctx, max_items, raw_s, f_s, pd, n, d_cs, d_cl, d_cd, C, d_repidx, d_nrep, d_st, d_flags, d_list, d_meta, d_partial);
        }
      }
      {
        ProfScope ps(ctx, "disp_reduce", 0);
        // this rank's per-segment sums; the cross-rank all-reduce follows and
        // k_seg_update steps the (identical) state machines
        hipLaunchKernelGGL(k_seg_reduce, dim3((S + 3) / 4), dim3(256), 0, s,
                           d_partial, d_slb, d_sle, S, d_total, nullptr, d_flags,
                           d_nrep, C, d_res);
      }
      if (reduce(d_total, S, user)) {
        rc = fail(H3D_EHIP, "allreduce callback failed");
        break;
      }
      {
        ProfScope ps(ctx, "disp_update", 0);
        hipLaunchKernelGGL(k_seg_update, dim3(1), dim3(1024), 0, s, d_st, d_total,
                           d_flags, S, C, d_nrep, d_scb, d_sce, d_list, d_slb,
                           d_sle, d_res, d_meta, 0, 1, d_lpx, ctx->work_count, nullptr);
      }
      ++rounds;
    }
    if (rc) break;
    if (hipMemcpyAsync(h_meta, d_meta, 16, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      rc = fail(H3D_EHIP, "disp round sync failed: %s", hipGetErrorString(hipGetLastError()));
      break;
    }
    if (std::getenv("H3D_DEBUG"))
      fprintf(stderr, "[h3d] disp rounds=%d active_items=%d live_segments=%d\n", rounds,
              h_meta[1], h_meta[3]);
    // terminate on the genome-wide live-segment count (identical on every
    // rank), not on this rank's own work-list length: a rank without pixels
    // in the still-active segments must keep joining the collective reduce
    if (h_meta[3] == 0) break;
    if (rounds > 200000) {
      rc = fail(H3D_ENOCONV, "estimate_disp did not terminate");
      break;
    }
    batch = std::min(batch * 2, 8);
  }
  if (rc) return rc;
  // a launch error of the qcml loop is this call's, not a later call's
  HIP_TRY(hipGetLastError());
  std::vector<int32_t> fl(S);
  if (!have_res) {
    // (the multi-rank path) the results into the pinned zone; the smoother
    // runs behind the copies, the host waits for the copies only
    HIP_TRY(hipMemcpyAsync(h_resd, d_res, (size_t)S * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(h_sst, d_st, (size_t)S * sizeof(SegState), hipMemcpyDeviceToHost, s));
    if (dev_tables) HIP_TRY(hipMemcpyAsync(h_bad, d_bad, 4, hipMemcpyDeviceToHost, s));
    hipEvent_t copied = ev_get(ctx);
    HIP_TRY(hipEventRecord(copied, s));
    const int trc = treq ? h3d_disp_tables_dev(ctx, d_res, D, C, treq->weighted, treq->frac,
                                               treq->aff, treq->d_tables)
                         : 0;
    const hipError_t e = hipEventSynchronize(copied);
    ctx->event_pool.push_back(copied);
    if (trc) return trc;
    if (e != hipSuccess) return fail(H3D_EHIP, "result copy: %s", hipGetErrorString(e));
  }
  std::memcpy(disp_per_dist, h_resd, (size_t)S * 8);
  std::memcpy(st.data(), h_sst, (size_t)S * sizeof(SegState));
  ctx->last_S = S;
  const int bad = dev_tables ? *h_bad : 0;
  stamp("results");
  if (bad) return fail(H3D_EARG, "dist outside [0, %d)", D);
  int all = 0;
  for (int sg = 0; sg < S; ++sg) {
    fl[sg] = st[sg].flags;
    all |= fl[sg];
  }
  if (seg_flags_out) std::memcpy(seg_flags_out, fl.data(), S * 4);
  if (const int frc = flags_to_code(all)) return frc;
  if (have_res && treq && D > kTableMaxD) {
    // the host smoother (h3d_disp_tables_dev's D > kTableMaxD branch), once,
    // on the final result
    const int trc = h3d_disp_tables_dev(ctx, d_res, D, C, treq->weighted, treq->frac,
                                        treq->aff, treq->d_tables);
    if (trc) return trc;
  }
  return 0;
}
}  // namespace

int h3d_disp_per_dist(h3d_ctx* ctx, const int64_t* raw, const double* f,
                      const int32_t* dist, int64_t n, int R, int C,
                      const int32_t* cond_of_rep, int D, int estimator,
                      double* disp_per_dist, int32_t* seg_flags) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  if (n > 0 && (!raw || !f || !dist)) return fail(H3D_EARG, "null input");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  int32_t* d_raw = nullptr;
  double* d_f = nullptr;
  int32_t* d_dist = nullptr;
  if (n > 0) {
    int64_t* d_raw64 = (int64_t*)scratch(ctx, "in_raw64", n * R * 8);
    d_raw = (int32_t*)scratch(ctx, "in_raw", n * R * 4);
    d_f = (double*)scratch(ctx, "in_f", n * R * 8);
    d_dist = (int32_t*)scratch(ctx, "in_dist", n * 4);
    int* d_ovf = (int*)scratch(ctx, "ovf", 4);
    if (!d_raw64 || !d_raw || !d_f || !d_dist || !d_ovf) return fail(H3D_ENOMEM, "inputs");
    HIP_TRY(hipMemcpyAsync(d_raw64, raw, n * R * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_f, f, n * R * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_dist, dist, n * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(d_ovf, 0, 4, s));
    hipLaunchKernelGGL(k_i64_to_i32, dim3(grid_for(ctx, n * R)), dim3(kBlock), 0, s,
                       d_raw64, d_raw, n * R, d_ovf);
    int ovf = 0;
    HIP_TRY(hipMemcpyAsync(&ovf, d_ovf, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (ovf) return fail(H3D_EINPUT, "raw counts must be in [0, 2^31)");
  }
  return h3d_disp_per_dist_dev(ctx, d_raw, d_f, d_dist, n, R, C, cond_of_rep, D,
                               estimator, disp_per_dist, seg_flags, nullptr, nullptr);
}

int h3d_disp_table(const double* col, int D, int weighted, double frac,
                   double auto_frac_factor, double* table_out) {
  if (!col || !table_out || D < 1) return fail(H3D_EARG, "null argument / D");
  std::vector<double> x, y, xs(D);
  for (int d = 0; d < D; ++d) {
    xs[d] = d;
    if (std::isfinite(col[d])) {
      x.push_back(d);
      y.push_back(col[d]);
    }
  }
  if (x.size() < 2) return fail(H3D_EARG, "fewer than two finite dispersion points");
  std::vector<double> out;
  int rc;
  if (weighted)
    rc = h3dhost::weighted_lowess_fit_eval(x, y, y[0], frac, auto_frac_factor, xs, &out,
                                           /*pinned_min_weight=*/weighted != 2);
  else
    rc = h3dhost::lowess_fit_eval(x, y, y[0], frac >= 0 ? frac : 0.3, 0.01, xs, &out);
  if (rc) return fail(H3D_ENOCONV, "lowess fit failed (degenerate dispersion table)");
  std::memcpy(table_out, out.data(), D * 8);
  return 0;
}

// every condition's table in one call: (D, C) row-major in and out, one
// host thread per condition (the smoother is serial per condition); one
// ctypes call instead of a Python thread pool, whose dispatch cost more than
// the smoothing (r03: 1.36 ms for two conditions vs 0.75 ms in sequence on
// the container's CPU)
int h3d_disp_tables(const double* disp_per_dist, int D, int C, int weighted,
                    double frac, double auto_frac_factor, double* tables_out) {
  if (!disp_per_dist || !tables_out || D < 1 || C < 1 || C > kMaxConds)
    return fail(H3D_EARG, "null argument / D / C");
  std::vector<std::vector<double>> cols(C, std::vector<double>(D)), outs(C, std::vector<double>(D));
  for (int c = 0; c < C; ++c)
    for (int d = 0; d < D; ++d) cols[c][d] = disp_per_dist[(size_t)d * C + c];
  std::vector<int> rcs(C, 0);
  std::vector<std::string> errs(C);
  auto one = [&](int c) {
    rcs[c] = h3d_disp_table(cols[c].data(), D, weighted, frac, auto_frac_factor,
                            outs[c].data());
    if (rcs[c]) errs[c] = h3derr::last();   // the message is thread-local
  };
  std::vector<std::thread> pool;
  for (int c = 1; c < C; ++c) pool.emplace_back(one, c);
  one(0);
  for (auto& t : pool) t.join();
  for (int c = 0; c < C; ++c)
    if (rcs[c]) return fail(rcs[c], "condition %d: %s", c, errs[c].c_str());
  for (int c = 0; c < C; ++c)
    for (int d = 0; d < D; ++d) tables_out[(size_t)d * C + c] = outs[c][d];
  return 0;
}

int h3d_disp_seg_stats(h3d_ctx* ctx, int S, int32_t* qiter, int32_t* evals) {
  if (!ctx) return fail(H3D_EARG, "null ctx");
  if (S != ctx->last_S || !ctx->h_res)
    return fail(H3D_EARG, "no estimate_disp result of %d segments (last: %d)", S, ctx->last_S);
  const SegState* h_sst = (const SegState*)((const double*)ctx->h_res + S);
  for (int s = 0; s < S; ++s) {
    if (qiter) qiter[s] = h_sst[s].qiter;
    if (evals) evals[s] = h_sst[s].evals;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// cml on given data (util/dispersion.py:46-80)
// ---------------------------------------------------------------------------

int h3d_cml(h3d_ctx* ctx, const double* data, int64_t n, int r, double* disp_out) {
  if (!ctx || !data || !disp_out) return fail(H3D_EARG, "null argument");
  if (n < 1 || r < 1 || r > kMaxReps) return fail(H3D_EARG, "n=%lld r=%d", (long long)n, r);
  if (n >= (int64_t)1 << 31) return fail(H3D_EARG, "n too large");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  // replicate-major (SoA) copy of the data: the pseudodata layout k_brent reads
  std::vector<double> soa((size_t)n * r);
  for (int64_t i = 0; i < n; ++i)
    for (int k = 0; k < r; ++k) soa[(size_t)k * n + i] = data[i * r + k];
  SegState st;
  seg_init(&st, n, r);  // phase kEqualize: the first evaluation is at x0
  std::vector<int32_t> rep_idx(kMaxReps);
  for (int k = 0; k < kMaxReps; ++k) rep_idx[k] = k;
  const int64_t seg[2] = {0, n};
  const int32_t nrep = r;
  double* d_pd = (double*)scratch(ctx, "cml_pd", (size_t)n * r * 8);
  int64_t* d_seg = (int64_t*)scratch(ctx, "cml_seg", 16);
  int32_t* d_ri = (int32_t*)scratch(ctx, "cml_ri", kMaxReps * 4);
  int32_t* d_nr = (int32_t*)scratch(ctx, "cml_nr", 4);
  SegState* d_st = (SegState*)scratch(ctx, "cml_st", sizeof(SegState));
  int* d_fl = (int*)scratch(ctx, "cml_fl", 4);
  double* d_res = (double*)scratch(ctx, "cml_res", 8);
  int* d_q = (int*)scratch(ctx, "cml_queue", 4);
  if (!d_pd || !d_seg || !d_ri || !d_nr || !d_st || !d_fl || !d_res || !d_q)
    return fail(H3D_ENOMEM, "cml scratch");
  HIP_TRY(hipMemcpyAsync(d_pd, soa.data(), soa.size() * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_seg, seg, 16, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_ri, rep_idx.data(), kMaxReps * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_nr, &nrep, 4, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_st, &st, sizeof(SegState), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(d_fl, 0, 4, s));
  const int m = r <= 4 ? 4 : r <= 8 ? 8 : r <= 16 ? 16 : 32;
  if (m == 4) launch_brent<4>(ctx, d_pd, n, d_seg, 1, 1, d_ri, d_nr, d_st, d_fl, d_res, d_q);
  else if (m == 8) launch_brent<8>(ctx, d_pd, n, d_seg, 1, 1, d_ri, d_nr, d_st, d_fl, d_res, d_q);
  else if (m == 16) launch_brent<16>(ctx, d_pd, n, d_seg, 1, 1, d_ri, d_nr, d_st, d_fl, d_res, d_q);
  else launch_brent<32>(ctx, d_pd, n, d_seg, 1, 1, d_ri, d_nr, d_st, d_fl, d_res, d_q);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(&st, d_st, sizeof(SegState), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (st.flags & kFlagBrentFail)
    return fail(H3D_ENOCONV, "bounded minimisation failed (reference: assert res.success)");
  // the search ended in seg_step's qcml update: disp = delta / (1 - delta)
  *disp_out = st.disp;
  return 0;
}

// ---------------------------------------------------------------------------
// bh
// ---------------------------------------------------------------------------

int h3d_bh(const double* p, int64_t n, double* q) {
  if (n < 0 || (n > 0 && (!p || !q))) return fail(H3D_EARG, "null argument");
  h3dhost::bh(p, n, q);
  return 0;
}

}  // extern "C"

