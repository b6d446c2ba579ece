// libh3d internals shared by its HIP translation units (h3d_api.hip: the hot
// path; h3d_alt.hip: the alternative models): the context behind the C ABI's
// opaque h3d_ctx handle and the launch helpers. Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "h3d.h"
#include "h3d_errors.h"

#define HIP_TRY(expr)                                                      \
  do {                                                                     \
    hipError_t e_ = (expr);                                                \
    if (e_ != hipSuccess)                                                  \
      return h3derr::fail(H3D_EHIP, "%s failed: %s (%s:%d)", #expr,        \
                          hipGetErrorString(e_), __FILE__, __LINE__);      \
  } while (0)

namespace h3d {

// prepare_data state between h3d_union_count and h3d_union_fill
struct PrepUnion {
  int R = 0, n_bins = 0;
  int64_t n_entries = 0, n_px = 0;
  // device
  int64_t* keys_sorted = nullptr;  // n_entries
  int32_t* ent_sorted = nullptr;   // n_entries
  int32_t* run_of = nullptr;       // n_entries (exclusive-scanned heads)
  int32_t* px_of_run = nullptr;    // runs -> pixel (or -1)
  int64_t* run_start = nullptr;    // runs + 1
  double* ent_val = nullptr;       // raw value per entry (summed duplicates not needed: canonical CSR)
  int32_t* ent_rep = nullptr;      // replicate per entry
  double* bias = nullptr;          // (n_bins, R)
  int64_t n_runs = 0;
};

}  // namespace h3d

namespace h3dint {

struct ProfEntry {
  double ms = 0.0;
  int64_t launches = 0;
  int64_t units = 0;
};

// a device dispersion table enqueued by h3d_disp_tables_dev whose status
// has not been read yet (h3d_lrt_dev_tab / h3d_disp_tables_wait settle it)
struct TablePending {
  const double* dpd = nullptr;
  double* tables = nullptr;
  int D = 0, C = 0, weighted = 1;
  double frac = -1.0, aff = 15.0;
  int active = 0, on_host = 0;
};

}  // namespace h3dint

struct h3d_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  int n_cu = 256;
  std::map<const void*, int> resident;  // kernel -> resident workgroups / CU
  // 0 off; 1: the roofline kernels only ("disp_work", "lrt"); 2: every
  // scope. Events are collected lazily (profile_read / reset / close), so
  // the launch path never waits on them.
  int prof = 0;
  std::map<std::string, h3dint::ProfEntry> stats;
  std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<int64_t> pending_units;
  std::vector<hipEvent_t> event_pool;
  // grow-only device scratch, by slot
  std::map<std::string, std::pair<void*, size_t>> bufs;
  // prepare_data state between h3d_union_count and h3d_union_fill
  h3d::PrepUnion prep;
  // [equalize, nll] pixel-replicates processed by disp_work (measurement)
  unsigned long long* work_count = nullptr;
  // pinned host word the disp loop polls (active work items), kept for the
  // ctx's lifetime (a per-call hipHostFree would synchronise the device)
  int32_t* h_meta = nullptr;
  // pinned staging of estimate_disp's per-call tables (one H2D copy)
  void* h_stage = nullptr;
  size_t h_stage_bytes = 0;
  // pinned landing zone of estimate_disp's results (per-segment dispersion,
  // state, the distance check): pageable device-to-host copies blocked the
  // host one after another at the end of every call
  void* h_res = nullptr;
  size_t h_res_bytes = 0;
  // recorded after each H2D copy out of h_stage: the next call waits on it
  // before rewriting (or freeing) the buffer, whichever way the last call
  // returned
  hipEvent_t h_stage_done = nullptr;
  // pinned bounce buffers for the small host<->device copies of the host
  // entry points (h2d_pinned / pinned_rd): a copy from or to pageable memory
  // is staged by the HIP runtime behind every other pageable copy in flight
  // -- e.g. the class's background result copies -- and a 4-byte flag read
  // waited tens of ms behind them (r06an)
  void* bounce = nullptr;
  size_t bounce_cap = 0, bounce_off = 0;
  hipEvent_t bounce_ev = nullptr;
  hipStream_t bounce_stream = nullptr;
  void* land = nullptr;
  size_t land_cap = 0;
  // tuning knobs (env at h3d_open): H3D_DISP_W = min waves/SIMD of the
  // disp_work register budget (1, 2, 3, 4); H3D_DISP_SORT = 0 (distance) or
  // 1 (distance, total count)
  int disp_w = 4;  // measured best (sweep at 7413b12, equalize ms/step for
                   // W 1/2/3/4: 10.7 / 10.55 / 9.76 / 9.62)
  // H3D_DISP_SORT: pixel order inside a distance segment. 0 position, 1
  // (total count) -- r01: 55.6 -> 52.5 ms --, 2 one (max, min count) order
  // per condition -- r02 cfg2: equalize 7.62 -> 5.68 ms, 277 -> 311 Mpx/s;
  // cfg4 equalize 118 -> 111 ms (profiles/r02/sortab)
  int disp_sort = 2;
  int nll_w = 1;  // H3D_NLL_W: min waves/SIMD of the NLL-only pass (1, 2, 4)
  // H3D_DISP_M2 / _W2: the M = 2 instantiation for R_c <= 2 and its
  // equalize register budget. r02 cfg2 (10 steps, two runs): M = 4 305 / 316
  // Mpx/s; M = 2 at W 4 / 5 / 6: 320 (327) / 317 / 307 -- the gain is
  // k_brent<2> (3.5 vs 3.9 ms), equalize is unchanged (same VGPR profile)
  int disp_w2 = 4;
  // k_disp_work: eighths of the task rounds dealt statically (the rest from
  // a device counter); H3D_EQ_STATIC8
  int eq_static8 = 4;
  // H3D_PACK_GATHER: a condition of <= 2 replicates gathers from a 32-byte
  // packed copy of its replicates' (raw, f) written by the key pass (one
  // sector per pixel instead of a raw and an f line)
  int pack_gather = 1;
  int disp_m2 = 1;
  // H3D_BRENT: 1 = gang Brent searches (k_brent_gang) where one workgroup
  // per segment leaves CUs idle, 2 = always, 0 = k_brent only
  int brent_gang = 1;
  int gang_aborts = 0;  // gang waits that timed out (fell back to k_brent)
  // H3D_BRENT_LDS_KB: LDS per k_brent workgroup for the segment's staged
  // head (0 = stream every evaluation from memory). With the log table in
  // LDS too, r03am: 64 / 96 / 128 KB 2.62-2.66 ms of Brent per cfg2 step,
  // 80 / 112 / 144 KB 2.73-2.80 (the replicate rows' LDS stride), 0 KB 2.67
  int brent_lds_kb = 128;
  double qcml_tol = 1e-4;  // h3d_set_qcml_tol (qcml's tol, dispersion.py:10)
  // gang Brent slice (pixels; 0 = sized from the call, gang_setup_dev)
  int gang_px = 0;
  // k_brent_gang tag epoch (tags carry it, so they need no clearing between
  // launches) and the tag buffer it is valid for
  int gang_epoch = 0;
  void* gang_tag_buf = nullptr;
  size_t gang_tag_cap = 0;  // the tag allocation's capacity when last cleared
  // segments of the last estimate_disp call whose final states are in h_res
  // (h3d_disp_seg_stats)
  int last_S = 0;
  h3dint::TablePending tab_pending;
  // H3D_DEV_SEG_TABLES (default 1): estimate_disp's chunk / segment tables
  // built on the device (k_disp_tables) where no gangs are needed
  int dev_seg_tables = 1;
  int disp_w8 = 4;  // H3D_DISP_W8: equalize register budget for M = 8
                    // (cfg4 sweep r02, ms/step W 1/2/3/4: 214/214/199/197)
};

namespace h3dint {

constexpr int kLaunchBlock = 256;
// distances per condition the device smoother holds in LDS (h3d_table.hip);
// beyond it h3d_disp_tables_dev runs the host smoother inside the call
constexpr int kTableMaxD = 1024;

// grow-only device buffer of the ctx, by slot name (nullptr on OOM)
void* scratch(h3d_ctx* ctx, const char* slot, size_t bytes);
// the same, but a grown buffer keeps its first `keep` bytes (stream-ordered
// copy; growth at least doubles the capacity)
void* scratch_keep(h3d_ctx* ctx, const char* slot, size_t bytes, size_t keep);
hipEvent_t ev_get(h3d_ctx* ctx);
// host -> device copy of `bytes` through the ctx's pinned bounce buffer,
// stream-ordered on s (the source may be reused at once)
int h2d_pinned(h3d_ctx* ctx, void* d_dst, const void* src, size_t bytes, hipStream_t s);
// a pinned landing zone of >= bytes for device -> host copies (grow-only;
// one user at a time: the caller synchronises before reading it and before
// its next call), nullptr on failure
void* pinned_rd(h3d_ctx* ctx, size_t bytes);
// device -> host copy through the pinned landing zone, synchronous on s
int d2h_sync(h3d_ctx* ctx, void* dst, const void* d_src, size_t bytes, hipStream_t s);
// folds the recorded event pairs into ctx->stats (synchronises the stream)
void prof_collect(h3d_ctx* ctx);
// grid of a grid-stride elementwise kernel over n items
int grid_for(h3d_ctx* ctx, int64_t n, int per_cu = 8);
// validates a replicate -> condition map; per-condition replicate counts and
// replicate indices (C x kMaxReps, design order)
int check_cond(const int32_t* cond_of_rep, int R, int C, std::vector<int>* nrep,
               std::vector<int32_t>* rep_idx);
// kernel status flags -> H3D_E* code (+ message)
int flags_to_code(int fl);
// the device table of h3d_disp_tables_dev (h3d_table.hip): copy its status
// (before the stream sync), settle it (after): 1 = redone on the host
int table_status_copy(h3d_ctx* ctx, int* h_st);
int table_settle(h3d_ctx* ctx, const int* h_st);

// wraps one kernel launch with HIP events on the ctx stream when profiling
struct ProfScope {
  h3d_ctx* ctx;
  const char* name;
  int64_t units;
  hipEvent_t a = nullptr, b = nullptr;
  bool on;
  ProfScope(h3d_ctx* c, const char* n, int64_t u, int level = 2)
      : ctx(c), name(n), units(u), on(c->prof >= level) {
    // bound the pending list (collecting synchronises the stream)
    if (on && ctx->pending.size() > 16384) prof_collect(ctx);
    if (on) {
      a = ev_get(ctx);
      b = ev_get(ctx);
      (void)hipEventRecord(a, ctx->stream);
    }
  }
  ~ProfScope() {
    if (on) {
      (void)hipEventRecord(b, ctx->stream);
      ctx->pending.push_back({name, {a, b}});
      ctx->pending_units.push_back(units);
    }
  }
};

}  // namespace h3dint
