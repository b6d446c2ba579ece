// gfx950 kernels of the hic3defdr hot path (estimate_disp + lrt).
//
// Layout in HBM:
//   * LRT inputs stay in the reference's pixel order, replicate-minor (AoS):
//     raw (n, R) int32, f (n, R) f64, dist (n) int32 -> one lane per pixel
//     reads its R contiguous values (16 B / 32 B vector loads for R = 4).
//   * estimate_disp re-orders the disp pixels by distance once (stable radix
//     sort on dist) into replicate-major (SoA) copies raw_s[r][i], f_s[r][i]
//     and the pseudodata buffer pd[r][i], so a segment (distance d) is a
//     contiguous index range and every per-replicate access is coalesced.
//   * work items = (chunk of 256 pixels of one distance) x condition; one
//     256-thread workgroup per work item, one pixel per lane.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "h3d_model.h"

namespace h3d {

constexpr int kChunk = 256;  // pixels per disp work item (= block size)
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / 64;  // disp partials per work item
// k_brent: one workgroup per segment. 1024 threads: a cfg2 step has ~500
// segments, so the workgroup count, not the register budget, set the waves
// per SIMD; measured (tools/ab_lib.sh) k_brent<2> 3.34 -> 2.95 ms per step
// against 512 (768: 3.25). M >= 16 keeps 512 threads: its loop needs more
// than the 128 VGPRs a 1024-thread workgroup leaves a lane.
template <int M>
constexpr int brent_block() {
  return M >= 16 ? 512 : 1024;
}

// deterministic wave sum (fixed butterfly); result valid in every lane
__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// deterministic block sum of one double per thread (fixed butterfly per wave,
// then waves in order); result valid in thread 0.
__device__ inline double block_sum(double v, double* lds) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int w = 0; w < nw; ++w) t += lds[w];
  }
  return t;
}

static __global__ void k_i64_to_i32(const int64_t* __restrict__ in,
                             int32_t* __restrict__ out, int64_t n,
                             int* __restrict__ overflow) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = in[i];
    if (v < 0 || v > 0x7fffffffLL) atomicOr(overflow, 1);
    out[i] = (int32_t)v;
  }
}

static __global__ void k_iota(int32_t* __restrict__ out, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int32_t)i;
}

// destination row of every replicate (a kernel argument by value): the SoA
// row of replicate r is raw[r][i] / f[r][i]
struct SoaRows {
  int32_t* raw[kMaxReps];
  double* f[kMaxReps];
};

// AoS (n, R) -> distance-sorted SoA rows
static __global__ void k_gather_soa(const int32_t* __restrict__ perm,
                                    const int32_t* __restrict__ raw,
                                    const double* __restrict__ f, int64_t n, int R,
                                    SoaRows dst) {
  if (R == 4 && ((uintptr_t)raw & 15) == 0 && ((uintptr_t)f & 15) == 0) {
    // the common shape: one 16 B load of the raw row, two 16 B loads of the
    // f row per pixel (rows are 16 B aligned), so the random row gather
    // issues 3 memory instructions per lane instead of 8
    const int4* raw4 = reinterpret_cast<const int4*>(raw);
    const double2* f2 = reinterpret_cast<const double2*>(f);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
      const int64_t src = perm[i];
      const int4 rv = raw4[src];
      const double2 fa = f2[2 * src], fb = f2[2 * src + 1];
      dst.raw[0][i] = rv.x;
      dst.raw[1][i] = rv.y;
      dst.raw[2][i] = rv.z;
      dst.raw[3][i] = rv.w;
      dst.f[0][i] = fa.x;
      dst.f[1][i] = fa.y;
      dst.f[2][i] = fb.x;
      dst.f[3][i] = fb.y;
    }
    return;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t src = perm[i];
    for (int r = 0; r < R; ++r) {
      dst.raw[r][i] = raw[src * R + r];
      dst.f[r][i] = f[src * R + r];
    }
  }
}

// Gather of ONE condition's replicates through that condition's own pixel
// order: dst row j (replicate reps[j]) = raw / f column reps[j] of the AoS
// rows perm[i]. A workgroup takes kGatherTile output pixels, reads their
// row slices cooperatively (consecutive lanes walk along a row, so a wave's
// load covers whole row slices instead of 64 scattered words), transposes
// them through LDS and writes each replicate's run of the tile coalesced.
// One pixel order PER CONDITION is sound because every consumer of a
// condition's SoA rows (equalize, the NLL, the segment sums) touches only
// that condition's replicates, and all the orders share the distance
// segments.
constexpr int kGatherTile = 128;

static __global__ __launch_bounds__(256) void k_gather_cond_tile(
    const int32_t* __restrict__ perm, const int32_t* __restrict__ raw,
    const double* __restrict__ f, int64_t n, int R, const int32_t* __restrict__ reps,
    int nr, SoaRows dst) {
  constexpr int TP = kGatherTile, LD = kGatherTile + 1;  // +1: bank spread
  __shared__ int64_t s_src[TP];
  __shared__ int s_rep[kMaxReps];
  __shared__ double s_buf[kMaxReps * LD];
  int32_t* s_ibuf = reinterpret_cast<int32_t*>(s_buf);
  if (threadIdx.x < nr) s_rep[threadIdx.x] = reps[threadIdx.x];
  for (int64_t t0 = (int64_t)blockIdx.x * TP; t0 < n; t0 += (int64_t)gridDim.x * TP) {
    const int np = (int)((n - t0) < TP ? (n - t0) : TP);
    if (threadIdx.x < np) s_src[threadIdx.x] = perm[t0 + threadIdx.x];
    __syncthreads();
    const int tot = np * nr;
    for (int q = threadIdx.x; q < tot; q += blockDim.x) {
      const int p = q / nr, j = q - p * nr;
      s_ibuf[j * LD + p] = raw[s_src[p] * R + s_rep[j]];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < nr * TP; q += blockDim.x) {
      const int j = q / TP, p = q - j * TP;
      if (p < np) dst.raw[j][t0 + p] = s_ibuf[j * LD + p];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < tot; q += blockDim.x) {
      const int p = q / nr, j = q - p * nr;
      s_buf[j * LD + p] = f[s_src[p] * R + s_rep[j]];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < nr * TP; q += blockDim.x) {
      const int j = q / TP, p = q - j * TP;
      if (p < np) dst.f[j][t0 + p] = s_buf[j * LD + p];
    }
    __syncthreads();
  }
}

// per-condition sort key (distance, max count, min count over the
// condition's replicates; each capped to its half of the cbits count bits).
// Modelled on the cfg2 census (tools/order_experiment.py): wave lane
// utilisation of the equalize pass 0.68 with the total-count key -> 0.79.
// count code of the 16-bit key: exact below 128, then 8 counts per code up
// to 1151 (counts that high are a few near-diagonal pixels, whose trip counts
// vary slowly with the count): the key fits 24 bits at D <= 256, one radix
// pass fewer than 12-bit caps (census, tools/q2q_stats.py --key: the same
// modelled lane utilisation)
__device__ inline uint64_t count_code8(uint64_t v) {
  return v < 128 ? v : (v < 1152 ? 128 + ((v - 128) >> 3) : 255);
}

template <typename K>
__global__ void k_dist_cond_keys(const int32_t* __restrict__ dist,
                                 const int32_t* __restrict__ raw, int64_t n, int R,
                                 const int32_t* __restrict__ reps, int nr, int cbits,
                                 K* __restrict__ keys) {
  const int lo = cbits / 2, hi = cbits - lo;
  const uint64_t cap_lo = (1ull << lo) - 1ull, cap_hi = (1ull << hi) - 1ull;
  const uint64_t dcap = (uint64_t)(K)~(K)0 >> cbits;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t mx = 0, mn = ~0ull;
    for (int j = 0; j < nr; ++j) {
      const uint64_t v = (uint32_t)raw[i * R + reps[j]];
      mx = v > mx ? v : mx;
      mn = v < mn ? v : mn;
    }
    uint64_t d = (uint32_t)dist[i];
    if (d > dcap) d = dcap;
    if (cbits == 16) {
      // (distance, min code, max code): min first models 1-2 % better
      keys[i] = (K)((d << 16) | (count_code8(mn) << 8) | count_code8(mx));
      continue;
    }
    if (mx > cap_hi) mx = cap_hi;
    if (mn > cap_lo) mn = cap_lo;
    keys[i] = (K)((d << cbits) | (mx << lo) | mn);
  }
}

// k_dist_cond_keys for every condition at once when each has <= 2
// replicates (32-bit keys): one streaming pass over the pixels' raw and f
// rows writes condition c's keys (keys + c n) and its (raw, f) of each pixel
// as one 32-byte record (packed + c n) for k_gather_pack2 -- the gather
// through the condition's sort order then touches one 32-byte sector per
// pixel instead of a line of the raw rows and a line of the f rows.
// reps: kMaxReps entries per condition, as the per-condition pass.
struct alignas(32) CondPack2 {
  int32_t raw[4];  // [0, nr) used
  double f[2];
};

static __global__ void k_dist_cond_keys_pack2(const int32_t* __restrict__ dist,
                                              const int32_t* __restrict__ raw,
                                              const double* __restrict__ f, int64_t n,
                                              int R, int C, const int32_t* __restrict__ reps,
                                              const int32_t* __restrict__ nrep,
                                              uint32_t* __restrict__ keys,
                                              CondPack2* __restrict__ packed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t d = (uint32_t)dist[i];
    if (d > 0xffffu) d = 0xffffu;
    for (int c = 0; c < C; ++c) {
      const int r0 = reps[c * kMaxReps], r1 = nrep[c] > 1 ? reps[c * kMaxReps + 1] : r0;
      const uint32_t v0 = (uint32_t)raw[i * R + r0], v1 = (uint32_t)raw[i * R + r1];
      const uint64_t mx = v0 > v1 ? v0 : v1, mn = v0 < v1 ? v0 : v1;
      keys[c * n + i] = (uint32_t)((d << 16) | (count_code8(mn) << 8) | count_code8(mx));
      int4 rv;
      rv.x = (int)v0;
      rv.y = (int)v1;
      rv.z = 0;
      rv.w = 0;
      double2 fv;
      fv.x = f[i * R + r0];
      fv.y = f[i * R + r1];
      int4* q = reinterpret_cast<int4*>(packed + c * n + i);
      q[0] = rv;
      reinterpret_cast<double2*>(q + 1)[0] = fv;
    }
  }
}

// The gather of one condition (<= 2 replicates) through its sort order from
// the packed records: dst rows j < nr of pixel i = record perm[i].
static __global__ void k_gather_pack2(const int32_t* __restrict__ perm,
                                      const CondPack2* __restrict__ packed, int64_t n,
                                      int nr, SoaRows dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int4* q = reinterpret_cast<const int4*>(packed + perm[i]);
    const int4 rv = q[0];
    const double2 fv = reinterpret_cast<const double2*>(q + 1)[0];
    dst.raw[0][i] = rv.x;
    dst.f[0][i] = fv.x;
    if (nr > 1) {
      dst.raw[1][i] = rv.y;
      dst.f[1][i] = fv.y;
    }
  }
}

// sort key (distance, total count capped to cbits bits): inside a distance
// segment pixels of similar depth sit in the same wave, so the q2qnbinom
// branches (tail side, series vs continued fraction) diverge less. The count
// only orders pixels inside a segment (which segment a pixel joins is fixed
// by the distance bits), so capping it changes no result beyond the order of
// the segment's partial sums. K = uint32_t (16 count bits) whenever the
// distance fits the other 16: fewer radix passes over half the key bytes.
template <typename K>
__global__ void k_dist_count_keys(const int32_t* __restrict__ dist,
                                  const int32_t* __restrict__ raw, int64_t n,
                                  int R, int cbits, K* __restrict__ keys) {
  const uint64_t cap = (1ull << cbits) - 1ull;
  // distances outside the key's range (incl. negative ones) saturate to the
  // largest code, which is >= D: the caller's segment check rejects them
  const uint64_t dcap = (uint64_t)(K)~(K)0 >> cbits;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t tot = 0;
    for (int r = 0; r < R; ++r) tot += (uint32_t)raw[i * R + r];
    if (tot > cap) tot = cap;
    uint64_t d = (uint32_t)dist[i];
    if (d > dcap) d = dcap;
    keys[i] = (K)((d << cbits) | tot);
  }
}

template <typename K>
__global__ void k_key_dist(const K* __restrict__ keys, int64_t n, int cbits,
                           int32_t* __restrict__ dist_s) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dist_s[i] = (int32_t)((uint64_t)keys[i] >> cbits);
}

// seg_start[d] = first index with dist_s >= d (d = 0..D)
static __global__ void k_seg_bounds(const int32_t* __restrict__ dist_s, int64_t n,
                             int D, int64_t* __restrict__ seg_start) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d > D) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (dist_s[mid] < d)
      lo = mid + 1;
    else
      hi = mid;
  }
  seg_start[d] = lo;
}

// The estimate_disp driver's per-call tables built on the device from the
// segment bounds (the host built them after a sync on seg_start: ~0.1 ms of
// idle GPU per cfg2 step): per distance its chunks of kChunk pixels
// (chunk_start / len / distance, scanned over the distances in order), the
// first / end chunk of each distance, every segment's initial qcml state and
// pixel count. One 1024-thread block. *bad = 1 when a pixel's distance is
// outside [0, D) (seg_start does not span [0, n)). With task_seg non-null
// also k_brent_gang's task table: per distance C x ceil(len / gang_P)
// (segment, slice) entries in distance order (the caller pre-fills the
// table's unused tail with -1).
static __global__ __launch_bounds__(1024) void k_disp_tables(
    const int64_t* __restrict__ seg, int D, int C, int64_t n,
    const int32_t* __restrict__ n_rep, int64_t* __restrict__ cs,
    int32_t* __restrict__ cl, int32_t* __restrict__ cd, int32_t* __restrict__ scb,
    int32_t* __restrict__ sce, SegState* __restrict__ st, int64_t* __restrict__ lpx,
    int* __restrict__ bad, int64_t gang_P, int32_t* __restrict__ task_seg,
    int32_t* __restrict__ task_g, double tol, int task_len, int* __restrict__ seg_flags,
    int* __restrict__ gang_abort) {
  __shared__ int s_wsum[16], s_tsum[16];
  __shared__ int s_carry, s_tcarry;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    s_carry = 0;
    s_tcarry = 0;
    *bad = (seg[0] != 0 || seg[D] != n) ? 1 : 0;
    if (gang_abort) *gang_abort = 0;
  }
  // (the segment flags zeroed here rather than by a fill launch each call)
  if (seg_flags)
    for (int k = threadIdx.x; k < D * C; k += 1024) seg_flags[k] = 0;
  __syncthreads();
  for (int base = 0; base < D; base += 1024) {
    const int d = base + threadIdx.x;
    const int64_t len = d < D ? seg[d + 1] - seg[d] : 0;
    const int nch = (int)((len + kChunk - 1) / kChunk);
    // gang tasks of the distance (k_brent_gang): C x ceil(len / P) slices
    const int ntk = task_seg ? C * (int)((len + gang_P - 1) / gang_P) : 0;
    int x = nch, xt = ntk;  // inclusive scans over the block
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off, 64), yt = __shfl_up(xt, off, 64);
      if (lane >= off) {
        x += y;
        xt += yt;
      }
    }
    if (lane == 63) {
      s_wsum[wid] = x;
      s_tsum[wid] = xt;
    }
    __syncthreads();
    int before = 0, tot = 0, tbefore = 0, ttot = 0;
    for (int w = 0; w < 16; ++w) {
      before += (w < wid) ? s_wsum[w] : 0;
      tot += s_wsum[w];
      tbefore += (w < wid) ? s_tsum[w] : 0;
      ttot += s_tsum[w];
    }
    const int b0 = s_carry + before + x - nch;
    if (d < D && ntk) {
      const int t0 = s_tcarry + tbefore + xt - ntk, G = ntk / C;
      for (int c = 0; c < C; ++c)
        for (int j = 0; j < G; ++j) {
          task_seg[t0 + c * G + j] = d * C + c;
          task_g[t0 + c * G + j] = j;
        }
    }
    if (d < D) {
      scb[d] = b0;
      sce[d] = b0 + nch;
      const int64_t a = seg[d];
      for (int j = 0; j < nch; ++j) {
        cs[b0 + j] = a + (int64_t)j * kChunk;
        cl[b0 + j] = (int32_t)min((int64_t)kChunk, len - (int64_t)j * kChunk);
        cd[b0 + j] = d;
      }
      for (int c = 0; c < C; ++c) {
        seg_init(&st[d * C + c], (long long)len, n_rep[c], tol);
        lpx[d * C + c] = len;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      s_carry += tot;
      s_tcarry += ttot;
    }
    __syncthreads();
  }
  // the task table's unused tail (k_brent_gang skips -1 entries)
  if (task_seg)
    for (int t = s_tcarry + threadIdx.x; t < task_len; t += 1024) task_seg[t] = -1;
}

// Work item w of the active list: item = chunk * C + c.
// Equalize pass: per pixel equalize (scaled_nb.py:186-214) with the
// segment's current dispersion, write pseudodata, then the NLL term at the
// first Brent point. NLL pass: the NLL term (dispersion.py:67-70) at the
// segment's current Brent point. Wave partials -> partial[w * 4 + wave].
// PH = the pass this instantiation runs (kEqualize or kNll): the list holds
// the equalize items first (meta[2] of them), then the NLL items, and each
// pass is its own kernel so the light NLL pass is not held to the register
// budget of q2qnbinom. W = minimum waves per SIMD asked of the allocator.
// NLL = false (single-rank driver): the equalize pass only writes the
// pseudodata; k_brent then evaluates every NLL of the segment's Brent search
// in one workgroup.
// k_disp_work's dynamic task heads in the work meta: 2 passes x 8 ranges,
// kTaskHeadStride ints (128 B) apart, after the first block of the meta
constexpr int kTaskHeadStride = 32;
constexpr int kWorkMetaInts = kTaskHeadStride * 17;

template <int M, int W, int PH, bool NLL = true>
__global__ __launch_bounds__(kBlock, W) void k_disp_work(
    const int32_t* __restrict__ raw_s, const double* __restrict__ f_s,
    double* __restrict__ pd, int64_t n, const int64_t* __restrict__ chunk_start,
    const int32_t* __restrict__ chunk_len, const int32_t* __restrict__ chunk_d,
    int C, const int32_t* __restrict__ rep_idx /* C x kMaxReps */,
    const int32_t* __restrict__ n_rep /* C */, const SegState* __restrict__ st,
    int* __restrict__ seg_flags, const int32_t* __restrict__ list,
    int32_t* __restrict__ meta /* [len, active, eq_len, live], task heads */,
    double* __restrict__ partial, int static8) {
  const int beg = (PH == kEqualize) ? 0 : meta[2];
  const int end = (PH == kEqualize) ? meta[2] : meta[0];
  // Tasks are (item, wave) pairs: wave q of a block evaluates pixels
  // [64 q, 64 q + 64) of an item, and the waves run independently (no block
  // barrier). The first static8 / 8 of the rounds are dealt round-robin; the
  // remaining tasks are split into 8 ranges, each with its own head counter
  // (128 B apart, zeroed by k_seg_update): a wave dequeues from the range of
  // its block group (blockIdx % 8 -- the blocks of one XCD under the
  // observed round-robin placement; speed only), then from the others once
  // that range is spent. The item costs vary with the incomplete-gamma trip
  // counts, and a static deal left the waves that drew the dearer items
  // running alone at the end of the launch; one head for every wave
  // saturates (~88 dequeues / us, MI355X_MICROARCH.md "dequeue").
  constexpr int kWv = kBlock / 64;
  const int lane = threadIdx.x & 63;
  const int64_t t0 = (int64_t)beg * kWv, t1 = (int64_t)end * kWv;
  const int64_t wt = (int64_t)gridDim.x * kWv;
  // (fewer than two rounds of tasks: all dealt round-robin -- a wave does
  // at most two, and the waves left without a task would otherwise each
  // probe the 8 heads to find them empty)
  const int64_t tdyn = (t1 - t0 < 2 * wt) ? t1 : t0 + ((t1 - t0) / wt) * static8 / 8 * wt;
  const int64_t tl = t1 - tdyn;
  int32_t* heads = meta + kTaskHeadStride * (1 + (PH == kEqualize ? 0 : 8));
  const int grp = blockIdx.x & 7;
  unsigned spent = 0u;
  auto take = [&]() -> int64_t {
    if (tl <= 0) return t1;
#pragma unroll 1
    for (int k = 0; k < 8; ++k) {
      const int p = (grp + k) & 7;
      if ((spent >> p) & 1u) continue;
      const int64_t pb = tdyn + tl * p / 8, pe = tdyn + tl * (p + 1) / 8;
      int got = 0;
      if (lane == 0) got = atomicAdd(heads + kTaskHeadStride * p, 1);
      got = __shfl(got, 0, 64);
      if (pb + got < pe) return pb + got;
      spent |= 1u << p;
    }
    return t1;
  };
  // the table log's table in LDS (the equalize pass's logs: the prefactor of
  // every incomplete-gamma evaluation, lgamma of the shapes, the mean MLE's
  // start, log f): a per-lane global load sat on each one's chain
  __shared__ LogTab s_tab[kLogTabLen];
  for (int k = threadIdx.x; k < kLogTabLen; k += kBlock) s_tab[k] = kLogTab[k];
  __syncthreads();
  int64_t t = t0 + (int64_t)blockIdx.x * kWv + (threadIdx.x >> 6);
  if (t >= tdyn) t = take();
  // (taking the wave's next task at the top of this one, so the dequeue's
  // round trip runs under this task's arithmetic, measured slower: equalize
  // 2.57 -> 2.66 ms per cfg2 step, r06z)
  for (; t < t1; t = (t + wt < tdyn) ? t + wt : take()) {
    const int w = (int)(t / kWv);
    const int q = (int)(t - (int64_t)w * kWv);
    const int item = list[w];
    const int chunk = item / C, c = item - chunk * C;
    const int s = chunk_d[chunk] * C + c;
    constexpr int phase = PH;
    const int nr = n_rep[c];
    double term = 0.0;
    const int i = q * 64 + lane;
    H3D_SEC_BEGIN(t_task);
    if (i < chunk_len[chunk] && nr < 8) {
      // Rolled replicate loop: the q2qnbinom code (the bulk of the kernel)
      // is emitted once instead of once per replicate slot. Sums run
      // sequentially from 0 in replicate order = numpy's row sum for n < 8.
      constexpr int MS = M < 8 ? M : 8;  // slots for nr < 8
      const int64_t px = chunk_start[chunk] + i;
      const NllConst kc = st[s].k;
      const int32_t* ri = rep_idx + c * kMaxReps;
      double lgsum = 0.0, z = 0.0;
      if (phase == kEqualize) {
        const double alpha = st[s].disp;
        double x[MS], f[MS], as[MS], lf[MS];
#pragma unroll
        for (int k = 0; k < MS; ++k) {
          const bool on = k < nr;
          x[k] = on ? (double)raw_s[(int64_t)ri[k] * n + px] : 0.0;
          f[k] = on ? f_s[(int64_t)ri[k] * n + px] : 1.0;
          lf[k] = on ? log_fast_checked(f[k], s_tab) : 0.0;
          as[k] = alpha;
        }
        int fl = 0;
        H3D_SEC_BEGIN(t_fit);
        const double f_mean = exp_fast(np_sum<MS>(lf, nr) / nr) - 0.0;
        const double mu = fit_mu<MS>(x, f, as, nr, ~0u, &fl, s_tab);
        H3D_SEC_END(0, t_fit);
        if (fl) atomicOr(&seg_flags[s], fl);
        const double mu_out0 = mu * f_mean;
        // The reference clamps (mu_in, mu_out) to 0.25 in place and carries
        // the clamped mu_out into the later replicates (scaled_nb.py:209-213,
        // 240-242). Resolve that carry first -- fc = the first replicate
        // whose pair fails the >= 0.25 test -- so the replicates can be
        // visited in any order: upper-tail ones (x >= mu_in: the continued
        // fraction path of the incomplete gamma) first, then lower-tail ones
        // (power series). Lanes of a wave then run the same branch of
        // igam_pq in each slot instead of serialising both.
        int fc = nr;
        unsigned up = 0u, lo = 0u;
#pragma unroll
        for (int k = MS - 1; k >= 0; --k)
          if (k < nr) {
            const double mi = mu * f[k];
            if (!(mi >= 0.25 && mu_out0 >= 0.25)) fc = k;
            if (x[k] >= mi)
              up |= 1u << k;
            else
              lo |= 1u << k;
          }
        LgamCache cache;
#pragma unroll 1
        for (int j = 0; j < nr; ++j) {
          int k;
          if (up) {
            k = __builtin_ctz(up);
            up &= up - 1u;
          } else {
            k = __builtin_ctz(lo);
            lo &= lo - 1u;
          }
          const int64_t o = (int64_t)ri[k] * n + px;
          double mu_in = mu * f_s[o];
          double mu_out = (k > fc) ? 0.25 : mu_out0;
          H3D_SEC_BEGIN(t_q2q);
          pd[o] = q2q((double)raw_s[o], &mu_in, &mu_out, alpha, &cache, s_tab);
          H3D_SEC_END(13, t_q2q);
        }
      }
      if (phase == kEqualize) H3D_SEC_END(14, t_task);
      if constexpr (!NLL) continue;
      // NLL term in replicate order (numpy's row sum) over the pseudodata
      // (in the equalize pass: the values this thread just wrote). All loads
      // are issued up front into the slot registers; the rolled loop then
      // consumes slot 0 and shifts the slots down (static indices only), so
      // the lgamma code is emitted once and no load latency sits inside it.
      {
        double d[MS];
#pragma unroll
        for (int k = 0; k < MS; ++k)
          d[k] = (k < nr) ? pd[(int64_t)ri[k] * n + px] : 0.0;
#pragma unroll 1
        for (int k = 0; k < nr; ++k) {
          const double dk = d[0];
#pragma unroll
          for (int j = 0; j + 1 < MS; ++j) d[j] = d[j + 1];
          lgsum += lgam_nll(dk + kc.r, s_tab);
          z += dk;
        }
      }
      term = lgsum + kc.lg_nr - lgam_nll(z + kc.nr, s_tab) - kc.n_lg_r;
    } else if (M >= 8 && i < chunk_len[chunk]) {
      // >= 8 replicates in the condition: numpy's pairwise row sums
      const int64_t px = chunk_start[chunk] + i;
      double d[M];
      int ri[M];
#pragma unroll
      for (int k = 0; k < M; ++k) ri[k] = (k < nr) ? rep_idx[c * kMaxReps + k] : 0;
      if (phase == kEqualize) {
        double x[M], f[M];
#pragma unroll
        for (int k = 0; k < M; ++k) {
          if (k < nr) {
            x[k] = (double)raw_s[(int64_t)ri[k] * n + px];
            f[k] = f_s[(int64_t)ri[k] * n + px];
          } else {
            x[k] = 0.0;
            f[k] = 1.0;
          }
        }
        const int fl = equalize_pixel<M>(x, f, nr, st[s].disp, d, s_tab);
        if (fl) atomicOr(&seg_flags[s], fl);
#pragma unroll
        for (int k = 0; k < M; ++k)
          if (k < nr) pd[(int64_t)ri[k] * n + px] = d[k];
        if constexpr (!NLL) continue;
      } else {
#pragma unroll
        for (int k = 0; k < M; ++k)
          d[k] = (k < nr) ? pd[(int64_t)ri[k] * n + px] : 0.0;
      }
      const NllConst kc = st[s].k;
      term = nll_pixel<M>(d, nr, kc, s_tab);
    }
    // one partial per wave (fixed shuffle tree -> deterministic); no block
    // barrier, so the waves of a block run their items independently
    if constexpr (NLL) {
      const double wt_sum = wave_sum(term);
      if (lane == 0) partial[(int64_t)w * kWavesPerBlock + q] = wt_sum;
    }
  }
}

// seg_total[s] = sum of the segment's wave partials in list order (one wave
// per segment, fixed reduction tree -> deterministic)
// With `st` non-null (no cross-rank reduction between the two steps), the
// wave then advances its segment's qcml/Brent state machine itself: the
// segments step in parallel across the chip instead of inside the single
// list-building workgroup of k_seg_update.
static __global__ void k_seg_reduce(const double* __restrict__ partial,
                             const int32_t* __restrict__ seg_lb,
                             const int32_t* __restrict__ seg_le, int S,
                             double* __restrict__ seg_total,
                             SegState* __restrict__ st,
                             const int* __restrict__ seg_flags,
                             const int32_t* __restrict__ n_rep, int C,
                             double* __restrict__ result) {
  const int s = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= S) return;
  const int64_t b = (int64_t)seg_lb[s] * kWavesPerBlock,
                e = (int64_t)seg_le[s] * kWavesPerBlock;
  double v = 0.0;
  for (int64_t j = b + lane; j < e; j += 64) v += partial[j];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if (lane == 0) {
    seg_total[s] = v;
    if (st) {
      SegState cur = st[s];
      if (cur.phase != kDone) {
        cur.flags |= seg_flags[s];
        seg_step(&cur, v, n_rep[s % C]);
        st[s] = cur;
        if (cur.phase == kDone) result[s] = cur.result;
      }
    }
  }
}

// One workgroup: with `step`, advance every active segment's qcml/Brent
// state machine with its (rank-reduced) total -- otherwise k_seg_reduce has
// already stepped them -- then rebuild the active work list.
static __global__ __launch_bounds__(1024) void k_seg_update(
    SegState* __restrict__ st, const double* __restrict__ seg_total,
    const int* __restrict__ seg_flags, int S, int C,
    const int32_t* __restrict__ n_rep, const int32_t* __restrict__ seg_chunk_b,
    const int32_t* __restrict__ seg_chunk_e, int32_t* __restrict__ list,
    int32_t* __restrict__ seg_lb,
    int32_t* __restrict__ seg_le, double* __restrict__ result,
    int32_t* __restrict__ meta /* [len, active, eq_len, live] */, int first, int step,
    const int64_t* __restrict__ seg_px /* this rank's pixels per segment */,
    unsigned long long* __restrict__ work_count /* [equalize, nll] pixel-reps */,
    int* __restrict__ brent_queue /* [k_brent, k_brent_gang] or null */,
    int64_t gang_P = 0, int32_t* __restrict__ gang_seg = nullptr,
    int32_t* __restrict__ gang_g = nullptr) {
  // the next iteration's Brent work queues start at 0 (two memset launches
  // fewer per qcml iteration)
  if (brent_queue && threadIdx.x == 0) {
    brent_queue[0] = 0;
    brent_queue[1] = 0;
  }
  // Every cross-thread step is a wave shuffle tree plus one LDS slot per wave
  // (16 waves): no contended LDS atomics, two barriers per 1024 segments.
  constexpr int kW = 1024 / 64;
  __shared__ unsigned long long wsum[2][kW];
  __shared__ int32_t wscan[3][kW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // 1. advance the state machines; count the equalize / NLL items of the next
  // round, and the pixel-replicates they visit (measurement: algorithmic bytes
  // of the disp kernels)
  unsigned long long weq = 0ull, wnll = 0ull;
  int ceq = 0, live = 0;
  for (int s = threadIdx.x; s < S; s += blockDim.x) {
    int phase;
    if (!first && step) {
      SegState cur = st[s];
      if (cur.phase != kDone) {
        cur.flags |= seg_flags[s];
        seg_step(&cur, seg_total[s], n_rep[s % C]);
        st[s] = cur;
        if (cur.phase == kDone) result[s] = cur.result;
      }
      phase = cur.phase;
    } else {
      // stepped by k_seg_reduce (or nothing to step yet)
      phase = st[s].phase;
      if (first && phase == kDone) result[s] = st[s].result;
    }
    const unsigned long long w = (unsigned long long)seg_px[s] * n_rep[s % C];
    if (phase == kEqualize) {
      weq += w;
      ceq += seg_chunk_e[s / C] - seg_chunk_b[s / C];
    }
    if (phase == kNll) wnll += w;
    live += (phase != kDone) ? 1 : 0;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    weq += __shfl_xor(weq, off, 64);
    wnll += __shfl_xor(wnll, off, 64);
    ceq += __shfl_xor(ceq, off, 64);
    live += __shfl_xor(live, off, 64);
  }
  if (lane == 0) {
    wsum[0][wid] = weq;
    wsum[1][wid] = wnll;
    wscan[0][wid] = ceq;
    wscan[1][wid] = live;
  }
  __syncthreads();
  int eq_total = 0, live_total = 0;
#pragma unroll
  for (int w = 0; w < kW; ++w) {
    eq_total += wscan[0][w];
    live_total += wscan[1][w];
  }
  if (threadIdx.x == 0) {
    unsigned long long a = 0ull, b = 0ull;
    for (int w = 0; w < kW; ++w) {
      a += wsum[0][w];
      b += wsum[1][w];
    }
    work_count[0] += a;
    work_count[1] += b;
  }
  // 2. list: the equalize items of every segment first (offsets from 0), then
  // the NLL items (offsets from eq_total); one pass, both counts scanned at
  // once per 1024-segment slab. With gang tables: also the gang task list of
  // the segments the next Brent launch searches (phase kEqualize), their
  // ceil(pixels / gang_P) slices each -- compact, so k_brent_gang dequeues no
  // task of a finished segment (cfg2's tail iterations spent ~40 us skipping
  // the full table's ~3.7 k tasks one atomic at a time)
  int base_eq = 0, base_nll = eq_total, base_g = 0;
  for (int s0 = 0; s0 < S; s0 += blockDim.x) {
    __syncthreads();  // wscan reuse
    const int s = s0 + threadIdx.x;
    int phase = kDone, cnt = 0;
    if (s < S) {
      phase = st[s].phase;
      cnt = seg_chunk_e[s / C] - seg_chunk_b[s / C];
    }
    const int ce = (phase == kEqualize) ? cnt : 0;
    const int cn = (phase == kNll) ? cnt : 0;
    const int cg = (gang_seg && phase == kEqualize && seg_px[s] > 0)
                       ? (int)((seg_px[s] + gang_P - 1) / gang_P)
                       : 0;
    int ie = ce, in = cn, ig = cg;  // inclusive wave scans
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int ue = __shfl_up(ie, off, 64), un = __shfl_up(in, off, 64);
      const int ug = __shfl_up(ig, off, 64);
      if (lane >= off) {
        ie += ue;
        in += un;
        ig += ug;
      }
    }
    if (lane == 63) {
      wscan[0][wid] = ie;
      wscan[1][wid] = in;
      wscan[2][wid] = ig;
    }
    __syncthreads();
    int pe = 0, pn = 0, pg = 0, te = 0, tn = 0, tg = 0;
#pragma unroll
    for (int w = 0; w < kW; ++w) {
      const int ve = wscan[0][w], vn = wscan[1][w], vg = wscan[2][w];
      if (w < wid) {
        pe += ve;
        pn += vn;
        pg += vg;
      }
      te += ve;
      tn += vn;
      tg += vg;
    }
    if (s < S) {
      const bool eq = phase == kEqualize;
      const int beg = eq ? base_eq + pe + ie - ce : base_nll + pn + in - cn;
      const int c_here = eq ? ce : cn;
      // finished segments keep an empty range (k_seg_reduce writes 0)
      seg_lb[s] = beg;
      seg_le[s] = beg + c_here;
      const int d = s / C, c = s % C;
      const int cb = seg_chunk_b[d];
      for (int j = 0; j < c_here; ++j) list[beg + j] = (cb + j) * C + c;
      const int gb = base_g + pg + ig - cg;
      for (int j = 0; j < cg; ++j) {
        gang_seg[gb + j] = s;
        gang_g[gb + j] = j;
      }
    }
    base_eq += te;
    base_nll += tn;
    base_g += tg;
  }
  if (threadIdx.x == 0) {
    meta[0] = base_nll;
    meta[1] = base_nll;
    meta[2] = eq_total;
    // the gang task list's length (k_brent_gang's bound when it has one)
    meta[4] = gang_seg ? base_g : -1;
    // segments not yet kDone, genome-wide: with a cross-rank reduce every
    // rank steps identical state machines, so this count (unlike this
    // rank's own list length meta[1]) is the same on every rank and is what
    // the host loop terminates on
    meta[3] = live_total;
  }
  // k_disp_work's dynamic task heads (2 passes x 8 ranges)
  if (threadIdx.x < 16) meta[kTaskHeadStride * (1 + threadIdx.x)] = 0;
}

// The whole bounded-Brent search of cml (dispersion.py:46-80) for every
// segment whose pseudodata the equalize pass just wrote (phase kEqualize):
// one workgroup per segment (taken from a device queue), every NLL
// evaluation in-kernel over the segment's pseudodata (contiguous in the
// distance-sorted SoA, L2/MALL-resident across the evaluations), a fixed-order
// block reduction per evaluation (deterministic), and the state machine
// stepped by every thread on the same total (uniform, no broadcast). Exits
// when the segment needs its next equalize pass (next qcml iteration) or is
// done; seg_step bounds the loop (500 Brent evaluations -> kFlagBrentFail).
// The NLL work is compute-bound (lgamma); measured r02 on cfg2 against a
// dynamically scheduled variant (persistent workgroups draining a device
// ring of (segment, 2048-pixel chunk) tasks with agent-scope hand-offs):
// 4.6 vs 6.4 ms per step -- the per-task acquire and arrival traffic cost
// more than the tail the static grid leaves idle.
// seg_step out of line for k_brent: run by one thread once per evaluation,
// its registers stay out of the NLL loop's budget (the state stays in LDS:
// stepping a register copy measured slower, Brent 1.97-2.00 -> 2.01-2.02 ms
// per cfg2 step, r06ae). (nll_const's two lgammas
// of the next trial point on two lanes at once measured within noise:
// Brent 2.00-2.01 -> 1.98-2.00 ms per cfg2 step, r06aa -- not kept.)
static __device__ __noinline__ void seg_step_ool(SegState* s, double total, int n_reps) {
  seg_step(s, total, n_reps);
}

// One thread's share of a segment's NLL terms at one Brent trial point:
// pixels [b, el) from the LDS head, [el, e) from memory, two pixels per
// iteration (px, px + block): their lgammas are independent chains the
// scheduler interleaves (the NLL is bound by FP64 dependency latency at 4
// waves/SIMD); the terms still join the sum in pixel order (M >= 8: one
// pixel per trip -- the pair spilled at the 128-VGPR budget of
// __launch_bounds__(512, 4)). MODE 2: every argument >= kNllLargeR
// (nll_pixel_large); 1: >= kNllMidR (nll_pixel_mid); 0: nll_pixel.
// (nll_pixel_large).
#ifndef H3D_BRENT_PAIR2
#define H3D_BRENT_PAIR2 2
#endif
// pixels per trip of brent_segment_sum
template <int M>
constexpr int kPair2() {
  return M <= 2 ? H3D_BRENT_PAIR2 : M <= 4 ? 2 : 1;
}
#ifndef H3D_BRENT_PRIO
#define H3D_BRENT_PRIO 1
#endif
#ifndef H3D_BRENT_PRIO_DIV
#define H3D_BRENT_PRIO_DIV 4  // priority steps per evaluation (levels 3..0)
#endif
// The wave's issue priority by its progress through the segment (kPrio,
// k_brent): 3 at the start of an evaluation, one lower at each quarter of
// its trips. The SIMD otherwise prefers the older of its four waves
// throughout, so the waves finished one after another and the last ran
// alone (H3D_BRENT_CLOCK, r06v: the four age ranks' sums took 1.26 / 1.75 /
// 2.33 / 2.89 G cycles); a wave ahead now yields to the ones behind it.
// Arbitration only: the terms and their order are unchanged. Measured
// against levels from the wave's trips relative to the workgroup's running
// count (an LDS counter per trip): Brent 2.01 -> 2.05 ms per cfg2 step
// (r06y) -- the quarters stay.
__device__ __forceinline__ void brent_prio(int& cur, int trip, int ntr) {
  const int lv = __builtin_amdgcn_readfirstlane(
      3 - min(3, (H3D_BRENT_PRIO_DIV * trip) / max(ntr, 1)));
  if (lv == cur) return;
  cur = lv;
  if (lv == 2)
    __builtin_amdgcn_s_setprio(2);
  else if (lv == 1)
    __builtin_amdgcn_s_setprio(1);
  else if (lv == 0)
    __builtin_amdgcn_s_setprio(0);
}

template <int M, int kBlockT, int MODE, bool kPrio = false>
__device__ __forceinline__ double brent_segment_sum(
    const double* s_pd, int64_t lds_px, const double* __restrict__ pd, int64_t n,
    const int* ri, int nr, int64_t b, int64_t el, int64_t e, const NllConst& kc,
    const LogTab* s_tab) {
  double acc = 0.0;
  [[maybe_unused]] int trip = 0, lv = 3;
  [[maybe_unused]] const int ntr = (int)((e - b + kPair2<M>() * kBlockT - 1) / (kPair2<M>() * kBlockT));
  if constexpr (kPrio) __builtin_amdgcn_s_setprio(3);
  constexpr int kPair = kPair2<M>();
  auto term = [&](const double* v) {
    if constexpr (MODE == 2) return nll_pixel_large<M>(v, nr, kc, s_tab);
    else if constexpr (MODE == 1) return nll_pixel_mid<M>(v, nr, kc, s_tab);
    else return nll_pixel<M>(v, nr, kc, s_tab);
  };
  for (int64_t i = threadIdx.x; i < el - b; i += kPair * kBlockT) {
    if constexpr (kPrio) brent_prio(lv, trip++, ntr);
    double v[kPair][M];
    bool on[kPair];
#pragma unroll
    for (int q = 0; q < kPair; ++q) {
      const int64_t j = i + (int64_t)q * kBlockT;
      on[q] = q == 0 || j < el - b;
#pragma unroll
      for (int k = 0; k < M; ++k) v[q][k] = (k < nr && on[q]) ? s_pd[k * lds_px + j] : 0.0;
    }
    double t[kPair];
#pragma unroll
    for (int q = 0; q < kPair; ++q) t[q] = term(v[q]);
#pragma unroll
    for (int q = 0; q < kPair; ++q)
      if (on[q]) acc += t[q];
  }
  for (int64_t px = el + threadIdx.x; px < e; px += kPair * kBlockT) {
    if constexpr (kPrio) brent_prio(lv, trip++, ntr);
    double v[kPair][M];
    bool on[kPair];
#pragma unroll
    for (int q = 0; q < kPair; ++q) {
      const int64_t qx = px + (int64_t)q * kBlockT;
      on[q] = q == 0 || qx < e;
#pragma unroll
      for (int k = 0; k < M; ++k) v[q][k] = (k < nr && on[q]) ? pd[(int64_t)ri[k] * n + qx] : 0.0;
    }
    double t[kPair];
#pragma unroll
    for (int q = 0; q < kPair; ++q) t[q] = term(v[q]);
#pragma unroll
    for (int q = 0; q < kPair; ++q)
      if (on[q]) acc += t[q];
  }
  return acc;
}

// The segment's first `lds_px` pixels are staged in LDS once per search (the
// dynamic shared buffer, up to ~150 KB: one 1024-thread workgroup per CU);
// every evaluation reads them from there and streams only the rest -- the
// segment used to be re-read from beyond L2 on every evaluation (PMC: 859 MB
// fetched per launch for 74 MB of pseudodata, waves waiting half the time).
#ifdef H3D_BRENT_CLOCK
// measurement build only: per-wave shader-clock totals of k_brent's phases
// [sum, barrier after the sum, seg_step (wave 0), barrier after the step,
// head staging, whole kernel], printed by launch_brent
__device__ unsigned long long g_brent_clk[6 + 2 * 16];
#define H3D_BCLK(v) const long long v = clock64()
#define H3D_BADD(i, d) clk[i] += (unsigned long long)(d)
#else
#define H3D_BCLK(v)
#define H3D_BADD(i, d)
#endif

template <int M>
__global__ __launch_bounds__(brent_block<M>(), M >= 16 ? 2 : 4) void k_brent(
    const double* __restrict__ pd, int64_t n,
    const int64_t* __restrict__ seg_start /* D + 1 */, int S, int C,
    const int32_t* __restrict__ rep_idx /* C x kMaxReps */,
    const int32_t* __restrict__ n_rep /* C */, SegState* __restrict__ st,
    const int* __restrict__ seg_flags, double* __restrict__ result,
    int* __restrict__ queue, unsigned long long* __restrict__ work_count,
    int64_t lds_px, const int32_t* __restrict__ gate_meta, int live_min,
    const int* __restrict__ gang_abort) {
  extern __shared__ double s_pd[];  // [nr][lds_px]
  // gate (device-side choice between this kernel and k_brent_gang, both
  // launched): run when the live segments fill the chip, or when a gang
  // has aborted
  if (gate_meta && gate_meta[3] < live_min && !(gang_abort && *gang_abort)) return;
  // the state machine lives in LDS and is stepped by thread 0; the data loop
  // only holds the four NLL constants (the SegState in every thread's VGPRs
  // spilled at the 1024-thread register budget)
  __shared__ SegState s_st;
  constexpr int kBrentBlock = brent_block<M>();
  __shared__ double wpart[kBrentBlock / 64];
  __shared__ int s_next, s_more;
  // the NLL log's table in LDS: its lookup address depends on the value, so
  // the load sits on every lgamma's dependency chain (a global / L1 round
  // trip otherwise)
  __shared__ LogTab s_tab[kLogTabLen];
  for (int t = threadIdx.x; t < kLogTabLen; t += kBrentBlock) s_tab[t] = kLogTab[t];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#ifdef H3D_BRENT_CLOCK
  unsigned long long clk[6] = {0, 0, 0, 0, 0, 0};
  H3D_BCLK(k_t0);
#endif
  while (true) {
    __syncthreads();  // s_next / s_st reuse
    if (threadIdx.x == 0) s_next = atomicAdd(queue, 1);
    __syncthreads();
    const int s = s_next;
    if (s >= S) break;
    if (st[s].phase != kEqualize) continue;  // done, or nothing to search
    H3D_BCLK(c_stage0);
    if (threadIdx.x == 0) {
      s_st = st[s];
      s_st.flags |= seg_flags[s];
    }
    const int d = s / C, c = s - (s / C) * C;
    const int nr = n_rep[c];
    const int64_t b = seg_start[d], e = seg_start[d + 1];
    int ri[M];
#pragma unroll
    for (int k = 0; k < M; ++k) ri[k] = (k < nr) ? rep_idx[c * kMaxReps + k] : 0;
    const int64_t el = (e - b < lds_px) ? e : b + lds_px;  // [b, el) in LDS
    for (int64_t i = threadIdx.x; i < el - b; i += kBrentBlock) {
#pragma unroll
      for (int k = 0; k < M; ++k)
        if (k < nr) s_pd[k * lds_px + i] = pd[(int64_t)ri[k] * n + b + i];
    }
    int evals = 0;
    __syncthreads();
    H3D_BCLK(c_stage1);
    H3D_BADD(4, c_stage1 - c_stage0);
    while (true) {
      H3D_BCLK(c0);
      const NllConst kc = s_st.k;
      // every lgamma argument >= r: at r >= kNllLargeR / kNllMidR the short
      // paths (nll_pixel_large / _mid), the same for every thread of the
      // segment
      constexpr bool kPr = H3D_BRENT_PRIO != 0;
      const double acc = (kc.r >= kNllLargeR)
          ? brent_segment_sum<M, kBrentBlock, 2, kPr>(s_pd, lds_px, pd, n, ri, nr, b, el, e, kc, s_tab)
          : (kc.r >= kNllMidR)
          ? brent_segment_sum<M, kBrentBlock, 1, kPr>(s_pd, lds_px, pd, n, ri, nr, b, el, e, kc, s_tab)
          : brent_segment_sum<M, kBrentBlock, 0, kPr>(s_pd, lds_px, pd, n, ri, nr, b, el, e, kc, s_tab);
      double wacc = acc;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) wacc += __shfl_xor(wacc, off, 64);
      if (lane == 0) wpart[wid] = wacc;
      H3D_BCLK(c1);
      __syncthreads();
      H3D_BCLK(c2);
      if (threadIdx.x == 0) {
        double total = 0.0;
#pragma unroll
        for (int w = 0; w < kBrentBlock / 64; ++w) total += wpart[w];
        seg_step_ool(&s_st, total, nr);
        s_more = (s_st.phase == kNll) ? 1 : 0;
      }
      H3D_BCLK(c3);
      ++evals;
      __syncthreads();  // s_st / s_more / wpart
      H3D_BCLK(c4);
      H3D_BADD(0, c1 - c0);
      H3D_BADD(1, c2 - c1);
      H3D_BADD(2, c3 - c2);
      H3D_BADD(3, c4 - c3);
      if (!s_more) break;
    }
    if (threadIdx.x == 0) {
      s_st.last_evals = evals;
      st[s] = s_st;
      if (s_st.phase == kDone) result[s] = s_st.result;
      atomicAdd(&work_count[1], (unsigned long long)(e - b) * nr * evals);
    }
  }
#ifdef H3D_BRENT_CLOCK
  H3D_BCLK(k_t1);
  clk[5] = (unsigned long long)(k_t1 - k_t0);
  if (lane == 0) {
    for (int i = 0; i < 6; ++i) atomicAdd(&g_brent_clk[i], clk[i]);
    // per wave of the workgroup: its sum and first-barrier cycles
    if (wid < 16) {
      atomicAdd(&g_brent_clk[6 + wid], clk[0]);
      atomicAdd(&g_brent_clk[22 + wid], clk[1]);
    }
  }
#endif
}

// ---- gang Brent: a segment's search over several co-resident workgroups ----
// k_brent runs a segment's whole bounded-Brent search in ONE workgroup, so a
// call with fewer segments than CUs leaves CUs idle: a rank of the distance
// re-shard at N = 8 owns ~50 of cfg3's segments of ~230 k pixels each, and
// its k_brent ran on 50 CUs. Here a segment of n pixels is split into G
// slices of P pixels (the host sizes P so the whole call has about two
// resident grids of slices); a gang of G workgroups each adds its slice's
// NLL terms per evaluation, publishes the partial, and waits for the gang's
// other partials. Every member then sums the G partials in slice order
// (deterministic) and steps its own copy of the state machine -- the same
// inputs, so the same trial point in every member, no broadcast. Member 0
// writes the state back.
//
// Exchange: per (segment, slice, evaluation parity) a partial and a tag
// (evaluation + 1), written with relaxed agent-scope stores (coherent across
// the XCDs' L2s instruction by instruction), the tag only after the partial's
// store has completed; the readers (the lanes of wave 0, one slice each)
// poll the tags, then load the partials -- one vector load per 64 slices. A
// release / acquire pair at agent scope writes back / invalidates the whole
// L2 on gfx950 (buffer_wbl2 / buffer_inv), and a single arrival counter with
// partials read one by one cost ~20 us per evaluation (r03 A/B: 13.3 vs
// 2.8 ms of Brent per cfg2 step).
//
// Ordering argument (why the relaxed pair is enough here). In the AMDGPU
// memory model an agent-scope release is "buffer_wbl2 sc1; s_waitcnt
// vmcnt(0)" and an acquire "s_waitcnt vmcnt(0); buffer_inv sc1": the L2
// write-back / invalidate exist to make NON-atomic data visible across the
// XCDs; the waitcnt orders the stores. Every datum this exchange publishes
// is itself an agent-scope atomic (the partial and the tag), which the
// hardware performs at the agent's coherence point rather than in a
// non-coherent L2 line, so the only ordering left to enforce is that the
// partial's store is complete before the tag's is issued -- the
// s_waitcnt(0) between them (the signal fences keep the compiler from
// moving either across it) -- and, on the reader's side, that the partial
// loads are issued after the tag loads returned (the same waitcnt after the
// poll). Those are the waitcnt halves of the release / acquire sequences.
// The data the searches read otherwise (pseudodata, SegState) were written
// by earlier kernels of the stream, ordered by the kernel boundary. A
// bounded wait (below) still ends every gang if this ever failed to hold,
// and the ctx counts such aborts (h3d_profile_read "gang_aborts").
//
// Progress: workgroups take tasks (segment, slice) from one queue in order,
// the slices of a segment consecutive. A workgroup only waits for tasks of
// its own segment; the segment at the queue head is the only one with both
// taken and untaken tasks, so as long as G <= the workgroups that can run
// at once (the host caps G by the resident grid), every wait ends. A spin
// bound (`timeout` wall-clock ticks) still ends every wait -- e.g. when
// another process holds CUs: the gang then raises `abort` and every member
// exits without writing its segment back, which therefore stays in the
// kEqualize phase and simply repeats this qcml iteration (re-equalized with
// the unchanged dispersion = the same pseudodata) under the one-workgroup
// k_brent, which the host switches to once it sees the flag.
constexpr int kGangThreads = 256;

template <int M>
__global__ __launch_bounds__(kGangThreads) void k_brent_gang(
    const double* __restrict__ pd, int64_t n,
    const int64_t* __restrict__ seg_start /* D + 1 */, int S, int C,
    const int32_t* __restrict__ rep_idx /* C x kMaxReps */,
    const int32_t* __restrict__ n_rep /* C */, SegState* __restrict__ st,
    const int* __restrict__ seg_flags, double* __restrict__ result,
    int* __restrict__ queue, const int32_t* __restrict__ task_seg,
    const int32_t* __restrict__ task_g, int T, int64_t P,
    double* __restrict__ part /* 2 x S x gmax */, int* __restrict__ tag /* 2 x S x gmax */,
    int gmax, int* __restrict__ abort_flag, long long timeout,
    unsigned long long* __restrict__ work_count, int epoch,
    const int32_t* __restrict__ gate_meta, int live_max) {
  // gate (device-side choice, see k_brent): run while the live segments
  // leave CUs idle, unless a gang has aborted
  if (gate_meta && (gate_meta[3] >= live_max || *abort_flag)) return;
  // the compact task list of k_seg_update when it built one
  if (gate_meta && gate_meta[4] >= 0 && gate_meta[4] < T) T = gate_meta[4];
  __shared__ SegState s_st;
  __shared__ double wpart[kGangThreads / 64];
  __shared__ int s_next, s_more, s_abort;
  __shared__ LogTab s_tab[kLogTabLen];  // the NLL log's table, as k_brent
  for (int t = threadIdx.x; t < kLogTabLen; t += kGangThreads) s_tab[t] = kLogTab[t];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  while (true) {
    __syncthreads();  // s_next / s_st reuse
    if (threadIdx.x == 0) s_next = atomicAdd(queue, 1);
    __syncthreads();
    const int t = s_next;
    if (t >= T) break;
    const int s = task_seg[t], g = task_g[t];
    if (s < 0) continue;  // unused entry of a device-built task table
    // every member reads the phase before the gang's first evaluation, so
    // before member 0 can write the segment back
    if (st[s].phase != kEqualize) continue;
    if (threadIdx.x == 0) {
      s_st = st[s];
      s_st.flags |= seg_flags[s];
      s_abort = 0;
    }
    const int d = s / C, c = s - (s / C) * C;
    const int nr = n_rep[c];
    const int64_t b = seg_start[d], e = seg_start[d + 1];
    const int G = (int)((e - b + P - 1) / P);
    const int64_t sb = b + (int64_t)g * P;
    const int64_t se = (sb + P < e) ? sb + P : e;
    int ri[M];
#pragma unroll
    for (int k = 0; k < M; ++k) ri[k] = (k < nr) ? rep_idx[c * kMaxReps + k] : 0;
    int evals = 0;
    __syncthreads();
    while (true) {
      const NllConst kc = s_st.k;
      // the slice (no LDS head), two pixels per trip for M <= 4, as k_brent
      // (the progress priority of k_brent measured neutral here, r06z)
      double acc = (kc.r >= kNllLargeR)
          ? brent_segment_sum<M, kGangThreads, 2>(nullptr, 0, pd, n, ri, nr, sb, sb, se, kc, s_tab)
          : (kc.r >= kNllMidR)
          ? brent_segment_sum<M, kGangThreads, 1>(nullptr, 0, pd, n, ri, nr, sb, sb, se, kc, s_tab)
          : brent_segment_sum<M, kGangThreads, 0>(nullptr, 0, pd, n, ri, nr, sb, sb, se, kc, s_tab);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
      if (lane == 0) wpart[wid] = acc;
      __syncthreads();
      if (wid == 0) {
        double mine = 0.0;
#pragma unroll
        for (int w = 0; w < kGangThreads / 64; ++w) mine += wpart[w];
        double total = mine;
        bool ok = true;
        if (G > 1) {
          const size_t base = ((size_t)(evals & 1) * S + s) * gmax;
          // tags carry the launch's epoch: no tag from an earlier launch
          // matches, so the tags need no clearing between launches
          // (evals < kMaxFun = 500 < 1024)
          const int want = (epoch << 10) | (evals + 1);
          if (lane == 0) {
            __hip_atomic_store(&part[base + g], mine, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            __builtin_amdgcn_s_waitcnt(0);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            __hip_atomic_store(&tag[base + g], want, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          }
          // wave 0 polls the G tags, lane q the slices q, q + 64, ...
          const long long t0 = wall_clock64();
          while (true) {
            bool mine_ready = true;
            for (int q = lane; q < G; q += 64)
              mine_ready &= __hip_atomic_load(&tag[base + q], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) == want;
            if (__all(mine_ready)) break;
            __builtin_amdgcn_s_sleep(1);
            const bool stop =
                __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                wall_clock64() - t0 > timeout;
            if (stop) {
              if (lane == 0)
                __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              ok = false;
              break;
            }
          }
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
          __builtin_amdgcn_s_waitcnt(0);
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
          if (ok) {
            double sum = 0.0;
            for (int q = lane; q < G; q += 64)
              sum += __hip_atomic_load(&part[base + q], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
            total = sum;  // the same fixed tree in every member
          }
        }
        if (lane == 0) {
          if (ok) {
            seg_step_ool(&s_st, total, nr);
            s_more = (s_st.phase == kNll) ? 1 : 0;
          } else {
            s_abort = 1;
            s_more = 0;
          }
        }
      }
      ++evals;
      __syncthreads();  // s_st / s_more / s_abort / wpart
      if (!s_more) break;
    }
    if (s_abort) return;  // the whole workgroup: s_abort is uniform
    if (threadIdx.x == 0 && g == 0) {
      st[s] = s_st;
      if (s_st.phase == kDone) result[s] = s_st.result;
      atomicAdd(&work_count[1], (unsigned long long)(e - b) * nr * evals);
    }
  }
}

// Per-pixel LRT (lrt.py:7-50) in the reference pixel order; disp from the
// (D, C) table (analysis.py:218: disp = disp_fn(dist), evaluated per d).
// TAB: the pipeline's call -- refit, the (D, C) table read by dist, no wide
// dispersions -- as compile-time facts, so the kernel carries none of the
// other modes' code (their registers and the SGPR spills around their
// uniform branches); the runtime flags are then ignored.
#ifndef H3D_LRT_WAVES
#define H3D_LRT_WAVES 1
#endif
template <int M, int CM, bool TAB = false>
__global__ __launch_bounds__(kBlock, TAB ? H3D_LRT_WAVES : 1) void k_lrt(
    const int32_t* __restrict__ raw, const double* __restrict__ f,
    const int32_t* __restrict__ dist, const double* __restrict__ table,
    int64_t n, int R, int C, int D, const int32_t* __restrict__ cond_of_rep,
    int refit, double* __restrict__ p, double* __restrict__ llr,
    double* __restrict__ mu0, double* __restrict__ mu1,
    double* __restrict__ disp_out, int* __restrict__ flags, int wide) {
  int cond[M];
#pragma unroll
  for (int k = 0; k < M; ++k) cond[k] = (k < R) ? cond_of_rep[k] : -1;
  // the logpmf rows' log table in LDS (16 lookups per pixel at R = 4, each
  // on its term's dependency chain)
  __shared__ LogTab s_tab[kLogTabLen];
  for (int t = threadIdx.x; t < kLogTabLen; t += blockDim.x) s_tab[t] = kLogTab[t];
  __syncthreads();
  int fl_all = 0;
  if constexpr (TAB) {
    refit = 1;
    wide = 0;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    // dist == nullptr: `table` holds per-pixel dispersions, (n, C) -- or,
    // with `wide`, per replicate (n, R): lrt.py's disp argument as given
    const int d = (TAB || dist) ? dist[i] : 0;
    const double* trow = (TAB || dist) ? table + (int64_t)d * C
                                       : table + i * (wide ? R : C);
    const bool inb = (TAB || dist) ? (d >= 0 && d < D) : true;
    double dc[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) dc[c] = (c < C && inb && !wide) ? trow[c] : NAN;
    // counts stay int32 in registers (converted exactly where used): the
    // M = 24 / 32 instantiations must not spill
    int32_t x[M];
    double fv[M], a[M];
#pragma unroll
    for (int k = 0; k < M; ++k) {
      if (k < R) {
        x[k] = raw[i * R + k];
        fv[k] = f[i * R + k];
        double ak = 0.0;
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (c == cond[k]) ak = dc[c];
        a[k] = wide ? trow[k] : ak;
      } else {
        x[k] = 0;
        fv[k] = 1.0;
        a[k] = 1.0;
      }
    }
    double pv, lv, m0, m1[CM];
    fl_all |= lrt_pixel<M, CM>(x, fv, a, cond, R, C, refit != 0, &pv, &lv, &m0,
                               m1, s_tab);
    p[i] = pv;
    llr[i] = lv;
    mu0[i] = m0;
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) {
        mu1[i * C + c] = m1[c];
        if (disp_out) disp_out[i * C + c] = dc[c];
      }
  }
  if (fl_all) atomicOr(flags, fl_all);
}

}  // namespace h3d
