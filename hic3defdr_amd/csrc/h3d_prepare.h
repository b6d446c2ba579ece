// prepare_data kernels: union pixel table of R replicate CSR band matrices
// (reference util/matrices.py:92-129 + analysis/analysis.py:91-101) and the
// distance-conditional median-of-ratios size factors (util/scaling.py:68-127,
// util/binning.py:4-25).
//
// Union: every in-band non-zero entry of every replicate is staged (compacted
// per replicate, so scratch and the 2^31 cap follow the band) as a 64-bit key
// row * n_bins + col; one radix sort of (key, entry) groups a pixel's
// replicate entries into a run; a run is kept when the sum of its
// deconvoluted values (inverse bias 0 on zero-bias bins) is finite and > 0
// (the reference drops zero sums and filters isfinite / >= mean_thresh*R = 0).
// Keys sort lexicographically in (row, col): the reference's order (csr sum
// -> tocoo).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "h3d_model.h"

namespace h3d {

// (the union state PrepUnion lives in h3d_ctx.h, inside the h3d_ctx)

// row id of every CSR entry (one thread per row)
static __global__ void k_csr_rows(const int64_t* __restrict__ indptr, int n_bins,
                           int32_t* __restrict__ row_of) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_bins) return;
  for (int64_t j = indptr[i]; j < indptr[i + 1]; ++j) row_of[j] = i;
}

// entries staged for the union: in the band (0 <= col - row <= dist_max) and
// non-zero -- wipe_distances' survivors (util/matrices.py:41-62). Zero-bias
// bins are NOT dropped here: the reference's raw gather reads the raw matrix
// at every union pixel (analysis.py:91-95), so a replicate whose bias is 0 at
// a pixel another replicate put in the union still reports its count (and
// balanced v / 0 = inf); k_run_keep decides union membership.
__device__ inline bool union_stage(int i, int c, double v, int n_bins, int dist_max) {
  const int d = c - i;
  return (d >= 0) && (d <= dist_max) && (c < n_bins) && (v != 0.0);
}

static __global__ void k_union_flags(const int32_t* __restrict__ row_of,
                                     const int32_t* __restrict__ col,
                                     const double* __restrict__ val, int64_t n_ent,
                                     int n_bins, int dist_max,
                                     int32_t* __restrict__ flag) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n_ent;
       j += (int64_t)gridDim.x * blockDim.x)
    flag[j] = union_stage(row_of[j], col[j], val[j], n_bins, dist_max) ? 1 : 0;
}

// the kept entries of one replicate, compacted to ent_offset + pos[j]
// (pos = exclusive scan of the flags): only in-band entries are staged
static __global__ void k_union_keys(const int32_t* __restrict__ row_of,
                                    const int32_t* __restrict__ col,
                                    const double* __restrict__ val,
                                    const int32_t* __restrict__ flag,
                                    const int32_t* __restrict__ pos, int64_t n_ent,
                                    int64_t ent_offset, int rep, int n_bins,
                                    int64_t* __restrict__ keys,
                                    int32_t* __restrict__ ent_idx,
                                    int32_t* __restrict__ ent_rep,
                                    double* __restrict__ ent_val) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n_ent;
       j += (int64_t)gridDim.x * blockDim.x) {
    if (!flag[j]) continue;
    const int64_t g = ent_offset + pos[j];
    keys[g] = (int64_t)row_of[j] * n_bins + col[j];
    ent_idx[g] = (int32_t)g;
    ent_rep[g] = rep;
    ent_val[g] = val[j];
  }
}

// head[i] = 1 where a new non-sentinel key starts
static __global__ void k_run_heads(const int64_t* __restrict__ keys, int64_t n,
                            int64_t sentinel, int32_t* __restrict__ head) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = keys[i];
    head[i] = (k != sentinel && (i == 0 || keys[i - 1] != k)) ? 1 : 0;
  }
}

// run starts: run r begins at the entry whose inclusive head-scan equals r+1
static __global__ void k_run_starts(const int32_t* __restrict__ head,
                             const int32_t* __restrict__ run_incl, int64_t n,
                             int64_t* __restrict__ run_start) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    if (head[i]) run_start[run_incl[i] - 1] = i;
}

// keep flag per run: deconvoluted sum finite and > 0
static __global__ void k_run_keep(const int64_t* __restrict__ keys,
                           const int32_t* __restrict__ ent_sorted,
                           const int64_t* __restrict__ run_start,
                           int64_t n_runs, int64_t n_ent, int64_t sentinel,
                           const int32_t* __restrict__ ent_rep,
                           const double* __restrict__ ent_val, int R,
                           int n_bins, const double* __restrict__ bias,
                           int32_t* __restrict__ keep) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_runs;
       r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = run_start[r];
    const int64_t key = keys[b];
    const int64_t i = key / n_bins, c = key - i * n_bins;
    double tot = 0.0;
    for (int64_t j = b; j < n_ent && keys[j] == key; ++j) {
      const int e = ent_sorted[j];
      const int rep = ent_rep[e];
      // deconvolute(invert=True) (matrices.py:8-38): inverse bias 0 where
      // the bias is 0, so such entries add nothing to the union total
      const double b_i = bias[i * R + rep], b_c = bias[c * R + rep];
      const double bi = b_i == 0.0 ? 0.0 : 1.0 / b_i, bc = b_c == 0.0 ? 0.0 : 1.0 / b_c;
      tot += (bi * ent_val[e]) * bc;
    }
    keep[r] = (tot > 0.0 && tot - tot == 0.0) ? 1 : 0;
  }
}

// fill row/col/raw/balanced for kept runs (px = exclusive scan of keep)
static __global__ void k_union_fill(const int64_t* __restrict__ keys,
                             const int32_t* __restrict__ ent_sorted,
                             const int64_t* __restrict__ run_start,
                             const int32_t* __restrict__ keep,
                             const int32_t* __restrict__ px_incl,
                             int64_t n_runs, int64_t n_ent,
                             const int32_t* __restrict__ ent_rep,
                             const double* __restrict__ ent_val, int R,
                             int n_bins, const double* __restrict__ bias,
                             int32_t* __restrict__ row, int32_t* __restrict__ col,
                             int64_t* __restrict__ raw,
                             double* __restrict__ balanced) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_runs;
       r += (int64_t)gridDim.x * blockDim.x) {
    if (!keep[r]) continue;
    const int64_t p = px_incl[r] - 1;
    const int64_t b = run_start[r];
    const int64_t key = keys[b];
    const int64_t i = key / n_bins, c = key - i * n_bins;
    row[p] = (int32_t)i;
    col[p] = (int32_t)c;
    for (int k = 0; k < R; ++k) {
      raw[p * R + k] = 0;
      balanced[p * R + k] = 0.0 / (bias[i * R + k] * bias[c * R + k]);
    }
    for (int64_t j = b; j < n_ent && keys[j] == key; ++j) {
      const int e = ent_sorted[j];
      const int k = ent_rep[e];
      const double v = ent_val[e];
      raw[p * R + k] = (int64_t)v;
      balanced[p * R + k] = v / (bias[i * R + k] * bias[c * R + k]);
    }
  }
}

// ---- size factors ---------------------------------------------------------

// equal_bin with the stable tie order: sorted position k -> bin
// floor(k * (n_bins / n)) (numpy linspace(0, n_bins, n, endpoint=False,
// dtype=int)); bin_of_sorted[k]
static __global__ void k_equal_bin(int64_t n, int n_bins, int32_t* __restrict__ bin) {
  const double step = (double)n_bins / (double)n;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x)
    bin[k] = (int32_t)floor((double)k * step);
}

// bin boundaries over the sorted positions: bin_start[b] = first k with
// bin[k] >= b (b = 0..n_bins)
static __global__ void k_bin_bounds(const int32_t* __restrict__ bin, int64_t n,
                             int n_bins, int64_t* __restrict__ bin_start) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > n_bins) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (bin[mid] < b)
      lo = mid + 1;
    else
      hi = mid;
  }
  bin_start[b] = lo;
}

// ratio keys for the median: for sorted position k of bin b, replicate r:
// data / gmean(data, pseudocount 1) when every replicate > 0 (scaling.py:44-47)
// else +inf (sorts past the valid ones); valid rows counted per bin.
static __global__ void k_mor_keys(const double* __restrict__ balanced,
                           const int32_t* __restrict__ perm, int64_t n, int R,
                           const int32_t* __restrict__ bin,
                           double* __restrict__ keys,
                           int32_t* __restrict__ valid_per_bin) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = perm[k];
    bool ok = true;
    // gmean(x, pseudocount 1) = exp(nanmean(log(x + 1))) - 1 over the row:
    // numpy's row reduction (sequential below 8 replicates, pairwise from 8)
    double lg[kMaxReps];
    for (int r = 0; r < R; ++r) {
      const double v = balanced[i * R + r];
      ok = ok && (v > 0.0);
      lg[r] = log(v + 1);
    }
    const double gm = exp(np_sum<kMaxReps>(lg, R) / R) - 1;
    for (int r = 0; r < R; ++r)
      keys[(int64_t)r * n + k] = ok ? balanced[i * R + r] / gm : INFINITY;
    // valid rows per bin: bins are sorted along k, so a wave spans one or
    // two bins -- one atomic per (wave, bin) instead of one per row
    const int b = bin[k];
    unsigned long long pend = __ballot(ok);
    while (pend) {
      const int leader = __ffsll((long long)pend) - 1;
      const int bl = __shfl(b, leader, 64);
      const unsigned long long same = __ballot(ok && b == bl) & pend;
      if ((int)(threadIdx.x & 63) == leader) atomicAdd(&valid_per_bin[bl], (int)__popcll(same));
      pend &= ~same;
    }
  }
}

// per (replicate, bin): median of the first `valid` sorted ratios; d_per_bin
// = mean distance of the bin (exact: integer sum)
static __global__ void k_mor_median(const double* __restrict__ sorted_keys,
                             const int64_t* __restrict__ bin_start,
                             const int32_t* __restrict__ valid, int n_bins,
                             int64_t n, int R, double* __restrict__ s_per_bin) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_bins * R) return;
  const int b = t % n_bins, r = t / n_bins;
  const int64_t base = (int64_t)r * n + bin_start[b];
  const int64_t m = valid[b];
  double med = NAN;
  if (m > 0) {
    if (m % 2)
      med = sorted_keys[base + m / 2];
    else
      med = (sorted_keys[base + m / 2 - 1] + sorted_keys[base + m / 2]) / 2.0;
  }
  s_per_bin[(int64_t)b * R + r] = med;
}

static __global__ void k_bin_dist_sum(const int32_t* __restrict__ dist_sorted,
                               const int64_t* __restrict__ bin_start,
                               int n_bins, double* __restrict__ d_per_bin) {
  // one workgroup per bin; integer sum, so the reduction order is free
  __shared__ long long part[16];
  const int b = blockIdx.x;
  if (b >= n_bins) return;
  long long s = 0;
  for (int64_t k = bin_start[b] + threadIdx.x; k < bin_start[b + 1]; k += blockDim.x)
    s += dist_sorted[k];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w];
    const int64_t cnt = bin_start[b + 1] - bin_start[b];
    d_per_bin[b] = cnt ? (double)t / (double)cnt : NAN;
  }
}

// sf[i, r] = interp1d(d_per_bin, s_per_bin[:, r], extrapolate)(dist[i]) over
// the non-empty bins (compacted by the host: m points)
static __global__ void k_sf_interp(const int32_t* __restrict__ dist, int64_t n, int R,
                            const double* __restrict__ xp,
                            const double* __restrict__ yp /* m x R */, int m,
                            double* __restrict__ sf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double x = (double)dist[i];
    int lo = 0, hi = m;  // lower_bound
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (xp[mid] < x)
        lo = mid + 1;
      else
        hi = mid;
    }
    int idx = lo < 1 ? 1 : (lo > m - 1 ? m - 1 : lo);
    const int a = idx - 1, b = idx;
    for (int r = 0; r < R; ++r) {
      const double slope = (yp[(int64_t)b * R + r] - yp[(int64_t)a * R + r]) / (xp[b] - xp[a]);
      sf[i * R + r] = slope * (x - xp[a]) + yp[(int64_t)a * R + r];
    }
  }
}

// exact-distance mode: sf[i, r] = s_per_bin[bin(dist[i]), r]
static __global__ void k_sf_exact(const int32_t* __restrict__ perm,
                           const int32_t* __restrict__ bin, int64_t n, int R,
                           const double* __restrict__ s_per_bin,
                           double* __restrict__ sf) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = perm[k];
    for (int r = 0; r < R; ++r) sf[i * R + r] = s_per_bin[(int64_t)bin[k] * R + r];
  }
}

// bin of every pixel in its original position (bin_of_sorted scattered
// through the distance sort's permutation)
static __global__ void k_scatter_bin(const int32_t* __restrict__ perm,
                              const int32_t* __restrict__ bin_of_sorted,
                              int64_t n, int32_t* __restrict__ bin_orig) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x)
    bin_orig[perm[k]] = bin_of_sorted[k];
}

// simple_scaling's column sums per (bin, replicate) (scaling.py:64:
// np.sum(data, axis=0) over the bin's rows in their original order, which
// numpy accumulates row by row): one lane per (bin, replicate) walks the
// bin's members (grouped by bin, original order inside) sequentially
static __global__ void k_bin_colsum(const double* __restrict__ balanced,
                             const int32_t* __restrict__ members,
                             const int64_t* __restrict__ bin_start, int n_bins,
                             int R, double* __restrict__ colsum) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_bins * R) return;
  const int b = t / R, r = t - (t / R) * R;
  const int64_t e = bin_start[b + 1];
  double s = 0.0;
  int64_t k = bin_start[b];
  // the loads are independent: keep 8 in flight ahead of the dependent adds
  for (; k + 8 <= e; k += 8) {
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = balanced[(int64_t)members[k + j] * R + r];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
  }
  for (; k < e; ++k) s += balanced[(int64_t)members[k] * R + r];
  colsum[(int64_t)b * R + r] = s;
}

// exact mode bins: bin of sorted position = its distance rank among distinct
// distances (head flags scanned on device)
static __global__ void k_dist_heads(const int32_t* __restrict__ dist_sorted, int64_t n,
                             int32_t* __restrict__ head) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x)
    head[k] = (k == 0 || dist_sorted[k] != dist_sorted[k - 1]) ? 1 : 0;
}

static __global__ void k_minus_one(int32_t* __restrict__ v, int64_t n) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x)
    v[k] -= 1;
}

// ---- the disp pixels of a chromosome (estimate_disp / lrt inputs) ----------

// The disp_idx pixels of one chromosome, compacted in pixel order: raw, dist
// = col - row and f = bias[row] * bias[col] * sf -- the reference's products
// in its order (analysis.py:174-183 and :272-275, numpy evaluates left to
// right; a product of three never contracts, so the bits are numpy's). sel
// = the selected union-pixel indices (DeviceSelect over disp_idx). sf is
// (N, R), or (R,) with sf_per_rep (the non-conditional norms). Rows of R <= 4
// int32 / f64 go out as whole 16 B words where aligned.
static __global__ void k_disp_pixels(const int32_t* __restrict__ sel, int64_t n_out,
                                     const int32_t* __restrict__ row,
                                     const int32_t* __restrict__ col,
                                     const int32_t* __restrict__ raw,
                                     const double* __restrict__ sf, int sf_per_rep,
                                     const double* __restrict__ bias, int R,
                                     int32_t* __restrict__ raw_out,
                                     double* __restrict__ f_out,
                                     int32_t* __restrict__ dist_out) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n_out;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = sel[j];
    const int64_t r0 = row[i], c0 = col[i];
    dist_out[j] = (int32_t)(c0 - r0);
    for (int k = 0; k < R; ++k) {
      raw_out[j * R + k] = raw[i * R + k];
      const double bb = bias[r0 * R + k] * bias[c0 * R + k];
      f_out[j * R + k] = bb * (sf_per_rep ? sf[k] : sf[i * R + k]);
    }
  }
}

// f of re-sharded pixels rebuilt on the rank that receives them (the distance
// re-shard, parallel.disp_per_dist_by_distance): the sender ships (row,
// distance, chromosome, size-factor row) instead of f's 8R bytes, every rank
// holds the genome's bias rows (boff: chromosome g's first row, g + 1's
// bounds it) and size-factor rows (soff), and f is the product
// k_disp_pixels forms, in its order: (bias[row] * bias[row + d]) * sf -- so
// the rebuilt f is the sender's bit for bit. A key outside the tables
// (chromosome, row + d or the size-factor row) gives NaN and sets *bad.
static __global__ void k_pixel_f(const int32_t* __restrict__ row,
                                 const int32_t* __restrict__ dist,
                                 const int32_t* __restrict__ chrom,
                                 const int32_t* __restrict__ sfi, int64_t n, int R,
                                 const double* __restrict__ bias,
                                 const int64_t* __restrict__ boff,
                                 const double* __restrict__ sf,
                                 const int64_t* __restrict__ soff, int nchrom,
                                 double* __restrict__ f_out, int* __restrict__ bad) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int g = chrom[j];
    const int64_t r0 = row[j], c0 = r0 + dist[j], s = sfi[j];
    bool ok = g >= 0 && g < nchrom;
    int64_t b0 = 0, nb = 0, s0 = 0, ns = 0;
    if (ok) {
      b0 = boff[g];
      nb = boff[g + 1] - b0;
      s0 = soff[g];
      ns = soff[g + 1] - s0;
      ok = r0 >= 0 && r0 <= c0 && c0 < nb && s >= 0 && s < ns;
    }
    if (!ok) {
      for (int k = 0; k < R; ++k) f_out[j * R + k] = NAN;
      atomicOr(bad, 1);
      continue;
    }
    for (int k = 0; k < R; ++k) {
      const double bb = bias[(b0 + r0) * R + k] * bias[(b0 + c0) * R + k];
      f_out[j * R + k] = bb * sf[(s0 + s) * R + k];
    }
  }
}

// prepare_data's scaled and disp_idx (analysis.py:109-115):
//   scaled = balanced / size_factors,
//   mean = np.dot(scaled, design) / n_c,
//   disp_idx = all(mean >= mean_thresh, axis=1) & (dist >= dist_thresh_min).
// The product is summed over every replicate in order with the design's 0 / 1
// weights (a weight-0 term adds s * 0: 0, or NaN for an infinite s, as in the
// BLAS product). A row whose decision could depend on the product's
// summation order -- a non-finite scaled value, or a condition mean within
// 1e-12 relative of the threshold -- is flagged 2, and the host decides it
// with numpy's own product (h3d_scale_disp_dev). scaled goes out (n, R);
// flag (n) is 0 / 1 / 2.
struct ScaleDispArgs {
  uint32_t cond_mask[kMaxConds];  // replicate bits of each condition
  double count[kMaxConds];        // replicates per condition (the divisor)
  int C;
  double mean_thresh;
  int dist_min;
};

static __global__ void k_scale_disp(const double* __restrict__ bal,
                                    const double* __restrict__ sf, int sf_per_rep,
                                    const int32_t* __restrict__ row,
                                    const int32_t* __restrict__ col, int64_t n, int R,
                                    ScaleDispArgs a, double* __restrict__ scaled,
                                    uint8_t* __restrict__ flag) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    bool near = false;
    for (int k = 0; k < R; ++k) {
      const double v = bal[i * R + k] / (sf_per_rep ? sf[k] : sf[i * R + k]);
      scaled[i * R + k] = v;
      near |= !isfinite(v);
    }
    bool keep = (col[i] - row[i]) >= a.dist_min;
    for (int c = 0; c < a.C; ++c) {
      double acc = 0.0;
      for (int k = 0; k < R; ++k) {
        // the same IEEE quotient as above (re-derived, not re-read)
        const double v = bal[i * R + k] / (sf_per_rep ? sf[k] : sf[i * R + k]);
        acc += ((a.cond_mask[c] >> k) & 1u) ? v : v * 0.0;
      }
      const double mean = acc / a.count[c];
      keep &= mean >= a.mean_thresh;
      near |= fabs(mean - a.mean_thresh) <= 1e-12 * fabs(a.mean_thresh);
    }
    flag[i] = near ? 2 : (keep ? 1 : 0);
  }
}

// disp[i, c] = table[dist[i], c] (analysis.py:218 disp_fn(dist): the fitted
// function evaluated at integer distances IS its tabulation); NaN outside
// [0, D)
static __global__ void k_table_gather(const double* __restrict__ table, int D, int C,
                                      const int32_t* __restrict__ dist, int64_t n,
                                      double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int d = dist[i];
    const bool in = d >= 0 && d < D;
    for (int c = 0; c < C; ++c) out[i * C + c] = in ? table[(int64_t)d * C + c] : NAN;
  }
}

}  // namespace h3d
