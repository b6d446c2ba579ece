/* h3d.h — C ABI of libh3d.so, the MI355X-native hot path of hic3defdr.
 *
 * The reference (thomasgilgenast/hic3defdr 0.2.1) is pure Python and has no
 * FFI; this ABI sits behind its operator-level functions, which the Python
 * mirror (hic3defdr_amd) binds with ctypes:
 *
 *   h3d_union_*            <- util/matrices.py:92-129 sparse_union (+ the raw /
 *                              balanced gathers, analysis/analysis.py:91-101)
 *   h3d_size_factors_cmor  <- util/scaling.py:108-127 conditional_mor
 *   h3d_size_factors       <- util/scaling.py:10-149 (every norm prepare_data
 *                              dispatches, analysis/analysis.py:104-108)
 *   h3d_disp_per_dist      <- analysis/analysis.py:185-206 (estimator per
 *                              distance/condition; util/dispersion.py:10-80
 *                              qcml/cml, util/scaled_nb.py:71-275)
 *   h3d_disp_table         <- analysis/analysis.py:208-218 +
 *                              util/lowess.py:10-244 (the fitted disp_fn,
 *                              tabulated on every integer distance)
 *   h3d_lrt                <- util/lrt.py:7-50 (+ analysis/analysis.py:272-278)
 *   h3d_lrt_wide           <- util/lrt.py:7 lrt(raw, f, disp, design) as called
 *   h3d_cml                <- util/dispersion.py:46-80 cml
 *   h3d_bh / _ctx / _dev   <- analysis/analysis.py:286-303 (lib5c
 *                              adjust_pvalues = BH)
 *   h3d_find_clusters      <- util/clusters.py:73-97 find_clusters (threshold /
 *                              classify, analysis.py:366-486)
 *   h3d_format_clusters    <- util/clusters.py:129-130 save_clusters text,
 *                              util/cluster_table.py:67 "cluster" column
 *   h3d_lrt_poisson        <- analysis/alternatives.py:17-42 poisson_lrt
 *                              (Poisson3DeFDR.lrt, :73-115)
 *   h3d_mme_per_pixel      <- util/dispersion.py:83-104 mme_per_pixel
 *                              (Unsmoothed3DeFDR.estimate_disp,
 *                              alternatives.py:119-137)
 *
 * Conventions: 0 on success, a negative H3D_E* code otherwise (the message is
 * in h3d_last_error(), thread-local). Host buffers are C-contiguous and owned
 * by the caller; device buffers of the *_dev entry points are device pointers
 * the caller owns. Calls are synchronous unless they take a stream. One ctx
 * per device; a ctx is not shared between threads.
 */
#ifndef H3D_H_
#define H3D_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define H3D_OK 0
#define H3D_EARG (-1)    /* bad argument: null pointer, size, shape        */
#define H3D_EHIP (-2)    /* HIP runtime error                               */
#define H3D_ENOCONV (-3) /* numerical failure the reference raises on      */
#define H3D_ENOMEM (-4)  /* device allocation failed                       */
#define H3D_EINPUT (-5)  /* invalid numeric input (reference asserts)      */
#define H3D_ENODEV (-6)  /* no usable gfx950 device                        */

#define H3D_EST_QCML 0
#define H3D_EST_CML 1
#define H3D_EST_MME 2

/* size-factor methods (util/scaling.py) */
#define H3D_NORM_CONDITIONAL_MOR 0     /* :108-127, (n, R)                */
#define H3D_NORM_CONDITIONAL_SCALING 1 /* :130-149, (n, R)                */
#define H3D_NORM_MEDIAN_OF_RATIOS 2    /* :27-47, (R,)                    */
#define H3D_NORM_SIMPLE_SCALING 3      /* :50-65, (R,)                    */
#define H3D_NORM_NO_SCALING 4          /* :10-24, (R,)                    */

/* per-segment / per-pixel status bits (also in *flags outputs) */
#define H3D_FLAG_NOROOT 1   /* all-zero counts: no MLE (ref ValueError)      */
#define H3D_FLAG_NOCONV 2   /* MLE solver did not converge                   */
#define H3D_FLAG_BRENT 4    /* bounded Brent failed (ref assert res.success) */
#define H3D_FLAG_QGUARD 8   /* qcml did not converge in 1000 iterations      */
#define H3D_FLAG_BADIN 16   /* alpha/b not positive finite (ref assert)      */

typedef struct h3d_ctx h3d_ctx;

/* All-reduce hook for multi-GPU estimate_disp: called between data passes
 * with a DEVICE buffer of `count` doubles that must be summed in place across
 * ranks on the ctx stream (e.g. torch.distributed.all_reduce over RCCL).
 * Return 0 on success. */
typedef int (*h3d_allreduce_fn)(double* dev_buf, int64_t count, void* user);

int h3d_version(void);
int h3d_device_count(void);
h3d_ctx* h3d_open(int device);
void h3d_close(h3d_ctx* ctx);
const char* h3d_last_error(void);
/* stream the ctx launches on (hipStream_t); NULL = the ctx's own stream */
int h3d_set_stream(h3d_ctx* ctx, void* stream);
/* qcml's convergence tolerance for the ctx's later estimate_disp calls
 * (util/dispersion.py:10-43 qcml(..., tol=1e-4): iterate while
 * |disp - new disp| > tol); default 1e-4, the value the reference's
 * estimate_disp uses. H3D_EARG for a negative or non-finite tol. */
int h3d_set_qcml_tol(h3d_ctx* ctx, double tol);

/* ---- prepare_data ------------------------------------------------------ */

/* Native reader of the replicate contact matrices: scipy.sparse.save_npz
 * archives as the reference loads them with scipy.sparse.load_npz
 * (analysis/analysis.py:94,100 through util/matrices.py:122-124). Host only,
 * no context. _info reads the archive's directory and the shape / format /
 * data headers; _read inflates indptr, indices and data (libdeflate when
 * the system has libdeflate.so.0, else zlib; one thread each) into caller
 * buffers of n_rows + 1, nnz, nnz entries, converting to
 * int64 / int32 / float64, and sets *canonical = 1 when every row's columns
 * are strictly increasing (the layout h3d_union_count takes as is). H3D_EARG
 * for a missing file, a non-CSR archive or an unsupported dtype. */
int h3d_npz_csr_info(const char* path, int64_t* n_rows, int64_t* n_cols,
                     int64_t* nnz);
int h3d_npz_csr_read(const char* path, int64_t n_rows, int64_t nnz,
                     int64_t* indptr, int32_t* indices, double* data,
                     int* canonical);
/* The same, with `slack` writable bytes before `indices` and before `data`:
 * a member of the target's width (little-endian int32 indices; 8-byte data:
 * float64, or int64 / uint64 converted in place) whose .npy header fits in
 * the slack is inflated in place (the header lands in the slack), with no
 * scratch copy. slack 0 = h3d_npz_csr_read. */
int h3d_npz_csr_read_slack(const char* path, int64_t n_rows, int64_t nnz,
                           int64_t* indptr, int32_t* indices, double* data,
                           int64_t slack, int* canonical);
/* 1 when the reader inflates through libdeflate, 0 through zlib. */
int h3d_npz_backend(void);
/* A one-column text file as np.loadtxt reads it -- load_bias's bias vectors
 * (core.py:35-60: np.loadtxt per replicate file): one number per line, blank
 * lines and '#' comments skipped, values by strtod (correctly rounded, as
 * numpy's parser). *n = the values written to out (capacity cap). H3D_EINPUT
 * for any line that is not exactly one decimal number (the caller then reads
 * the file with np.loadtxt and its errors); H3D_EARG for a missing file or
 * more than cap values. Host only. */
int h3d_read_text_column(const char* path, double* out, int64_t cap, int64_t* n);

/* Union pixel set of R upper-triangular CSR replicate matrices restricted to
 * 0 <= col-row <= dist_max and to bins whose bias is non-zero in every
 * replicate (matrices.py:92-129 with deconvolute(invert=True)). Two-pass:
 * count, then fill. indptr[r] has n_bins+1 entries, indices[r]/data[r] nnz[r].
 * bias is (n_bins, R) row-major and already bias_thresh-filtered
 * (core.py:35-60). */
int h3d_union_count(h3d_ctx* ctx, int R, int n_bins, const int64_t* const* indptr,
                    const int32_t* const* indices, const double* const* data,
                    const int64_t* nnz, const double* bias, int dist_max,
                    int64_t* n_px_out);
/* row/col (n_px), raw (n_px, R) int64 = summed counts, balanced (n_px, R) =
 * raw / (bias[row, r] * bias[col, r]) (analysis.py:91-101). */
int h3d_union_fill(h3d_ctx* ctx, int32_t* row, int32_t* col, int64_t* raw,
                   double* balanced, int64_t n_px);
/* h3d_union_fill that also leaves the union in caller-owned DEVICE buffers
 * (each may be NULL): d_row / d_col (n_px) int32, d_raw (n_px, R) int32 --
 * H3D_EINPUT, after the host outputs are written, if a count does not fit
 * --, d_balanced (n_px, R). The host `balanced` may be NULL when d_balanced
 * is not (the device computes scaled from it, h3d_scale_disp_dev), the host
 * `raw` when d_raw is not (the caller fetches it in the background). The
 * product keeps a chromosome resident this way between prepare_data and
 * estimate_disp / lrt (analysis.py:128-133 writes the same arrays to the
 * outdir, :169-183 and :261-275 read them back). */
int h3d_union_fill_dev(h3d_ctx* ctx, int32_t* row, int32_t* col, int64_t* raw,
                       double* balanced, int64_t n_px, int32_t* d_row,
                       int32_t* d_col, int32_t* d_raw, double* d_balanced);

/* Distance-conditional median-of-ratios size factors (scaling.py:68-127) with
 * n_bins equal-number distance bins (stable tie order), or
 * exact distances when n_bins == 0. balanced (n, R), dist (n) -> sf (n, R). */
int h3d_size_factors_cmor(h3d_ctx* ctx, const double* balanced,
                          const int32_t* dist, int64_t n, int R, int n_bins,
                          double* sf_out);

/* Size factors of any norm (scaling.py): the conditional methods condition
 * on distance (n_bins equal-number bins, or exact distances when n_bins ==
 * 0; scaling.py:68-105) and write sf (n, R); the global ones write one
 * factor per replicate, sf (R). balanced (n, R), dist (n; unused by the
 * global methods, may be NULL). */
int h3d_size_factors(h3d_ctx* ctx, const double* balanced, const int32_t* dist,
                     int64_t n, int R, int norm, int n_bins, double* sf_out);
/* The same on a DEVICE balanced (n, R) (h3d_union_fill_dev's), dist (n) on
 * the host; sf on the host as h3d_size_factors writes it and, when d_sf_out
 * is not NULL, in that device buffer too ((n, R) or (R,)); sf_out may be
 * NULL for the conditional norms when d_sf_out is given. */
int h3d_size_factors_dev(h3d_ctx* ctx, const double* d_balanced,
                         const int32_t* dist, int64_t n, int R, int norm,
                         int n_bins, double* sf_out, double* d_sf_out);

/* prepare_data's scaled and disp_idx on the device (analysis.py:109-115,
 * replaces the host `balanced / size_factors`, `np.dot(scaled, design) /
 * n_c` and `np.all(mean >= mean_thresh, axis=1) & (dist >= dist_thresh_min)`):
 * d_balanced (n, R) and d_sf ((n, R), or (R,) with sf_per_rep) on the device,
 * design (R, C) 0/1 row-major on the host. Writes scaled (n, R) and flag (n)
 * to the host and, when d_flag_out / d_scaled_out are not NULL, flag /
 * scaled to those device buffers (scaled_out may then be NULL).
 * flag = 1 / 0 is disp_idx; 2 marks a row whose decision could depend on the
 * product's summation order (a non-finite scaled value, or a mean within
 * 1e-12 relative of mean_thresh): the caller decides those rows with numpy's
 * product. Synchronous. */
int h3d_scale_disp_dev(h3d_ctx* ctx, const double* d_balanced, const double* d_sf,
                       int sf_per_rep, const int32_t* d_row, const int32_t* d_col, int64_t n,
                       int R, int C, const uint8_t* design, double mean_thresh,
                       int dist_thresh_min, double* scaled_out, uint8_t* flag_out,
                       uint8_t* d_flag_out, double* d_scaled_out);

/* The disp pixels of one chromosome on the device (analysis.py:169-183 for
 * estimate_disp, :261-275 for lrt): the union pixels whose d_disp_idx (n,
 * 0/1) is set, in pixel order -> d_raw_out (n_disp, R) int32, d_f_out
 * (n_disp, R) = bias[row] * bias[col] * sf (numpy's products in numpy's
 * order), d_dist_out (n_disp) = col - row. Inputs: d_row / d_col (n),
 * d_raw (n, R) int32, d_sf (n, R), or (R,) with sf_per_rep (the
 * non-conditional norms, broadcast as analysis.py:274-275 does), bias
 * (n_bins, R) on the HOST (core.py:35-60, filtered). n_disp = the caller's
 * count of set flags (H3D_EARG if the device counts another). Synchronous. */
int h3d_disp_pixels_dev(h3d_ctx* ctx, const int32_t* d_row, const int32_t* d_col,
                        const int32_t* d_raw, const double* d_sf, int sf_per_rep,
                        const double* bias, int n_bins, const uint8_t* d_disp_idx,
                        int64_t n, int R, int64_t n_disp, int32_t* d_raw_out,
                        double* d_f_out, int32_t* d_dist_out);

/* f of pixels received by the distance re-shard, rebuilt from their keys
 * (replaces shipping f; analysis.py:169-183 forms it on the rank that
 * prepared the chromosome): pixel j of genome chromosome d_chrom[j] at
 * (d_row[j], d_row[j] + d_dist[j]) with size-factor row d_sfi[j] gets
 * d_f_out[j, k] = (bias[row, k] * bias[col, k]) * sf[sfi, k] -- the product
 * and order of h3d_disp_pixels_dev, so bit for bit the sender's f. d_bias
 * (B, R): every chromosome's (filtered) bias rows stacked, chromosome g's
 * from d_boff[g] (nchrom + 1 offsets); d_sf (S, R) its size-factor rows from
 * d_soff[g]. A key outside its chromosome's rows is H3D_EINPUT (its f NaN).
 * Synchronous. */
int h3d_pixel_f_dev(h3d_ctx* ctx, const int32_t* d_row, const int32_t* d_dist,
                    const int32_t* d_chrom, const int32_t* d_sfi, int64_t n, int R,
                    const double* d_bias, const int64_t* d_boff, const double* d_sf,
                    const int64_t* d_soff, int nchrom, double* d_f_out);

/* ---- estimate_disp ----------------------------------------------------- */

/* Per-(distance, condition) dispersion (analysis.py:185-206). raw/f (n, R),
 * dist (n) in [0, D); cond_of_rep (R) in [0, C). Output disp_per_dist (D, C)
 * (NaN for empty slices), seg_flags (D, C) optional. */
int h3d_disp_per_dist(h3d_ctx* ctx, const int64_t* raw, const double* f,
                      const int32_t* dist, int64_t n, int R, int C,
                      const int32_t* cond_of_rep, int D, int estimator,
                      double* disp_per_dist, int32_t* seg_flags);

/* Same on device-resident inputs: d_raw (n, R) int32, d_f (n, R), d_dist (n).
 * `reduce` (optional) makes the per-segment sums global across ranks; every
 * rank must pass the same D, C, cond_of_rep. */
int h3d_disp_per_dist_dev(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                          const int32_t* d_dist, int64_t n, int R, int C,
                          const int32_t* cond_of_rep, int D, int estimator,
                          double* disp_per_dist, int32_t* seg_flags,
                          h3d_allreduce_fn reduce, void* user);

/* Work of the last h3d_disp_per_dist[_dev] / h3d_estimate_disp_dev call on
 * the ctx, per (distance, condition) segment s = d * C + c (S = D * C):
 * qcml iterations (equalize passes) and bounded-Brent NLL evaluations. The
 * multi-GPU distance owners balance on these (measurement). */
int h3d_disp_seg_stats(h3d_ctx* ctx, int S, int32_t* qiter, int32_t* evals);

/* Smoothed dispersion function of one condition, tabulated at d = 0..D-1
 * (lowess.py:95-244 weighted_lowess_fit if weighted, else lowess_fit;
 * left_boundary = first finite value, as analysis.py:212). frac < 0 = auto.
 * weighted: 0 lowess_fit; 1 weighted, the smallest scaled weight pinned to
 * exactly 1; 2 weighted with the reference's own
 * w * (1 / w) scaling (lowess.py:183-184), whose floor (:201) drops a
 * minimum weight that rounds to 1 - 2^-53. Every weighted entry point below
 * takes the same three values. */
int h3d_disp_table(const double* disp_per_dist_col, int D, int weighted,
                   double frac, double auto_frac_factor, double* table_out);

/* h3d_disp_table for every column of disp_per_dist (D, C), row-major in and
 * out, the conditions on concurrent host threads (analysis.py:208-219's
 * per-condition loop). */
int h3d_disp_tables(const double* disp_per_dist, int D, int C, int weighted,
                    double frac, double auto_frac_factor, double* tables_out);

/* The same tables computed on the GPU (one workgroup per condition, D <=
 * 1024; larger D runs the host smoother inside the call), device buffers
 * in and out, enqueued on the ctx stream without waiting: the estimate_disp
 * -> lrt step stays on the device (analysis.py:226-240 between :198-246 and
 * :249-276). Its status is settled by the next h3d_lrt_dev_tab (which
 * re-runs the LRT if a degenerate fit had to be redone on the host) or by
 * h3d_disp_tables_wait; both return the reference's error as
 * h3d_disp_tables would. The buffers must stay valid until then. */
int h3d_disp_tables_dev(h3d_ctx* ctx, const double* d_disp_per_dist, int D,
                        int C, int weighted, double frac,
                        double auto_frac_factor, double* d_tables_out);
int h3d_disp_tables_wait(h3d_ctx* ctx);

/* estimate_disp (qcml, h3d_disp_per_dist_dev without a reduce) whose
 * smoothed tables are computed on the device from the result in place
 * (analysis.py:198-246 then :226-240): disp_per_dist (D, C) on the host as
 * h3d_disp_per_dist_dev returns it, the tables into d_tables_out (device,
 * (D, C)), the smoother running while the call returns. Settled like
 * h3d_disp_tables_dev; it reads the ctx's result buffer, so the next
 * estimate_disp call on the ctx must come after h3d_lrt_dev_tab /
 * h3d_disp_tables_wait. */
int h3d_estimate_disp_dev(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                          const int32_t* d_dist, int64_t n, int R, int C,
                          const int32_t* cond_of_rep, int D, int weighted,
                          double frac, double auto_frac_factor,
                          double* disp_per_dist, int32_t* seg_flags,
                          double* d_tables_out);

/* disp[i, c] = tables[dist[i], c] on the device (analysis.py:218 disp_fn(dist)
 * at integer distances = the tabulation; NaN outside [0, D)): d_tables (D,
 * C), d_dist (n) -> d_disp_out (n, C). A pending h3d_disp_tables_dev /
 * h3d_estimate_disp_dev table is settled first (h3d_disp_tables_wait).
 * Synchronous. */
int h3d_table_gather_dev(h3d_ctx* ctx, const double* d_tables, int D, int C,
                         const int32_t* d_dist, int64_t n, double* d_disp_out);

/* ---- lrt --------------------------------------------------------------- */

/* Per-pixel LRT (lrt.py:7-50) with disp[i, c] = disp_table[dist[i], c]
 * (disp_table (D, C)); with dist == NULL, disp_table is the per-pixel
 * dispersion array (n, C) itself (the reference's disp_<chrom>.npy, as
 * analysis.py:269-278 loads it). Outputs p, llr, mu0 (n), mu1 (n, C);
 * disp_out (n, C) optional. */
int h3d_lrt(h3d_ctx* ctx, const int64_t* raw, const double* f,
            const int32_t* dist, const double* disp_table, int64_t n, int R,
            int C, const int32_t* cond_of_rep, int D, int refit_mu, double* p,
            double* llr, double* mu0, double* mu1, double* disp_out);

int h3d_lrt_dev(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                const int32_t* d_dist, const double* disp_table, int64_t n,
                int R, int C, const int32_t* cond_of_rep, int D, int refit_mu,
                double* d_p, double* d_llr, double* d_mu0, double* d_mu1,
                double* d_disp);

/* h3d_lrt_dev with the per-distance table (D, C) in DEVICE memory (from
 * h3d_disp_tables_dev; d_dist required). */
int h3d_lrt_dev_tab(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                    const int32_t* d_dist, const double* d_disp_table,
                    int64_t n, int R, int C, const int32_t* cond_of_rep, int D,
                    int refit_mu, double* d_p, double* d_llr, double* d_mu0,
                    double* d_mu1, double* d_disp);

/* lrt.py:7-50 with the reference's own disp argument: per pixel AND
 * replicate dispersions disp_wide (n, R) (lrt.py's `disp`, as analysis.py:277
 * builds it with np.dot(disp, design.T); any (n, R) values are taken as
 * given). Outputs as h3d_lrt. */
int h3d_lrt_wide(h3d_ctx* ctx, const int64_t* raw, const double* f,
                 const double* disp_wide, int64_t n, int R, int C,
                 const int32_t* cond_of_rep, int refit_mu, double* p,
                 double* llr, double* mu0, double* mu1);

/* dispersion.py:46-80 cml on given data (n, r), already divided by f: the
 * bounded-Brent minimisation of the NB conditional NLL on the GPU (one
 * k_brent search); *disp = delta / (1 - delta). H3D_ENOCONV where the
 * reference's assert res.success would fail. */
int h3d_cml(h3d_ctx* ctx, const double* data, int64_t n, int r, double* disp);

/* ---- bh ---------------------------------------------------------------- */

/* Benjamini-Hochberg q-values over the finite p-values (NaN elsewhere), on
 * the host CPU (no ctx). */
int h3d_bh(const double* p, int64_t n, double* q);

/* The same on the ctx's GPU: one radix sort of (p, index), the ratio
 * p_(j) / ((j + 1) / m), a reverse min-scan, a scatter -- bit-identical to
 * h3d_bh. _ctx: host buffers (synchronous); _dev: device buffers, stream-
 * ordered on the ctx stream (n < 2^31). */
int h3d_bh_ctx(h3d_ctx* ctx, const double* p, int64_t n, double* q);
int h3d_bh_dev(h3d_ctx* ctx, const double* d_p, int64_t n, double* d_q);

/* The same BH over p-values sharded across ranks (analysis.py:286-303 over
 * every chromosome, hic3defdr_amd.parallel.bh_sharded; the rank exchange is
 * the caller's). Device buffers on the ctx stream, each call returns once
 * the stream has drained (the caller moves the results between ranks next);
 * every q has h3d_bh_dev's bits.
 *   _sort: (p, val) pairs sorted by p ascending, non-finite p last (key
 *     +inf); val NULL = 0..n-1; *m_finite (host, synchronous) = finite count.
 *   _scan: for a bucket of mb sorted finite p-values at global ranks
 *     offset .. offset + mb - 1 of m: scanned[j] = min over j' >= j of
 *     p[j'] / ((offset + j' + 1) / m); *bucket_min (host, synchronous) =
 *     scanned[0] (+inf for an empty bucket).
 *   _finish: q[j] = min(scanned[j], higher_min) clipped at 1, higher_min =
 *     the minimum of the higher buckets' bucket_min (+inf for the last). */
int h3d_bh_sort_dev(h3d_ctx* ctx, const double* d_p, const int64_t* d_val, int64_t n,
                    double* d_key_out, int64_t* d_val_out, int64_t* m_finite);
int h3d_bh_scan_dev(h3d_ctx* ctx, const double* d_ps, int64_t mb, int64_t offset,
                    int64_t m, double* d_scanned, double* bucket_min);
int h3d_bh_finish_dev(h3d_ctx* ctx, const double* d_scanned, int64_t mb, double higher_min,
                      double* d_q);

/* ---- threshold / classify / collect (host) ------------------------------ */

/* Clusters of a pixel list (clusters.py:73-97 find_clusters with its
 * DirectedDisjointSet, :15-70): connectivity 1 = 4-neighbour cross, 2 = the
 * 8-neighbourhood (scipy generate_binary_structure(2, connectivity)).
 * label[i] = cluster of pixel i, numbered in the order of the reference's
 * get_groups() list; *n_clusters = number of clusters. Host code. */
int h3d_find_clusters(const int64_t* row, const int64_t* col, int64_t n,
                      int connectivity, int64_t* label, int64_t* n_clusters);

/* h3d_find_clusters plus the pixel order the reference writes: order (n) =
 * the pixel indices cluster by cluster (get_groups() order), each cluster in
 * the iteration order of the reference's Python set of (i, j) tuples --
 * CPython 3.8-3.10's set table replayed over the same adds and |= merges
 * (clusters.py:34-66), which is the order save_clusters (clusters.py:129-130)
 * and clusters_to_table (cluster_table.py:64-78, list(cluster)) write.
 * The pixels must be distinct. Host code. */
int h3d_find_clusters_ordered(const int64_t* row, const int64_t* col, int64_t n,
                              int connectivity, int64_t* label, int64_t* n_clusters,
                              int64_t* order);

/* "[[i, j], [i, j], ...]" text of each cluster (clusters.py:129-130 JSON,
 * cluster_table.py:67 TSV "cluster" column): cluster k is the pixels
 * order[starts[k] .. starts[k+1]). Concatenated into buf (cap bytes; NULL to
 * size), ends[k] = end offset of cluster k (optional), *len = total bytes. */
int h3d_format_clusters(const int64_t* row, const int64_t* col,
                        const int64_t* order, const int64_t* starts,
                        int64_t n_clusters, char* buf, int64_t cap,
                        int64_t* ends, int64_t* len);

/* ---- alternative models (analysis/alternatives.py) ---------------------- */

/* Poisson LRT (alternatives.py:25-42 with refit_mu=True, the only mode
 * Poisson3DeFDR uses and the only one the reference can run: its refit_mu=False
 * branch builds mu_hat_alt transposed and fails in np.dot). mu0 =
 * np.average(raw / f, weights=f) over all replicates, mu1[:, c] the same over
 * condition c's; llr = sum log poisson.pmf(raw | mu0 f) - sum log
 * poisson.pmf(raw | mu1[cond] f); p = chi2(C - 1).sf(-2 llr). raw/f (n, R) ->
 * p, llr, mu0 (n), mu1 (n, C). */
int h3d_lrt_poisson(h3d_ctx* ctx, const int64_t* raw, const double* f,
                    int64_t n, int R, int C, const int32_t* cond_of_rep,
                    double* p, double* llr, double* mu0, double* mu1);
int h3d_lrt_poisson_dev(h3d_ctx* ctx, const int32_t* d_raw, const double* d_f,
                        int64_t n, int R, int C, const int32_t* cond_of_rep,
                        double* d_p, double* d_llr, double* d_mu0,
                        double* d_mu1);

/* Per-pixel method-of-moments dispersion of every condition's replicates
 * (dispersion.py:83-104 mme_per_pixel(data[:, design[:, c]], f)): data (n, R)
 * (divided by f (n, R) when f != NULL) -> disp (n, C) = max((var - mean) /
 * mean^2, min_disp), var with ddof 1; NaN stays NaN (numpy maximum).
 * min_disp = -inf for no floor; Unsmoothed3DeFDR uses 1e-7. */
int h3d_mme_per_pixel(h3d_ctx* ctx, const double* data, const double* f,
                      int64_t n, int R, int C, const int32_t* cond_of_rep,
                      double min_disp, double* disp);

/* ---- measurement -------------------------------------------------------- */

/* Per-kernel HIP-event timing on the ctx stream; on = 0 off, 1 the roofline
 * kernels only ("disp_work", "lrt"), 2 every scope. Events are read back
 * lazily (profile_read / profile_reset). name in {"disp_work" (the
 * equalize pass), "disp_nll", "disp_reduce", "disp_update", "disp_prep",
 * "lrt"}. units: algorithmic HBM bytes for "disp_work" / "disp_nll"
 * (counted on the device since the last reset), pixels for "lrt" /
 * "disp_prep". name "gang_aborts": *launches = gang Brent waits of the ctx
 * that timed out (the searches then finished under k_brent). */
int h3d_profile_enable(h3d_ctx* ctx, int on);
int h3d_profile_read(h3d_ctx* ctx, const char* name, double* total_ms,
                     int64_t* launches, int64_t* units);
int h3d_profile_reset(h3d_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* H3D_H_ */
