"""Benchmark: pixels/sec through estimate_disp + lrt (BASELINE.json metric).

Workloads (BASELINE.json configs):
- cfg2 (configs[1], the N = 1 default): one synthetic chromosome of 20,000
  bins, 4 replicates (2 + 2 conditions), dist_thresh_max 250 (SURVEY.md §8(d)
  generator, seed = rank). Untimed setup: generate the input files, run the
  product's GPU prepare_data, upload raw / f / dist of the disp pixels to
  HBM. One step = estimate_disp (qcml per distance x condition) + the lowess
  smoothing tables (on the GPU from estimate_disp's result in place,
  h3d_estimate_disp_dev; H3D_DEV_TABLE=1 / 0 for the separate device / the
  host smoother) + lrt (fused per-pixel GLM fits + LRT) on the resident
  inputs, outputs left in HBM.
- cfg3 (configs[2], the N > 1 default; --config cfg3 at any N): the whole
  mouse genome at 10 kb -- 20 mm10-sized chromosomes, 4 replicates, dmax 200,
  ~46 M disp pixels -- STRONG scaling: the chromosomes are LPT-sharded over
  the ranks, each rank draws only its own (synthetic.draw_band, no files)
  and holds them in HBM. One step = estimate_disp over the whole genome (the
  distance re-shard: distances LPT-assigned by pixel count, one all_to_all
  of the disp pixels, the single-GPU driver per rank, one all-reduce of the
  D x C table) + lowess tables + lrt of the rank's own pixels + the
  genome-wide BH (parallel.bh_sharded: a sample sort of the p-values over
  the ranks, each rank ranking one value range on its GPU).

The CPU baseline (rank 0, N = 1, cfg2) runs FIRST, before anything touches
the GPU (its worker pool forks): the CPU restatement (oracle/, numpy/scipy)
with the reference's parallel structure on every allowed core (the affinity
mask bounded by the cgroup CPU quota -- the GPU box's share per GPU; both
reported), calibrated against the reference itself on the same input and
cores in the build container (profiles/r05/cpu_calibration.json, reported
beside the rows): the fallback-fixed row
(brentq only on the failed pixel) on the FULL cfg2 chromosome, and the
faithful row (the reference's O(fail * N) brentq fallback,
scaled_nb.py:162-181, LRT on one process per chromosome as
analysis.py:247-257) on a 1,000-bin sample -- its O(fail * N) cost grows
super-linearly with the chromosome, so the survey's own measurement of the
reference at cfg2 is quoted beside it.

The north star's headline shape, cfg3 (the whole mouse genome), is measured
beside the cfg2 line at N = 1 (other_configs.cfg3): the genome is drawn once
before the GPU is touched, the fallback-fixed restatement runs estimate_disp +
lrt over all of it ONCE on every allowed core (other_configs.cfg3.
cpu_baseline, with gpu_over_cpu), and after the GPU's timed steps on the same
genome every pixel's p, the genome-wide BH calls at FDR 0.01 / 0.05 / 0.1 and
the segments beyond 1e-6 are compared (vs_cpu_restatement, identical_calls).
e2e_cfg3_run_to_qvalues: the same shape END TO END from files through the
class (the genome written in the reference's layout before the GPU starts).

Roofline denominators: the spec peaks and this GPU's measured ones
(measured_peaks: FP64 FMA chains and a 16 B/lane copy, libh3d_peak.so, run
before the headline); the dominant kernel's launch time from the live HIP
events and from the committed rocprofv3 stats of the same command.

Prints ONE JSON line on rank 0.
"""
import argparse
import hashlib
import json
import os
import shutil
import statistics
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

METRIC = ("pixels/sec through estimate_disp+lrt, 4 reps @10kb; "
          "max-|Δq| vs reference")

PMC_SUMMARY = os.path.join(REPO, 'profiles', 'pmc_default.json')
# rocprofv3 --kernel-trace --stats of the same default command (the kernel
# durations the committed PMC summary is read against)
KSTATS = os.path.join(REPO, 'profiles', 'kernel_stats_default.json')
# spec peaks: FP64 vector 78.6 TFLOP/s is AMD's MI355X product figure (dense,
# no sparsity; MI355X_MICROARCH.md gives no FP64 number); HBM3E 8.0 TB/s spec
# (MI355X_MICROARCH.md: 6.29 TB/s measured with a float4 copy). The bench
# measures both on the box before the headline (measured_peaks,
# libh3d_peak.so) and reports every fraction against both.
FP64_PEAK_TFLOPS = 78.6
HBM_PEAK_GBS = 8000.0
CPU_RUNS = 4


# ---------------------------------------------------------------------------
# committed PMC summary (tools/pmc_passes.sh over the default command)
# ---------------------------------------------------------------------------

def pmc_combined(kernels, per, bins, dmax):
    """Counters of several kernels that share one unit of work (a qcml
    iteration's Brent searches: k_brent and k_brent_gang are both launched
    every iteration and one returns at once) summed over all their
    dispatches and divided by the dispatches of `per`."""
    parts = [(k, pmc_kernel(k, bins, dmax)) for k in kernels]
    base = pmc_kernel(per, bins, dmax)
    if not base:
        return None
    tot = {'hbm_bytes': 0.0, 'f64_flops': 0.0, 'thread': 0.0, 'active': 0.0}
    for _, q in parts:
        if not q:
            continue
        for k in ('hbm_bytes', 'f64_flops'):
            tot[k] += q[k] * q['dispatches']
        if q['lane_util'] is not None:
            tot['thread'] += q['lane_util'] * q['active_insts']
            tot['active'] += q['active_insts']
    n = base['dispatches']
    return {'hbm_bytes': tot['hbm_bytes'] / n, 'f64_flops': tot['f64_flops'] / n,
            'lane_util': tot['thread'] / tot['active'] if tot['active'] else None,
            'dispatches': n}


def pmc_kernel(kernel, bins, dmax):
    """Per-launch counters of `kernel` (name prefix) from the committed PMC
    summary of this same default command: HBM bytes (FETCH_SIZE x2 gfx950
    correction + WRITE_SIZE), FP64 flops issued ((ADD + MUL + TRANS + 2 FMA)
    x 64 lanes), lane utilisation. Counters cannot be read inside the timed
    run; None unless the workload is the one they were measured on."""
    try:
        d = json.load(open(PMC_SUMMARY))
    except (OSError, ValueError):
        return None
    if d.get('bins') != bins or d.get('dmax') != dmax:
        return None
    acc, n = {}, 0
    for key, e in d['kernels'].items():
        if not key.split('[')[0].split('(')[0].strip().endswith(kernel):
            continue
        n += e['dispatches']
        for c in ('hbm_read_bytes_corrected', 'hbm_write_bytes',
                  'SQ_INSTS_VALU_ADD_F64', 'SQ_INSTS_VALU_MUL_F64',
                  'SQ_INSTS_VALU_FMA_F64', 'SQ_INSTS_VALU_TRANS_F64',
                  'SQ_THREAD_CYCLES_VALU', 'SQ_ACTIVE_INST_VALU'):
            acc[c] = acc.get(c, 0.0) + e.get(c, 0.0)
    if not n:
        return None
    flops = 64.0 * (acc['SQ_INSTS_VALU_ADD_F64'] + acc['SQ_INSTS_VALU_MUL_F64']
                    + acc['SQ_INSTS_VALU_TRANS_F64']
                    + 2.0 * acc['SQ_INSTS_VALU_FMA_F64'])
    lu = acc['SQ_THREAD_CYCLES_VALU'] / (64.0 * acc['SQ_ACTIVE_INST_VALU']) \
        if acc['SQ_ACTIVE_INST_VALU'] else None
    return {'hbm_bytes': (acc['hbm_read_bytes_corrected'] +
                          acc['hbm_write_bytes']) / n,
            'f64_flops': flops / n, 'lane_util': lu, 'dispatches': n,
            'active_insts': acc['SQ_ACTIVE_INST_VALU']}


def measured_peaks(device):
    """The box's own roofline denominators (csrc/h3d_peak.hip): independent
    v_fma_f64 chains at 8 waves per SIMD on every CU, and a 16 B/lane
    streaming copy of 2 GiB (read + write bytes), each the best of 10 timed
    launches after a warm-up. None when libh3d_peak.so is absent."""
    import ctypes
    from hic3defdr_amd import build as h3dbuild
    path = os.path.join(h3dbuild.LIBDIR, 'libh3d_peak.so')
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    buf = (ctypes.c_double * 4)()
    st = lib.h3d_peak_fp64(device, 10, buf)
    fp64 = {'best_tflops': buf[0], 'median_tflops': buf[1],
            'flops_per_launch': buf[2], 'best_ms': buf[3],
            'kernel': 'k_fma_chains: 8 independent v_fma_f64 chains x 16 '
                      'unrolled x 2048 trips per lane, 8 waves per SIMD, '
                      'every CU'} if st == 0 else {'error': st}
    st = lib.h3d_peak_copy(device, ctypes.c_int64(1 << 30), 10, buf)
    hbm = {'best_gbs': buf[0], 'median_gbs': buf[1],
           'bytes_per_launch': buf[2], 'best_ms': buf[3],
           'kernel': 'k_copy16: double2 load + store per lane, grid-stride, '
                     '1 GiB -> 1 GiB, 16 waves per CU; read + write bytes'} \
        if st == 0 else {'error': st}
    return {'fp64': fp64, 'hbm': hbm, 'source': 'bench.py measured_peaks '
            '(hic3defdr_amd/csrc/h3d_peak.hip), run on this GPU before the '
            'headline'}


def _peak(peaks, kind):
    try:
        return peaks[kind]['best_tflops' if kind == 'fp64' else 'best_gbs']
    except (TypeError, KeyError):
        return None


def rocprof_avg_us(kernel, bins, dmax):
    """Average launch duration of `kernel` (name prefix) in the committed
    rocprofv3 --kernel-trace --stats summary of the default command, or None
    unless the workload is the one it was measured on."""
    import csv
    try:
        meta = json.load(open(KSTATS))
    except (OSError, ValueError):
        return None
    if meta.get('bins') != bins or meta.get('dmax') != dmax:
        return None
    calls = tot = 0
    with open(os.path.join(REPO, meta['csv'])) as fh:
        for row in csv.DictReader(fh):
            # 'void h3d::k_disp_work<2, 4, 0, false>(int const*, ...)'
            name = row['Name'].split('(')[0].strip()
            if name.endswith(kernel):
                calls += int(row['Calls'])
                tot += float(row['TotalDurationNs'])
    if not calls:
        return None
    return {'avg_us': tot / calls / 1e3, 'calls': calls,
            'source': meta['csv'], 'command': meta.get('command')}


def bytes_per_lrt_pixel(R, C):
    # raw int32 4R + f 8R + dist 4 in; p, llr, mu0 24 + mu1 8C + disp 8C out
    return 12 * R + 16 * C + 28


def fp64_roof(pmc, avg_s, peak_measured=None):
    if not pmc or not avg_s:
        return None
    ach = pmc['f64_flops'] / avg_s / 1e12
    out = {'achieved': ach, 'peak': FP64_PEAK_TFLOPS, 'unit': 'TFLOP/s',
           'frac': ach / FP64_PEAK_TFLOPS,
           'flops_per_launch': pmc['f64_flops'],
           'lane_util': pmc['lane_util']}
    if peak_measured:
        out['peak_measured'] = peak_measured
        out['frac_measured'] = ach / peak_measured
    if pmc['lane_util'] is not None:
        out['useful_frac'] = out['frac'] * pmc['lane_util']
    return out


# ---------------------------------------------------------------------------
# CPU baseline (runs before the GPU is touched)
# ---------------------------------------------------------------------------

def _qcml_task(args):
    import oracle
    data, f, faithful = args
    return oracle.qcml(data, f=f, faithful=faithful) if data.size else np.nan


def _lrt_task(args):
    import oracle
    raw, f, dw, design, faithful = args
    return oracle.lrt(raw, f, dw, design, faithful=faithful)[0]


def cpu_pipeline(pool, workers, raw, f, dist, design, D, faithful,
                 with_table=False, progress=False):
    """estimate_disp + lrt on the CPU with the reference's parallel structure:
    qcml per (distance, condition) over the pool (analysis.py:193-200), the
    lowess fit per condition, then the LRT -- faithful: one call over the
    chromosome (one process per chromosome, analysis.py:247-257);
    fallback-fixed: pixel blocks over the pool. Returns p (and the (D, C)
    disp_per_dist with ``with_table``)."""
    import oracle
    C = design.shape[1]
    order = np.argsort(dist, kind='stable')
    bounds = np.searchsorted(dist[order], np.arange(D + 1))
    def tasks():
        for c in range(C):
            cols = design[:, c]
            for d in range(D):
                sel = order[bounds[d]:bounds[d + 1]]
                yield raw[sel][:, cols], f[sel][:, cols], faithful
    # largest segments first would shorten the pool's tail, but the results
    # must come back in (condition, distance) order: imap keeps it
    def beat(it, what):
        # a progress line on stderr every ~30 s (long legs: the cfg3 genome)
        t = time.perf_counter()
        for k, v in enumerate(it):
            if progress and time.perf_counter() - t > 30:
                t = time.perf_counter()
                print('bench: cpu %s %d ...' % (what, k), file=sys.stderr,
                      flush=True)
            yield v
    dpd = np.array(list(beat(pool.imap(_qcml_task, tasks(), chunksize=2),
                             'segments'))).reshape(C, D).T
    disp = np.zeros((len(raw), C))
    for c in range(C):
        fin = np.isfinite(dpd[:, c])
        x, y = np.arange(D)[fin], dpd[fin, c]
        disp[:, c] = oracle.weighted_lowess_fit(x, y, left_boundary=y[0])(dist)
    dw = np.dot(disp, design.T)
    del disp
    if faithful:
        p = _lrt_task((raw, f, dw, design, True))
    else:
        blocks = np.array_split(np.arange(len(raw)), workers * 4)
        p = np.concatenate(list(beat(pool.imap(
            _lrt_task, ((raw[b], f[b], dw[b], design, False) for b in blocks)),
            'lrt blocks')))
    return (p, dpd) if with_table else p


# SURVEY.md §6 [probe]: the reference itself on cfg2 (20k bins, dmax 250;
# 3,774,156 disp pixels), n_threads=-1 on 8 cores: estimate_disp 35.69 s +
# lrt 3,167.8 s (3,281 brentq fallbacks, O(fail * N) each)
SURVEY_REF_CFG2 = {'value': 1178.0, 'unit': 'pixels/s', 'cores': 8,
                   'kind': 'reference',
                   'source': 'SURVEY.md section 6: the reference on cfg2 in '
                             'the survey container (Xeon, 8 cores)'}


def _cpu_inputs(bins, dmax, seed):
    import oracle
    from hic3defdr_amd import synthetic
    tmp = tempfile.mkdtemp(prefix='h3dbench_cpu_')
    try:
        kw = synthetic.write_dataset(tmp, {'chrS': bins}, dist_thresh_max=dmax,
                                     seed=seed)
        design = kw['design']
        npz = [p.replace('<chrom>', 'chrS') for p in kw['raw_npz_patterns']]
        bfs = [p.replace('<chrom>', 'chrS') for p in kw['bias_patterns']]
        prep = oracle.prepare_chrom(npz, bfs, design, dist_thresh_max=dmax)
        bias = oracle.load_bias(bfs)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    di = prep['disp_idx']
    row, col = prep['row'][di], prep['col'][di]
    return {'raw': prep['raw'][di],
            'f': bias[row] * bias[col] * prep['size_factors'][di],
            'dist': col - row, 'design': design}


def _cpu_rows(pool, workers, inp, dmax, faithful, runs):
    import oracle
    times, p = [], None
    for _ in range(runs):
        oracle.STATS['brentq_fallbacks'] = 0
        t0 = time.perf_counter()
        p = cpu_pipeline(pool, workers, inp['raw'], inp['f'], inp['dist'],
                         inp['design'], dmax + 1, faithful)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {'value': len(inp['raw']) / med, 'median_s': med,
            'runs_s': times}, p


def allowed_cpus():
    """(CPUs in this process' affinity mask, CPUs of its cgroup CPU quota or
    None): the host cores the CPU baseline may use. The GPU box shows the
    whole machine in os.cpu_count() and the affinity mask; its share per GPU
    is the cgroup quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open('/sys/fs/cgroup/cpu.max') as fh:      # cgroup v2
            q, per = fh.read().split()[:2]
            if q != 'max':
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:                                            # cgroup v1
            with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as fh:
                q = int(fh.read())
            with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as fh:
                per = int(fh.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    return aff, quota


def cpu_calibration():
    """The committed calibration of the restatement against the reference on
    the same input and cores (tools/cpu_calibration.py, build container)."""
    path = os.path.join(REPO, 'profiles', 'r05', 'cpu_calibration.json')
    try:
        with open(path) as fh:
            c = json.load(fh)
    except (OSError, ValueError):
        return None
    return {'source': 'profiles/r05/cpu_calibration.json '
                      '(tools/cpu_calibration.py)',
            'input': c['input'], 'cores': c['cores'],
            'reference_pixels_per_s': c['reference']['pixels_per_s'],
            'faithful_over_reference': c['ratio_faithful_over_reference'],
            'fallback_fixed_over_reference':
                c['ratio_fallback_fixed_over_reference'],
            'p_max_rel_vs_reference': c['p_max_rel_faithful_vs_reference']}


def cpu_baseline_run(full_bins, sample_bins, dmax, seed=123, full_runs=1):
    """fallback-fixed row on the full chromosome (`full_bins`; the headline
    workload's shape), faithful row on the `sample_bins` sample."""
    import multiprocessing
    import oracle
    ncpu = os.cpu_count() or 1
    workers, aff, quota = cpu_workers()
    full = _cpu_inputs(full_bins, dmax, seed) if full_bins else None
    sample = _cpu_inputs(sample_bins, dmax, seed)
    ctx = multiprocessing.get_context('fork')
    with ctx.Pool(workers) as pool:
        if full is not None:
            fixed, _ = _cpu_rows(pool, workers, full, dmax, False, full_runs)
        s_fixed, p_fixed = _cpu_rows(pool, workers, sample, dmax, False,
                                     CPU_RUNS)
        s_faith, p_faith = _cpu_rows(pool, workers, sample, dmax, True,
                                     CPU_RUNS)
    # the faithful row's cost is its secant failures x the chromosome's
    # pixels: the brentq fallbacks of its (in-process) LRT, last run
    n_fail = int(oracle.STATS['brentq_fallbacks'])
    if full is None:
        fixed = s_fixed
    n_full = len(full['raw']) if full is not None else len(sample['raw'])
    base = {'value': fixed['value'], 'unit': 'pixels/s', 'cores': workers,
            'cpu_count': ncpu, 'affinity_cpus': aff, 'cgroup_quota_cpus': quota,
            'kind': 'port',
            'variant': 'fallback-fixed (brentq on the failed pixel only; '
                       'LRT over pixel blocks on the pool)',
            'median_s': fixed['median_s'], 'runs_s': fixed['runs_s'],
            'sample': '1 synthetic chrom of %d bins (seed %d), dmax %d, 4 '
                      'reps 2+2: %d disp pixels -- the headline workload '
                      'shape; median of %d run(s)' % (
                          full_bins or sample_bins, seed, dmax, n_full,
                          full_runs),
            'fallback_fixed_on_sample': dict(s_fixed, pixels=len(
                sample['raw'])),
            'faithful': {
                'value': s_faith['value'], 'unit': 'pixels/s',
                'cores': workers,
                'variant': 'faithful O(fail*N) brentq (scaled_nb.py:162-181);'
                           ' qcml on the pool, LRT one process per chromosome',
                'sample': '%d-bin chromosome (seed %d): %d disp pixels, %d '
                          'LRT brentq fallbacks; median of %d runs'
                          % (sample_bins, seed, len(sample['raw']), n_fail,
                             CPU_RUNS),
                'median_s': s_faith['median_s'], 'runs_s': s_faith['runs_s'],
                'note': 'per-pixel cost grows with failures x chromosome '
                        'pixels; at cfg2 size see reference_at_cfg2'},
            'reference_at_cfg2': SURVEY_REF_CFG2,
            'calibration_vs_reference': cpu_calibration()}
    return base, {'raw': sample['raw'], 'f': sample['f'],
                  'dist': sample['dist'], 'design': sample['design'],
                  'p_fixed': p_fixed, 'p_faithful': p_faith}


def cpu_workers():
    """Every allowed core: the affinity mask bounded by the cgroup quota (the
    GPU box's share per GPU; 16 if a whole machine is visible and no quota
    says otherwise). Returns (workers, affinity, quota)."""
    aff, quota = allowed_cpus()
    workers = aff if quota is None else min(aff, max(1, int(quota)))
    if quota is None and aff > 64:
        workers = 16
    return workers, aff, quota


def cfg3_genome(dmax):
    """The cfg3 genome (BASELINE configs[2]) as other_config('cfg3') draws
    it: 20 mm10-sized chromosomes, seed 0, concatenated."""
    from hic3defdr_amd import synthetic
    t0 = time.perf_counter()
    parts = synthetic.draw_genome(list(synthetic.MM10_BINS), (2, 2), dmax,
                                  seed=0, workers=16)
    g = {'raw': np.concatenate([p[0] for p in parts]),
         'f': np.concatenate([p[1] for p in parts]),
         'dist': np.concatenate([p[2] for p in parts])}
    del parts
    g['generate_s'] = time.perf_counter() - t0
    return g


def cpu_cfg3_run(genome, dmax):
    """The north star's headline CPU leg: the fallback-fixed restatement's
    estimate_disp + lrt ONCE over the whole cfg3 genome (every distance pooled
    genome-wide, as analysis.py:169-206) on every allowed core. Returns (the
    row, p, disp_per_dist)."""
    import multiprocessing
    workers, aff, quota = cpu_workers()
    design = np.zeros((4, 2), dtype=bool)
    design[[0, 1], 0] = design[[2, 3], 1] = True
    ctx = multiprocessing.get_context('fork')
    with ctx.Pool(workers) as pool:
        t0 = time.perf_counter()
        p, dpd = cpu_pipeline(pool, workers, genome['raw'], genome['f'],
                              genome['dist'], design, dmax + 1, False,
                              with_table=True, progress=True)
        el = time.perf_counter() - t0
    n = len(genome['raw'])
    row = {'value': n / el, 'unit': 'pixels/s', 'cores': workers,
           'affinity_cpus': aff, 'cgroup_quota_cpus': quota, 'kind': 'port',
           'variant': 'fallback-fixed restatement (oracle/), qcml per '
                      '(distance, condition) on the pool, LRT over pixel '
                      'blocks on the pool',
           'elapsed_s': el,
           'sample': 'the WHOLE cfg3 genome, one run: 20 mm10-sized '
                     'chromosomes, %d disp pixels, dmax %d' % (n, dmax),
           'calibration_vs_reference': cpu_calibration()}
    return row, p, dpd


def cfg3_vs_cpu(ctx, p, dpd, cpu_p, cpu_dpd, dmax):
    """The GPU's cfg3 result against the CPU restatement's on the same
    genome: p per pixel, the genome-wide BH calls at three FDRs, and the
    segments whose disp_per_dist differs beyond 1e-6 (with the move in delta
    = disp / (1 + disp) in units of Brent's xatol 1e-5, dispersion.py:46-80:
    near-tied NLL comparisons)."""
    import oracle
    with np.errstate(all='ignore'):
        rel = np.abs(p - cpu_p) / np.maximum(cpu_p, 1e-300)
    rel[p == cpu_p] = 0.0
    q = ctx.bh(p)
    cq = oracle.adjust_pvalues(cpu_p)
    calls = {}
    for fdr in (0.01, 0.05, 0.1):
        a, b = q < fdr, cq < fdr
        calls['%g' % fdr] = {'gpu': int(a.sum()), 'cpu': int(b.sum()),
                             'differ': int(np.sum(a != b))}
    fin = np.isfinite(cpu_dpd)
    drel = np.zeros_like(cpu_dpd)
    drel[fin] = np.abs(dpd[fin] - cpu_dpd[fin]) / np.abs(cpu_dpd[fin])
    segs = segments_vs(dpd, cpu_dpd)
    return {'pixels': int(len(p)),
            'max_rel_dp': float(rel.max()),
            'pixels_rel_dp_gt_1e-6': int(np.sum(rel > 1e-6)),
            'max_abs_dq': float(np.max(np.abs(q - cq))),
            'calls': calls,
            'identical_calls': all(v['differ'] == 0 for v in calls.values()),
            'disp_per_dist_max_rel': float(drel.max()),
            'segments_beyond_1e-6': segs,
            'note': 'GPU (product kernels, device BH) vs the CPU restatement '
                    '(oracle/, BH = lib5c adjust_pvalues restated) on the same '
                    'genome; q-value calls at FDR 0.01 / 0.05 / 0.1'}


def sample_parity(ctx, sample, dmax):
    """The GPU on the CPU baseline's sample: p / q agreement and calls."""
    import oracle
    from hic3defdr_amd import _native
    design = sample['design']
    cond = design.argmax(axis=1)
    C = design.shape[1]
    out = ctx.disp_per_dist(sample['raw'], sample['f'], sample['dist'], cond,
                            C, dmax + 1)
    tab = _native.disp_tables(out)
    p, _, _, _, _ = ctx.lrt(sample['raw'], sample['f'], sample['dist'], tab,
                            cond)
    qg = _native.bh(p)
    res = {'sample_pixels': int(len(p))}
    for name, rp in (('fixed', sample['p_fixed']),
                     ('faithful', sample['p_faithful'])):
        qo = oracle.adjust_pvalues(rp)
        with np.errstate(all='ignore'):
            res['max_rel_dp_vs_cpu_%s' % name] = float(
                np.nanmax(np.abs(p - rp) / np.maximum(rp, 1e-300)))
            res['max_abs_dq_vs_cpu_%s' % name] = float(np.nanmax(np.abs(qg - qo)))
        res['identical_calls_q<0.05_%s' % name] = bool(
            np.array_equal(qg < 0.05, qo < 0.05))
    return res


GOLDEN = os.path.join(REPO, 'tests', 'golden')


def segments_vs(dpd, ref, bar=1e-6, xatol=1e-5):
    """The (distance, condition) segments of ``dpd`` beyond ``bar`` relative
    of ``ref``, each with its move in delta = disp / (1 + disp) -- the
    variable of cml's bounded Brent search (dispersion.py:72-80) -- in units
    of its xatol: a near-tied NLL comparison sends a search to another
    point within ~1 xatol."""
    fin = np.isfinite(ref) & np.isfinite(dpd)
    rel = np.zeros_like(ref)
    rel[fin] = np.abs(dpd[fin] - ref[fin]) / np.abs(ref[fin])
    return [{'distance': int(d), 'condition': int(c), 'rel': float(rel[d, c]),
             'd_delta_over_xatol': float(abs(
                 dpd[d, c] / (1 + dpd[d, c]) - ref[d, c] / (1 + ref[d, c]))
                 / xatol)}
            for d, c in zip(*np.nonzero(rel > bar))]


def parity_vs_reference(ctx, o, n, bins, dmax, seed, dpd=None):
    """The metric's second half, max-|dq| vs reference: the timed step's own
    p-values (left in HBM by the last timed step), BH on the device, against
    the REFERENCE's end-to-end run on this same chromosome
    (tests/golden/full_cfg2.npz: the reference's prepare_data +
    estimate_disp + lrt + bh, 50 k seeded sample pixels and the 2,000
    smallest p-values) and against the reference's own results under six
    pixel orders of its input (cfg2_spread.npz: the reference is only
    defined up to that spread). None unless the workload is that chromosome."""
    try:
        g = np.load(os.path.join(GOLDEN, 'full_cfg2.npz'))
        sp = np.load(os.path.join(GOLDEN, 'cfg2_spread.npz'))
    except OSError:
        return None
    if (int(g['meta_bins']), int(g['meta_dmax']), int(g['meta_seed'])) != \
            (bins, dmax, seed) or int(g['n_disp_pixels']) != n:
        return None
    ctx.bh_dev(o['p'].data_ptr(), n, o['q'].data_ptr())
    p, q = o['p'].cpu().numpy(), o['q'].cpu().numpy()
    s, t = g['sample_idx'], g['top_idx']

    def rel(a, b):
        return float(np.max(np.abs(a - b) / np.abs(b)))

    def dq(a, b):
        return float(np.max(np.abs(a - b)))
    out = {'reference': 'tests/golden/full_cfg2.npz (make_golden.py '
                        'run_full_cfg2: the reference run on this chromosome)',
           'pixels_compared': int(len(s) + len(t)),
           'max_abs_dq_vs_reference': max(dq(q[s], g['q']),
                                          dq(q[t], g['top_q'])),
           'max_rel_dq_vs_reference': max(rel(q[s], g['q']),
                                          rel(q[t], g['top_q'])),
           'max_rel_dp_vs_reference': max(rel(p[s], g['p']),
                                          rel(p[t], g['top_p'])),
           'identical_calls': all(
               np.array_equal(np.where(q < fdr)[0], g['calls_%g' % fdr])
               for fdr in (0.01, 0.05, 0.1))}
    near = []
    for k in sp['perms']:
        near.append((max(rel(p[s], sp['p_sample__%d' % k]),
                         rel(p[t], sp['p_top__%d' % k])),
                     max(dq(q[s], sp['q_sample__%d' % k]),
                         dq(q[t], sp['q_top__%d' % k])), int(k)))
    best = min(near)
    out['nearest_reference_order'] = {
        'order': best[2], 'max_rel_dp': best[0], 'max_abs_dq': best[1],
        'note': 'the reference re-run with the pixels of every segment in '
                'another order (cfg2_spread.npz, 6 orders incl. its own)'}
    if dpd is not None:
        # which segments carry a move beyond 1e-6 of the reference's own run
        # (a move of the bench's p from 3e-7 to 6e-6 names its segment here)
        out['segments_beyond_1e-6_vs_reference'] = segments_vs(
            dpd, g['disp_per_dist'])
    out['reference_own_spread'] = {
        'max_rel_dp': max(rel(sp['p_sample__%d' % k], g['p'])
                          for k in sp['perms']),
        'max_abs_dq': max(dq(sp['q_sample__%d' % k], g['q'])
                          for k in sp['perms']),
        'note': 'how far the reference moves itself under those orders '
                '(sample pixels)'}
    return out


# ---------------------------------------------------------------------------

def make_workload(tmp, name, bins, dmax, seed):
    import pandas as pd
    from hic3defdr_amd import HiC3DeFDR, synthetic
    kw = synthetic.write_dataset(tmp, {name: bins}, dist_thresh_max=dmax,
                                 seed=seed)
    design = pd.DataFrame(kw['design'], index=kw['reps'], columns=kw['conds'])
    h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                  bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                  design=design, outdir=os.path.join(tmp, 'out'),
                  dist_thresh_max=dmax)
    return h, kw


def e2e_cfg3_files(dmax):
    """The cfg3 genome written in the reference's input layout (per-replicate
    NPZ + bias files, loop clusters; synthetic.write_genome, a process pool)
    -- before the GPU is touched. Returns (directory, constructor kwargs,
    seconds)."""
    from hic3defdr_amd import synthetic
    base = tempfile.mkdtemp(prefix='h3dbench_cfg3e2e_')
    t0 = time.perf_counter()
    kw = synthetic.write_genome(base, synthetic.MM10_BINS, seed=3, workers=16,
                                dmax=dmax)
    return base, kw, time.perf_counter() - t0


def e2e_cfg3(base, kw, write_s, runs=2):
    """BASELINE configs[2] end to end through the class on one GPU: the 20
    chromosomes from their files through HiC3DeFDR.run_to_qvalues()'s stages
    (analysis.py:305-364: prepare_data per chromosome, the genome-wide
    estimate_disp, lrt, the loop-pixel BH), per stage, after one run paying
    the first-call costs (reported apart)."""
    import pandas as pd
    from hic3defdr_amd import HiC3DeFDR

    class _H:                     # the constructor arguments, no outdir yet
        pass
    h = _H()
    h.raw_npz_patterns, h.bias_patterns = kw['raw_npz_patterns'], \
        kw['bias_patterns']
    h.chroms = kw['chroms']
    h.design = pd.DataFrame(kw['design'], index=kw['reps'],
                            columns=kw['conds'])
    h.dist_thresh_max, h.loop_patterns, h.res = 200, kw['loop_patterns'], \
        10000
    first = _e2e_once(h, base, 'first', drop=True)
    per = [_e2e_once(h, base, k, drop=True) for k in range(runs)]
    out = {k: statistics.median(r[k] for r in per) for k in per[0]
           if k not in ('note', 'gc_collections', 'estimate_disp_stamps_ms')
           and per[0][k] is not None}
    out['gc_collections'] = [r['gc_collections'] for r in per]
    if 'estimate_disp_stamps_ms' in per[0]:
        out['estimate_disp_stamps_ms'] = [r['estimate_disp_stamps_ms']
                                          for r in per]
    out['runs_total_s'] = [r['total_s'] for r in per]
    out['first_run'] = {k: v for k, v in first.items() if k != 'note'}
    out['write_genome_s'] = write_s
    out['chromosomes'] = len(kw['chroms'])
    out['note'] = ('cfg3 from files: 20 mm10-sized chromosomes (seed 3), 4 '
                   'reps, dmax 200, loop clusters; ' + per[0]['note'] +
                   '; per-stage medians of %d runs after the first' % runs)
    return out


def e2e_wall(h, tmp, runs=3):
    """The product's whole run_to_qvalues on the same workload files (host
    I/O included), per stage: each stage's median over ``runs`` runs (a new
    object and outdir each) after one run of the class's first-call costs
    (its total reported apart), and every run's total."""
    first = _e2e_once(h, tmp, runs)
    per = [_e2e_once(h, tmp, k) for k in range(runs)]
    out = {k: statistics.median(r[k] for r in per) for k in per[0]
           if k not in ('note', 'gc_collections', 'estimate_disp_stamps_ms')
           and per[0][k] is not None}
    out['gc_collections'] = [r['gc_collections'] for r in per]
    if 'estimate_disp_stamps_ms' in per[0]:
        out['estimate_disp_stamps_ms'] = [r['estimate_disp_stamps_ms']
                                          for r in per]
    out['runs_total_s'] = [r['total_s'] for r in per]
    out['first_run'] = {k: v for k, v in first.items() if k != 'note'}
    out['note'] = per[0]['note'] + '; per-stage medians of %d runs after ' \
        'the first (first_run: the same run paying the class\'s first-call ' \
        'costs: the reader / copy threads, allocator growth)' % runs
    return out


class _GcClock(object):
    """Wall time the interpreter's garbage collector spent between start()
    and stop() (gc.callbacks), and its collections of each generation."""

    def __init__(self):
        self.t0, self.total, self.counts = None, 0.0, [0, 0, 0]

    def __call__(self, phase, info):
        if phase == 'start':
            self.t0 = time.perf_counter()
        elif self.t0 is not None:
            self.total += time.perf_counter() - self.t0
            self.counts[info.get('generation', 0)] += 1
            self.t0 = None

    def start(self):
        import gc
        gc.callbacks.append(self)
        return self

    def stop(self):
        import gc
        gc.callbacks.remove(self)
        return self


_E2E_STAMPS = {}


def _e2e_stamps_on():
    """H3D_E2E_STAMPS=1: the e2e legs time the host calls inside
    estimate_disp (tools/class_stamps.py's wrappers), per run."""
    if os.environ.get('H3D_E2E_STAMPS') != '1' or 'acc' in _E2E_STAMPS:
        return
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(
        __file__)), 'tools'))
    import class_stamps as cs
    import numpy
    import torch
    from hic3defdr_amd import _native
    from hic3defdr_amd.analysis import analysis, core, resident
    ctx = _native.context(0)
    for name in ('estimate_disp_dev', 'table_gather_dev'):
        cs.wrap(ctx, name, 'ctx.' + name)
    for name in ('disp_pixels', 'start_session', 'lrt_buffers'):
        cs.wrap(resident.Resident, name, 'Resident.' + name)
    cs.wrap(analysis, 'to_host_async', 'to_host_async')
    cs.wrap(torch, 'empty', 'torch.empty')
    cs.wrap(numpy, 'empty', 'numpy.empty')
    cs.wrap(torch.cuda.Stream, 'synchronize', 'Stream.synchronize')
    cs.wrap(torch.Tensor, 'cpu', 'Tensor.cpu')
    for name in ('_save_npy', 'save_data', 'save_disp_fn', '_barrier',
                 '_shards', '_resident', '_cond_of_rep', '_ctx'):
        cls = core.CoreHiC3DeFDR if hasattr(core.CoreHiC3DeFDR, name) \
            else analysis.AnalyzingHiC3DeFDR
        cs.wrap(cls, name, 'HiC3DeFDR.' + name)
    _E2E_STAMPS['acc'] = cs.ACC


def _cgroup_throttled_s():
    """Seconds this cgroup's threads have been held by its CPU quota
    (cgroup v2 cpu.stat throttled_usec), or None."""
    try:
        with open('/sys/fs/cgroup/cpu.stat') as fh:
            for ln in fh:
                if ln.startswith('throttled_usec'):
                    return int(ln.split()[1]) * 1e-6
    except (OSError, ValueError, IndexError):
        pass
    return None


def _e2e_once(h, tmp, k, drop=False):
    from hic3defdr_amd import HiC3DeFDR
    out = os.path.join(tmp, 'out_e2e_%s' % k)
    os.makedirs(out, exist_ok=True)
    # the harness's own garbage (earlier legs and runs) collected and frozen
    # before the clock starts: the collections timed are the product's
    # (a 50 ms collection of the bench's leftovers had landed in cfg3's lrt)
    import gc
    gc.collect()
    gc.freeze()
    gcc = _GcClock().start()
    thr0 = _cgroup_throttled_s()
    h2 = HiC3DeFDR(raw_npz_patterns=h.raw_npz_patterns,
                   bias_patterns=h.bias_patterns, chroms=h.chroms,
                   design=h.design, outdir=out,
                   dist_thresh_max=h.dist_thresh_max,
                   loop_patterns=h.loop_patterns, res=h.res)
    t = [time.perf_counter()]
    g = [0.0]
    h2.prepare_data(verbose=False)
    t.append(time.perf_counter())
    g.append(gcc.total)
    stamps = _E2E_STAMPS.get('acc')
    if stamps is not None:
        stamps.clear()
    h2.estimate_disp()
    t.append(time.perf_counter())
    g.append(gcc.total)
    est_stamps = {k: round(v * 1e3, 3) for k, v in stamps.items()} \
        if stamps is not None else None
    h2.lrt(verbose=False)
    t.append(time.perf_counter())
    g.append(gcc.total)
    h2.bh()
    t.append(time.perf_counter())
    g.append(gcc.total)
    h2.flush()
    t.append(time.perf_counter())
    g.append(gcc.total)
    gcc.stop()
    thr1 = _cgroup_throttled_s()
    del h2
    if drop:
        shutil.rmtree(out, ignore_errors=True)
    out_stamps = {'estimate_disp_stamps_ms': est_stamps} if est_stamps else {}
    return {**out_stamps, 'gc_s': gcc.total, 'gc_collections': gcc.counts,
            'gc_estimate_disp_s': g[2] - g[1],
            'cgroup_throttled_s': (thr1 - thr0) if thr0 is not None and
            thr1 is not None else None,
            'total_s': t[-1] - t[0], 'prepare_data_s': t[1] - t[0],
            'estimate_disp_s': t[2] - t[1], 'lrt_s': t[3] - t[2],
            'bh_s': t[4] - t[3], 'outdir_flush_s': t[5] - t[4],
            'estimate_disp_plus_lrt_s': t[3] - t[1],
            'note': 'HiC3DeFDR.run_to_qvalues stages on the bench workload, '
                    'NPZ parse included; the .npy outdir writes land on a '
                    'background thread (write-behind) -- outdir_flush_s is '
                    'the wait for the last of them, inside total_s'}


def _outputs(torch, dev, n, C):
    t_p = torch.empty(n, dtype=torch.float64, device=dev)
    return {'p': t_p, 'llr': torch.empty_like(t_p), 'mu0': torch.empty_like(t_p),
            'q': torch.empty_like(t_p),
            'mu1': torch.empty((n, C), dtype=torch.float64, device=dev),
            'disp': torch.empty((n, C), dtype=torch.float64, device=dev)}


def _upload(torch, dev, raw, f, dist_np):
    return (torch.from_numpy(np.ascontiguousarray(raw, dtype=np.int32)).to(dev),
            torch.from_numpy(np.ascontiguousarray(f)).to(dev),
            torch.from_numpy(np.ascontiguousarray(dist_np, dtype=np.int32)).to(dev))


def table_lrt(torch, dev, ctx, D, C):
    """The step's dispersion table -> LRT. H3D_DEV_TABLE=2 (default): the
    smoother runs on the device from estimate_disp's result in place
    (h3d_estimate_disp_dev, then h3d_lrt_dev_tab) -- use `.estimate` for the
    estimate_disp of the step; 1: the device smoother on an uploaded table
    (h3d_disp_tables_dev); 0: the host smoother (h3d_disp_tables) and an
    uploaded table. Callers whose table comes from elsewhere (the distance
    re-shard's all-reduce, the emulation's filled rows) call the object
    with it; `estimate` falls back to that path when the mode is not 2."""
    from hic3defdr_amd import _native
    mode = int(os.environ.get('H3D_DEV_TABLE', '2'))
    if mode >= 1 and not hasattr(ctx.lib, 'h3d_disp_tables_dev'):
        mode = 0
    if mode == 2 and not hasattr(ctx.lib, 'h3d_estimate_disp_dev'):
        mode = 1
    pin = torch.empty((D, C), dtype=torch.float64).pin_memory()
    t_dpd = torch.empty((D, C), dtype=torch.float64, device=dev)
    t_tab = torch.empty_like(t_dpd)
    fused = {'ready': False}

    def ptrs(o):
        return (o['p'].data_ptr(), o['llr'].data_ptr(), o['mu0'].data_ptr(),
                o['mu1'].data_ptr(), o['disp'].data_ptr())

    def estimate(t_raw, t_f, t_dist, n, R, cond):
        if mode == 2:
            fused['ready'] = True
            return ctx.estimate_disp_dev(t_raw.data_ptr(), t_f.data_ptr(),
                                         t_dist.data_ptr(), n, R, cond, C, D,
                                         t_tab.data_ptr())
        return ctx.disp_per_dist_dev(t_raw.data_ptr(), t_f.data_ptr(),
                                     t_dist.data_ptr(), n, R, cond, C, D)

    def run(dpd, t_raw, t_f, t_dist, n, R, cond, o):
        if fused['ready']:       # the tables of this dpd are on the device
            fused['ready'] = False
            ctx.lrt_dev_tab(t_raw.data_ptr(), t_f.data_ptr(), t_dist.data_ptr(),
                            t_tab.data_ptr(), D, n, R, cond, *ptrs(o))
        elif mode >= 1:
            pin.numpy()[...] = dpd
            t_dpd.copy_(pin, non_blocking=True)   # the ctx's stream
            ctx.disp_tables_dev(t_dpd.data_ptr(), D, C, t_tab.data_ptr())
            ctx.lrt_dev_tab(t_raw.data_ptr(), t_f.data_ptr(), t_dist.data_ptr(),
                            t_tab.data_ptr(), D, n, R, cond, *ptrs(o))
        else:
            tab = _native.disp_tables(dpd)
            ctx.lrt_dev(t_raw.data_ptr(), t_f.data_ptr(), t_dist.data_ptr(),
                        tab, n, R, cond, *ptrs(o))
    run.estimate = estimate
    run.mode = mode
    return run


def timed_run(args, ctx, dist, dev, step):
    """W untimed steps, then exactly K timed steps between barrier +
    synchronize on both sides (HIP events on the roofline kernels inside),
    then one untimed step with every kernel scope timed. Returns
    (elapsed max over ranks, roofline-kernel events, per-kernel ms)."""
    import torch
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.profile_reset()
    ctx.profile(True, level=1)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.profile(False)
    ev = {k: ctx.profile_read(k) for k in ('disp_work', 'lrt')}
    ctx.profile_reset()
    ctx.profile(True, level=2)
    step()
    torch.cuda.synchronize()
    ctx.profile(False)
    per = {k: ctx.profile_read(k) for k in
           ('disp_reduce', 'disp_update', 'disp_nll', 'disp_prep', 'disp_work',
            'lrt')}
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, ev, per


def total_over_ranks(dist, dev, n):
    if not dist:
        return n
    import torch
    t = torch.tensor([n], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def bench_line(args, world, n_local, tot_px, R, C, elapsed, ev, per, bins,
               dmax, workload, parallelism, scaling, peaks=None):
    w_ms, w_n, w_bytes = ev['disp_work']
    l_ms, l_n, _ = ev['lrt']
    n_ms, n_n, n_bytes = per['disp_nll']
    w_avg_s = (w_ms / max(w_n, 1)) / 1e3
    w_bpl = w_bytes / max(w_n, 1)
    w_ach = w_bpl / w_avg_s / 1e9 if w_avg_s else 0.0
    l_avg_s = (l_ms / max(l_n, 1)) / 1e3
    l_ach = (n_local * bytes_per_lrt_pixel(R, C)) / l_avg_s / 1e9 \
        if l_avg_s else 0.0
    # per qcml iteration (= equalize launch): k_brent and k_brent_gang are
    # both launched every iteration, the device running one of them
    n_iter = max(w_n // max(args.steps, 1), 1)
    n_avg_s = (n_ms / n_iter) / 1e3
    # R_c = 2 runs the M = 2 instantiation (libh3d default; M = 4 with
    # H3D_DISP_M2=0): whichever the committed summary measured
    eq_pmc = pmc_kernel('k_disp_work<2, 4, 0, false>', bins, dmax) \
        or pmc_kernel('k_disp_work<4, 4, 0, false>', bins, dmax)
    nll_pmc = pmc_combined(('k_brent<2>', 'k_brent_gang<2>'), 'k_brent<2>',
                           bins, dmax) \
        or pmc_kernel('k_brent<4>', bins, dmax)
    # the table-fed instantiation the resident distance path launches
    lrt_pmc = pmc_kernel('k_lrt<4, 2, true>', bins, dmax) \
        or pmc_kernel('k_lrt<4, 2, false>', bins, dmax)
    pk_fp64, pk_hbm = _peak(peaks, 'fp64'), _peak(peaks, 'hbm')
    eq_fp64 = fp64_roof(eq_pmc, w_avg_s, pk_fp64)
    # the same kernel's launch time from the committed rocprofv3 stats of
    # this command (another run, often another box): the fraction the
    # committed profiles reproduce
    eq_rp = rocprof_avg_us('k_disp_work<2, 4, 0, false>', bins, dmax)
    eq_fp64_rp = fp64_roof(eq_pmc, eq_rp['avg_us'] / 1e6, pk_fp64) \
        if eq_rp else None
    roof = {
        'bound': 'fp64', 'kernel': 'k_disp_work<2,4,kEqualize,false> (equalize pass)',
        'achieved': eq_fp64['achieved'] if eq_fp64 else None,
        'peak': FP64_PEAK_TFLOPS, 'unit': 'TFLOP/s',
        'frac': eq_fp64['frac'] if eq_fp64 else None,
        'useful_frac': eq_fp64.get('useful_frac') if eq_fp64 else None,
        'peak_measured': pk_fp64,
        'frac_measured': eq_fp64.get('frac_measured') if eq_fp64 else None,
        'peak_source': 'peak: AMD MI355X spec, vector FP64 dense; '
                       'peak_measured: this GPU, measured_peaks (FMA chains)',
        'rocprof': {'avg_launch_us': eq_rp['avg_us'], 'calls': eq_rp['calls'],
                    'frac': eq_fp64_rp['frac'],
                    'frac_measured': eq_fp64_rp.get('frac_measured'),
                    'source': eq_rp['source'], 'command': eq_rp['command']}
        if eq_fp64_rp else None,
        'lane_util': eq_pmc['lane_util'] if eq_pmc else None,
        'flops_per_launch': eq_pmc['f64_flops'] if eq_pmc else None,
        'flops_source': 'FP64 flops issued per launch, PMC '
                        '(ADD+MUL+TRANS+2*FMA)_F64 x 64 lanes, '
                        'profiles/pmc_default.json; useful_frac = '
                        'frac x lane_util',
        'traffic': eq_pmc['hbm_bytes'] if eq_pmc else None,
        'traffic_source': 'PMC HBM bytes per launch (FETCH_SIZE x2 '
                          '+ WRITE_SIZE), profiles/pmc_default.json',
        'avg_launch_us': w_avg_s * 1e6, 'launches': w_n,
        'hbm': {'achieved': w_ach, 'peak': HBM_PEAK_GBS,
                'unit': 'GB/s', 'frac': w_ach / HBM_PEAK_GBS,
                'peak_measured': pk_hbm,
                'frac_measured': w_ach / pk_hbm if pk_hbm else None,
                'bytes_per_launch': w_bpl,
                'note': 'algorithmic: 20 B per equalize pixel-'
                        'replicate (raw 4 + f 8 in, pseudodata 8 '
                        'out)'},
        'note': 'FP64-VALU bound (SURVEY.md finding 3): q2qnbinom '
                'incomplete-gamma series / continued fractions'}
    kernels = {k: v[0] for k, v in per.items()}
    kernels['note'] = 'one extra untimed step, every kernel timed (rank 0)'
    return {
        'metric': METRIC, 'value': tot_px * args.steps / elapsed,
        'unit': 'pixels/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': elapsed / args.steps * 1e3,
        'higher_is_better': True, 'scaling': scaling,
        'vs_baseline': None, 'dtype': 'f64',
        'data': 'synthetic (SURVEY.md 8(d) generator; no demo data '
                'offline)',
        'config': {'workload': workload, 'disp_pixels_rank0': n_local,
                   'disp_pixels_total': tot_px, 'parallelism': parallelism},
        'roofline': roof,
        'kernel_rooflines': {
            'nll_brent': {
                'fp64': fp64_roof(nll_pmc, n_avg_s, pk_fp64),
                'hbm_traffic_per_launch': nll_pmc['hbm_bytes']
                if nll_pmc else None,
                'algorithmic_bytes_per_launch': n_bytes / n_iter,
                'avg_launch_us': n_avg_s * 1e6,
                'note': 'per qcml iteration: k_brent + k_brent_gang (both '
                        'launched, the device runs one), PMC summed over '
                        'both'},
            'lrt': {'fp64': fp64_roof(lrt_pmc, l_avg_s, pk_fp64),
                    'hbm': {'achieved': l_ach, 'peak': HBM_PEAK_GBS,
                            'unit': 'GB/s', 'frac': l_ach / HBM_PEAK_GBS,
                            'peak_measured': pk_hbm,
                            'frac_measured': l_ach / pk_hbm if pk_hbm
                            else None,
                            'bytes_per_pixel': bytes_per_lrt_pixel(R, C)},
                    'hbm_traffic_per_launch': lrt_pmc['hbm_bytes']
                    if lrt_pmc else None,
                    'avg_launch_us': l_avg_s * 1e6}},
        'kernels_ms_per_step': kernels,
        'measured_peaks': peaks,
        'work_per_step': {
            'equalize_pixel_reps': w_bytes / 20.0 / args.steps,
            'nll_pixel_reps': n_bytes / 8.0,
            'equalize_launches': w_n / args.steps},
    }


OTHER_CONFIGS = {
    # BASELINE configs[2] / [3] on one GPU: the pixels drawn
    # in the band by the same generator (synthetic.draw_band), no files
    'cfg3': dict(npc=(2, 2), dmax=200,
                 workload='cfg3: the mouse genome at 10 kb, 20 mm10-sized '
                          'chromosomes, 4 reps (2+2), dist_thresh_max 200, one '
                          'genome-wide pooled estimate_disp + lrt'),
    'cfg4': dict(npc=(6, 6, 6), dmax=400,
                 workload='cfg4: human chr1 at 5 kb (49,792 bins), 18 reps '
                          '(6+6+6), dist_thresh_max 400, estimate_disp + lrt '
                          '(chi2 df 2)'),
}


def other_config(torch, ctx, dev, name, steps=2, warmup=1, genome=None,
                 keep=None):
    """One of the other north-star shapes through the bench's step
    (estimate_disp + tables + lrt on HBM-resident inputs, as cfg2), timed on
    this GPU after the headline measurement: `steps` steps after `warmup`,
    kernel times from one extra profiled step. ``genome``: the inputs already
    drawn (cfg3_genome); ``keep`` (a dict): receives the last step's p and
    disp_per_dist."""
    from hic3defdr_amd import synthetic
    cfg = OTHER_CONFIGS[name]
    bins = list(synthetic.MM10_BINS) if name == 'cfg3' else [49792]
    t0 = time.perf_counter()
    if genome is not None:
        raw, f, dist_np = genome['raw'], genome['f'], genome['dist']
        gen_s = genome['generate_s']
    else:
        # (one chromosome: its replicates on the threads; the data do not
        # depend on the thread count -- a seeded stream per replicate)
        parts = synthetic.draw_genome(bins, cfg['npc'], cfg['dmax'], seed=0,
                                      workers=16) if len(bins) > 1 else \
            [synthetic.draw_band(bins[0], cfg['npc'], cfg['dmax'], seed=0,
                                 chrom_index=0, workers=16)]
        raw = np.concatenate([p[0] for p in parts])
        f = np.concatenate([p[1] for p in parts])
        dist_np = np.concatenate([p[2] for p in parts])
        del parts
        gen_s = time.perf_counter() - t0
    n, R = raw.shape
    C = len(cfg['npc'])
    D = cfg['dmax'] + 1
    cond = np.repeat(np.arange(C), cfg['npc']).astype(np.int32)
    t_raw, t_f, t_dist = _upload(torch, dev, raw, f, dist_np)
    present = np.isin(np.arange(D), dist_np)
    del raw, f, dist_np
    genome = None
    o = _outputs(torch, dev, n, C)
    torch.cuda.synchronize()
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    tl = table_lrt(torch, dev, ctx, D, C)

    def step():
        dpd = tl.estimate(t_raw, t_f, t_dist, n, R, cond)
        tl(dpd, t_raw, t_f, t_dist, n, R, cond, o)
        return dpd

    first = None
    for _ in range(warmup):
        first = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(steps):
        dpd = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    ctx.profile_reset()
    ctx.profile(True, level=2)
    step()
    torch.cuda.synchronize()
    ctx.profile(False)
    ks = {k: ctx.profile_read(k)[0] for k in
          ('disp_work', 'disp_nll', 'disp_update', 'disp_prep', 'lrt')}
    p = o['p'].cpu().numpy()
    if keep is not None:
        keep['p'], keep['dpd'] = p, dpd
    ctx.set_stream(None)
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    del o, t_raw, t_f, t_dist
    torch.cuda.empty_cache()
    return {
        'workload': cfg['workload'], 'bins': int(sum(bins)), 'reps': int(R),
        'conds': int(C), 'disp_pixels': int(n), 'steps': steps,
        'warmup': warmup, 'value': n * steps / el, 'unit': 'pixels/s',
        'ms_per_step': el / steps * 1e3, 'kernels_ms_per_step': ks,
        'generate_s': gen_s,
        'checks': {
            'disp_finite_where_present': bool(np.all(np.isfinite(
                dpd[present]))),
            'disp_nan_where_absent': bool(np.all(np.isnan(dpd[~present]))),
            'p_in_0_1': bool(np.all((p >= 0) & (p <= 1))),
            'deterministic_disp': None if first is None else bool(
                np.array_equal(first, dpd, equal_nan=True))}}


def run_cfg2(args, world, rank, local, dist, ctx, dev, cpu, cfg3=None,
             peaks=None):
    """Weak scaling: one 20k-bin chromosome per rank (BASELINE configs[1])."""
    import torch
    from hic3defdr_amd import _native, parallel
    tmp = tempfile.mkdtemp(prefix='h3dbench_r%d_' % rank)
    try:
        h, kw = make_workload(tmp, 'chrB%d' % rank, args.bins, args.dmax, rank)
        # this rank's own chromosome, prepared directly: the object's
        # chrom=None path shards over the process group (LPT over ITS
        # chromosome list -- here one per rank -- would leave rank > 0 idle)
        for c in h.chroms:
            h.prepare_data(chrom=c, verbose=False)
        raw, f, dist_np, _ = h._f_and_dist()
        design = kw['design']
        R, C = design.shape
        D = args.dmax + 1
        cond = design.argmax(axis=1).astype(np.int32)
        n = len(raw)
        t_raw, t_f, t_dist = _upload(torch, dev, raw, f, dist_np)
        o = _outputs(torch, dev, n, C)
        torch.cuda.synchronize()
        # libh3d and the RCCL collectives share one real stream (torch's
        # default stream has handle 0 = "the ctx's own stream" to libh3d)
        stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        ctx.set_stream(stream.cuda_stream)
        # N > 1: pixels re-sharded by distance (one all_to_all, single-GPU
        # driver per rank, one table all-reduce); H3D_DISP_SHARD=pass keeps
        # them in place and all-reduces the NLL sums of every data pass
        by_dist = world > 1 and os.environ.get('H3D_DISP_SHARD') != 'pass'
        reduce = parallel.make_allreduce() if world > 1 and not by_dist \
            else None
        if args.noop_reduce and world == 1:
            def reduce(ptr, count):
                pass

        tl = table_lrt(torch, dev, ctx, D, C)
        last = {}

        def step():
            if by_dist:
                dpd = parallel.disp_per_dist_by_distance(
                    ctx, t_raw, t_f, t_dist, cond, C, D)
            elif reduce is None:
                dpd = tl.estimate(t_raw, t_f, t_dist, n, R, cond)
            else:
                dpd = ctx.disp_per_dist_dev(t_raw.data_ptr(), t_f.data_ptr(),
                                            t_dist.data_ptr(), n, R, cond, C,
                                            D, reduce=reduce)
            tl(dpd, t_raw, t_f, t_dist, n, R, cond, o)
            last['dpd'] = dpd
            return dpd

        elapsed, ev, per = timed_run(args, ctx, dist, dev, step)
        tot_px = total_over_ranks(dist, dev, n)
        if rank != 0:
            return None
        out = bench_line(
            args, world, n, tot_px, R, C, elapsed, ev, per, args.bins,
            args.dmax,
            'cfg2: per GPU 1 chrom x %d bins, 4 reps (2+2), dist_thresh_max '
            '%d, estimate_disp (qcml) + lrt on HBM-resident inputs'
            % (args.bins, args.dmax),
            'dp%d (chromosome shards; %s)' % (
                world, 'per-pass NLL sums, no-op reduce (the N > 1 driver on '
                'one GPU)' if reduce and world == 1 else
                'in-kernel Brent searches' if world == 1 else
                'distance re-shard: all_to_all of the disp pixels, in-kernel '
                'Brent per rank, table all-reduce' if by_dist
                else 'per-pass NLL all-reduce over RCCL'), 'weak',
            peaks=peaks)
        out['gang_aborts'] = ctx.profile_read('gang_aborts')[1]
        # the last step's disp_per_dist and p, hashed: A/B runs of kernel
        # variants that must not move a bit compare this
        torch.cuda.synchronize()
        hsh = hashlib.sha256(np.ascontiguousarray(last['dpd']).tobytes())
        hsh.update(o['p'].cpu().numpy().tobytes())
        out['result_sha16'] = hsh.hexdigest()[:16]
        if world == 1:
            out['parity_vs_reference'] = parity_vs_reference(
                ctx, o, n, args.bins, args.dmax, rank, last.get('dpd'))
        if cpu is not None:
            out['cpu_baseline'] = cpu[0]
            out['parity_sample'] = sample_parity(ctx, cpu[1], args.dmax)
        if world == 1 and not args.no_e2e:
            # the bench's own objects (CPU legs, fixtures) out of the
            # collector's young generations: their collections are not the
            # product's (cfg3 e2e: 60 ms of gc per run before, r06ae)
            import gc
            gc.collect()
            gc.freeze()
            _e2e_stamps_on()
            out['e2e_run_to_qvalues'] = e2e_wall(h, tmp)
            if cfg3 and cfg3.get('files'):
                base, kw, w_s = cfg3['files']
                try:
                    out['e2e_cfg3_run_to_qvalues'] = e2e_cfg3(base, kw, w_s)
                finally:
                    shutil.rmtree(base, ignore_errors=True)
        if world == 1 and not args.no_other_configs:
            oc, keep = {}, {}
            g3 = cfg3.pop('genome', None) if cfg3 else None
            oc['cfg3'] = other_config(torch, ctx, dev, 'cfg3', genome=g3,
                                      keep=keep)
            del g3
            if cfg3 and 'cpu' in cfg3:
                row, cpu_p, cpu_dpd = cfg3.pop('cpu')
                row['gpu_over_cpu'] = oc['cfg3']['value'] / row['value']
                oc['cfg3']['cpu_baseline'] = row
                par = cfg3_vs_cpu(ctx, keep['p'], keep['dpd'], cpu_p, cpu_dpd,
                                  OTHER_CONFIGS['cfg3']['dmax'])
                oc['cfg3']['vs_cpu_restatement'] = par
                oc['cfg3']['identical_calls'] = par['identical_calls']
                del cpu_p, cpu_dpd
            keep.clear()
            oc['cfg4'] = other_config(torch, ctx, dev, 'cfg4')
            out['other_configs'] = oc
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def run_cfg3(args, world, rank, local, dist, ctx, dev, peaks=None):
    """Strong scaling over the whole mouse genome (BASELINE configs[2])."""
    import torch
    from hic3defdr_amd import _native, parallel, synthetic
    bins = synthetic.MM10_BINS
    dmax = args.dmax3
    D = dmax + 1
    # H3D_BENCH_EMULATE=r/N (N = 1 only): time rank r's share of an N-GPU
    # run on this one GPU -- estimate_disp over the distances the LPT owner
    # table gives rank r (what it holds after the all_to_all), lrt + BH over
    # the chromosomes LPT gives it; the collectives are not run
    emu = os.environ.get('H3D_BENCH_EMULATE') if world == 1 else None
    e_rank, e_world = (int(v) for v in emu.split('/')) if emu else (rank, world)
    assign = parallel.lpt_assign({i: b for i, b in enumerate(bins)}, e_world)
    mine = sorted(assign[e_rank])
    t0 = time.perf_counter()
    # the re-shard ships the keys of f (row, chromosome, size-factor row;
    # H3D_RESHARD_FULL=1: the full record with f)
    compact = world > 1 and os.environ.get('H3D_RESHARD_FULL') != '1'
    parts = synthetic.draw_genome(bins, (2, 2), dmax, seed=0,
                                  indices=None if emu else mine, workers=16,
                                  keys=compact)
    keys = None
    if compact:
        keys = parallel.PixelKeys(
            torch.from_numpy(np.concatenate([p[3] for p in parts])).to(dev),
            torch.from_numpy(np.concatenate(
                [np.full(len(p[0]), i, dtype=np.int32)
                 for i, p in zip(mine, parts)])).to(dev),
            torch.zeros(sum(len(p[0]) for p in parts), dtype=torch.int32,
                        device=dev),
            {i: (p[4], np.ones((1, 4))) for i, p in zip(mine, parts)},
            len(bins))
    if emu:
        own = [p for i, p in enumerate(parts) if i in mine]
        d_all = np.concatenate([p[2] for p in parts])
        owner = parallel.distance_owners(
            np.bincount(d_all, minlength=D)[:D], e_world)
        keep = owner[d_all] == e_rank
        e_raw = np.concatenate([p[0] for p in parts])[keep]
        e_f = np.concatenate([p[1] for p in parts])[keep]
        e_dist = d_all[keep]
        del d_all
        parts = own
    raw = np.concatenate([p[0] for p in parts])
    f = np.concatenate([p[1] for p in parts])
    dist_np = np.concatenate([p[2] for p in parts])
    del parts
    gen_s = time.perf_counter() - t0
    R, C = 4, 2
    cond = np.array([0, 0, 1, 1], dtype=np.int32)
    n = len(raw)
    t_raw, t_f, t_dist = _upload(torch, dev, raw, f, dist_np)
    del raw, f
    if emu:
        e_n = len(e_raw)
        te_raw, te_f, te_dist = _upload(torch, dev, e_raw, e_f, e_dist)
        del e_raw, e_f
    o = _outputs(torch, dev, n, C)
    torch.cuda.synchronize()
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    bh_ops = parallel.DeviceBhOps(ctx)

    tl = table_lrt(torch, dev, ctx, D, C)

    # H3D_DISP_SHARD=pass (N > 1): pixels stay with their chromosomes' rank,
    # the per-pass NLL sums are all-reduced (no pixel exchange);
    # --noop-reduce (N = 1): that driver with a no-op reduce (measurement)
    per_pass = (world > 1 and os.environ.get('H3D_DISP_SHARD') == 'pass') \
        or (world == 1 and args.noop_reduce)
    reduce = (parallel.make_allreduce() if world > 1 else
              (lambda ptr, count: None)) if per_pass else None

    def step():
        if per_pass:
            dpd = ctx.disp_per_dist_dev(t_raw.data_ptr(), t_f.data_ptr(),
                                        t_dist.data_ptr(), n, R, cond, C, D,
                                        reduce=reduce)
        elif world > 1:
            dpd = parallel.disp_per_dist_by_distance(ctx, t_raw, t_f, t_dist,
                                                     cond, C, D, keys=keys)
        elif emu:
            dpd = ctx.disp_per_dist_dev(te_raw.data_ptr(), te_f.data_ptr(),
                                        te_dist.data_ptr(), e_n, R, cond, C, D)
            # the other ranks' rows (not run here): interpolated over this
            # rank's with a 2 % ripple, so the smoother sees a table of the
            # usual shape (a piecewise-linear table drives the weighted
            # lowess' rolling variance to ~0 and its fits degenerate)
            for c in range(C):
                fin = np.isfinite(dpd[:, c])
                gap = ~fin & (np.arange(D) >= 4)
                gi = np.flatnonzero(gap)
                dpd[gap, c] = np.interp(gi, np.flatnonzero(fin), dpd[fin, c]) \
                    * (1 + 0.02 * np.sin(1.7 * gi + c))
        else:
            dpd = tl.estimate(t_raw, t_f, t_dist, n, R, cond)
        tl(dpd, t_raw, t_f, t_dist, n, R, cond, o)
        if world > 1:
            o['q'] = parallel.bh_sharded(o['p'], bh_ops)
        else:
            ctx.bh_dev(o['p'].data_ptr(), n, o['q'].data_ptr())
        return dpd

    elapsed, ev, per = timed_run(args, ctx, dist, dev, step)
    tot_px = total_over_ranks(dist, dev, n)
    if rank != 0:
        return None
    out = bench_line(
        args, world, n, tot_px, R, C, elapsed, ev, per, sum(bins), dmax,
        'cfg3: whole mouse genome at 10 kb, 20 mm10-sized chromosomes (%d '
        'bins), 4 reps (2+2), dist_thresh_max %d, chromosomes LPT-sharded '
        'over %d GPU(s); step = genome-wide estimate_disp + lowess tables + '
        'lrt + genome-wide BH on HBM-resident inputs' % (sum(bins), dmax,
                                                          world),
        'dp%d: %s' % (world, ('one GPU, the per-pass driver with a no-op '
                              'reduce' if per_pass else 'one GPU')
                      if world == 1 else
                      'per-pass NLL all-reduce (pixels stay with their '
                      'chromosomes), LRT on own chromosomes, genome-wide BH '
                      'as a sample sort over the ranks' if per_pass else
                      'distance re-shard (LPT distance owners, all_to_all of '
                      'the disp pixels as %s, single-GPU driver per rank, '
                      'table all-reduce), LRT on own chromosomes, genome-wide BH '
                      'as a sample sort over the ranks (two all_to_alls of '
                      'the p-values)' % ('15-byte key records, f rebuilt on '
                                         'arrival' if compact else
                                         '52-byte raw / f / dist records')),
        'strong', peaks=peaks)
    out['gang_aborts'] = ctx.profile_read('gang_aborts')[1]
    out['config']['chromosomes_rank0'] = [int(i) for i in mine]
    out['config']['generate_s_rank0'] = gen_s
    if emu:
        out['emulated'] = {
            'rank': e_rank, 'of': e_world, 'disp_pixels_estimate_disp': e_n,
            'note': 'one rank\'s share of an N-GPU cfg3 run, timed alone on '
                    'one GPU: estimate_disp over its LPT-owned distances, lrt '
                    '+ BH over its LPT-owned chromosomes; no collectives (the '
                    'all_to_all, table all-reduce and BH exchanges are not '
                    'run). value = its pixels / time, NOT a scaling number'}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--config', choices=('auto', 'cfg2', 'cfg3'),
                    default='auto',
                    help='auto: cfg2 (BASELINE configs[1], 1 GPU) at N = 1, '
                         'cfg3 (configs[2], the genome sharded over the '
                         'node) at N > 1')
    ap.add_argument('--bins', type=int, default=20000)
    ap.add_argument('--dmax', type=int, default=250)
    ap.add_argument('--dmax3', type=int, default=200)
    ap.add_argument('--cpu-bins', type=int, default=1000,
                    help='the faithful CPU row sample')
    ap.add_argument('--cpu-full-bins', type=int, default=20000,
                    help='the fallback-fixed CPU row (0: the sample)')
    ap.add_argument('--cpu-full-runs', type=int, default=3,
                    help='runs of the full-chromosome CPU row (median)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-e2e', action='store_true')
    ap.add_argument('--no-e2e-cfg3', action='store_true',
                    help='skip the cfg3 run_to_qvalues-from-files leg')
    ap.add_argument('--no-cpu-cfg3', action='store_true',
                    help='skip the whole-genome CPU restatement run (cfg3)')
    ap.add_argument('--no-peaks', action='store_true',
                    help='skip the measured FP64 / HBM peaks')
    ap.add_argument('--no-other-configs', action='store_true',
                    help='skip the cfg3 / cfg4 lines measured after the '
                         'headline (N = 1)')
    ap.add_argument('--noop-reduce', action='store_true',
                    help='measurement: run the multi-rank estimate_disp driver '
                         '(per-pass NLL sums through the reduce hook) on one '
                         'GPU with a no-op reduce, i.e. the N > 1 kernel and '
                         'host-sync path without the collective')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    # H3D_DEVICE / H3D_BENCH_BACKEND=gloo: rehearsal of the N > 1 path with
    # several ranks on one GPU (RCCL needs one GPU per rank); the driver's
    # runs use LOCAL_RANK's GPU and nccl
    local = int(os.environ.get('H3D_DEVICE', os.environ.get('LOCAL_RANK', '0')))
    backend = os.environ.get('H3D_BENCH_BACKEND', 'nccl')
    config = args.config if args.config != 'auto' else \
        ('cfg2' if world == 1 else 'cfg3')
    cpu, cfg3 = None, {}
    if world == 1 and config == 'cfg2' and not args.no_cpu_baseline:
        cpu = cpu_baseline_run(args.cpu_full_bins, args.cpu_bins,
                               args.dmax, full_runs=args.cpu_full_runs)
        # (before the GPU: the pool forks)
    if world == 1 and config == 'cfg2':
        d3 = OTHER_CONFIGS['cfg3']['dmax']
        if not args.no_other_configs:
            cfg3['genome'] = cfg3_genome(d3)
            if not args.no_cpu_baseline and not args.no_cpu_cfg3:
                print('bench: cfg3 CPU leg (whole genome, %d pixels) ...'
                      % len(cfg3['genome']['raw']), file=sys.stderr,
                      flush=True)
                cfg3['cpu'] = cpu_cfg3_run(cfg3['genome'], d3)
        if not args.no_e2e and not args.no_e2e_cfg3:
            cfg3['files'] = e2e_cfg3_files(d3)
            # the genome's ~2 GB of input files reach the disk now, not in
            # the page cache's background writeback during the timed legs
            os.sync()
    import torch
    torch.cuda.set_device(local)
    # the process's threads on its GPU's NUMA node (H3D_NUMA_BIND=0: not)
    from hic3defdr_amd import numa
    numa_bind = numa.maybe_bind(local, default=True)
    peaks = None
    if rank == 0 and not args.no_peaks:
        peaks = measured_peaks(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == 'nccl':
            dist.init_process_group('nccl',
                                    device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    from hic3defdr_amd import _native
    ctx = _native.context(local)
    dev = torch.device('cuda', local)
    try:
        if config == 'cfg2':
            out = run_cfg2(args, world, rank, local, dist, ctx, dev, cpu,
                           cfg3, peaks)
        else:
            out = run_cfg3(args, world, rank, local, dist, ctx, dev, peaks)
        if rank == 0:
            out['numa_bind'] = numa_bind
            print(json.dumps(out), flush=True)
    finally:
        if dist:
            dist.destroy_process_group()


if __name__ == '__main__':
    main()
