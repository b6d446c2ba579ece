"""Where prepare_data's time goes on the bench workload (GPU box): the
stage's pieces timed by wrapping them (inputs = NPZ inflate + bias + loop
clusters on the reader thread; union / size factors / scale+disp on the
device; the queueing of the outdir saves), median of --runs runs.

    python tools/prep_profile.py [--bins 20000] [--dmax 250] [--runs 5]
    python tools/prep_profile.py --genome [--runs 3]   (cfg3: 20 chromosomes)

With --genome every piece is summed per run (median over the runs of the
per-run sums); ``prepare_data - prepare_chrom`` is the main thread's wait
for the reader.
"""
import argparse
import collections
import json
import os
import statistics
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--bins', type=int, default=20000)
    ap.add_argument('--dmax', type=int, default=250)
    ap.add_argument('--runs', type=int, default=5)
    ap.add_argument('--genome', action='store_true')
    ap.add_argument('--cprofile', type=int, default=0,
                    help='cProfile the last run, print the top N (stderr)')
    args = ap.parse_args()
    import pandas as pd
    from hic3defdr_amd import HiC3DeFDR, synthetic, _native
    from hic3defdr_amd.analysis import analysis, resident
    tmp = tempfile.mkdtemp(prefix='h3d_prep_')
    if args.genome:
        args.dmax = 200
        kw = synthetic.write_genome(tmp, synthetic.MM10_BINS, seed=3,
                                    workers=16, dmax=args.dmax)
    else:
        kw = synthetic.write_dataset(tmp, {'chrS': args.bins},
                                     dist_thresh_max=args.dmax, seed=123)
    design = pd.DataFrame(kw['design'], index=kw['reps'], columns=kw['conds'])
    acc = collections.defaultdict(list)

    def wrap(owner, name, label):
        f = getattr(owner, name)

        def g(*a, **k):
            t = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                acc[label].append(time.perf_counter() - t)
        setattr(owner, name, g)
    wrap(HiC3DeFDR, '_prepare_inputs', 'inputs (reader)')
    wrap(analysis, '_canonical_csr', 'one NPZ (reader pool)')
    wrap(HiC3DeFDR, '_prepare_chrom', 'prepare_chrom')
    wrap(_native.Context, 'sparse_union', '  sparse_union')
    wrap(resident.Resident, 'size_factors', '  size_factors')
    wrap(resident.Resident, 'scale_disp', '  scale_disp')
    wrap(resident.Resident, 'keep', '  keep')
    wrap(HiC3DeFDR, '_save_npy', '  _save_npy (each)')
    wrap(analysis, 'pixel_membership', '  loop_idx (pixel_membership)')
    wrap(analysis, 'load_cluster_pixels', 'load_cluster_pixels (reader)')
    runs = []
    for k in range(args.runs + 1):
        h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                      bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                      design=design, outdir=os.path.join(tmp, 'o%d' % k),
                      dist_thresh_max=args.dmax,
                      loop_patterns=kw.get('loop_patterns') if args.genome
                      else None, res=10000)
        if k == 0:
            h.prepare_data(verbose=False)   # first-call costs
            h.flush()
            acc.clear()
            continue
        prof = None
        if args.cprofile and k == args.runs:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t = time.perf_counter()
        h.prepare_data(verbose=False)
        acc['prepare_data'].append(time.perf_counter() - t)
        if prof is not None:
            import pstats
            prof.disable()
            pstats.Stats(prof, stream=sys.stderr).sort_stats(
                'tottime').print_stats(args.cprofile)
        t = time.perf_counter()
        h.flush()
        acc['flush'].append(time.perf_counter() - t)
        if args.genome:
            runs.append({key: sum(v) for key, v in acc.items()})
            acc.clear()
        import shutil
        shutil.rmtree(os.path.join(tmp, 'o%d' % k), ignore_errors=True)
    if args.genome:
        out = {key: {'median_ms_per_run': 1e3 * statistics.median(
            r.get(key, 0.0) for r in runs)} for key in runs[0]}
    else:
        out = {k: {'median_ms': 1e3 * statistics.median(v), 'calls': len(v)}
               for k, v in acc.items()}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
