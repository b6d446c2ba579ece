"""Where the class's estimate_disp / lrt wall time goes beyond its kernels:
wraps the host calls of the two stages in wall-clock timers and runs
bench.py's cfg2 workload through HiC3DeFDR (runs on the GPU box).

    python tools/class_stamps.py [--runs 5]

Prints per stage the median wall time of each wrapped call (summed per run)
and the stage totals.
"""
import argparse
import collections
import functools
import json
import os
import statistics
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ACC = collections.defaultdict(float)


def wrap(obj, name, label=None):
    fn = getattr(obj, name)
    label = label or '%s.%s' % (getattr(obj, '__name__', type(obj).__name__),
                                name)

    @functools.wraps(fn)
    def timed(*a, **k):
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            ACC[label] += time.perf_counter() - t
    setattr(obj, name, timed)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--runs', type=int, default=5)
    ap.add_argument('--no-flush', action='store_true',
                    help='no flush() between prepare_data and estimate_disp '
                         '(prepare_data\'s background copies and writes still '
                         'landing, as in run_to_qvalues)')
    args = ap.parse_args()
    import bench
    import torch  # noqa: F401
    from hic3defdr_amd import HiC3DeFDR, _native
    from hic3defdr_amd.analysis import analysis, core, d2h, resident
    tmp = tempfile.mkdtemp(prefix='h3d_stamps_')
    h, _ = bench.make_workload(tmp, 'chrB', 20000, 250, seed=0)
    ctx = _native.context(0)
    for name in ('estimate_disp_dev', 'table_gather_dev', 'lrt_dev_tab',
                 'disp_pixels_dev', 'bh_dev'):
        wrap(ctx, name, 'ctx.' + name)
    for name in ('disp_pixels', 'start_session', 'lrt_session',
                 'keep_pvalues', 'pvalues_session', '_current'):
        wrap(resident.Resident, name, 'Resident.' + name)
    wrap(analysis, 'to_host_async', 'to_host_async(analysis)')
    # inside to_host_async and the stages: allocations and the copy pool
    import numpy
    wrap(torch, 'empty', 'torch.empty')
    wrap(numpy, 'empty', 'numpy.empty')
    wrap(d2h, '_pool', 'd2h._pool')
    wrap(resident.Resident, 'lrt_buffers', 'Resident.lrt_buffers')
    wrap(torch.cuda, 'Event', 'torch.cuda.Event')
    for name in ('_save_npy', 'save_data', 'save_disp_fn', '_barrier',
                 '_shards', '_resident', '_cond_of_rep', '_lrt_run'):
        cls = core.CoreHiC3DeFDR if hasattr(core.CoreHiC3DeFDR, name) \
            else analysis.AnalyzingHiC3DeFDR
        wrap(cls, name, 'HiC3DeFDR.' + name)
    per = []
    for k in range(args.runs + 1):
        out = os.path.join(tmp, 'out_%d' % k)
        h2 = HiC3DeFDR(raw_npz_patterns=h.raw_npz_patterns,
                       bias_patterns=h.bias_patterns, chroms=h.chroms,
                       design=h.design, outdir=out,
                       dist_thresh_max=h.dist_thresh_max)
        h2.prepare_data(verbose=False)
        if not args.no_flush:
            h2.flush()
        row = {}
        for stage, fn in (('estimate_disp', h2.estimate_disp),
                          ('lrt', lambda: h2.lrt(verbose=False))):
            ACC.clear()
            t = time.perf_counter()
            fn()
            row[stage] = dict(ACC, total=time.perf_counter() - t)
        h2.flush()
        if k:
            per.append(row)
    out = {}
    for stage in per[0]:
        keys = sorted(set().union(*[r[stage].keys() for r in per]))
        out[stage] = {key: statistics.median(r[stage].get(key, 0.0)
                                             for r in per) * 1e3
                      for key in keys}
    print(json.dumps({'ms_medians': out, 'runs': args.runs}, indent=1))


if __name__ == '__main__':
    main()
