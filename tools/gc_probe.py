"""Which stage of the cfg3 run_to_qvalues (from files) triggers the
interpreter's larger collections, and what young objects they scan (GPU box).
    python tools/gc_probe.py"""
import collections
import gc
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import pandas as pd
    import torch  # noqa: F401
    from hic3defdr_amd import HiC3DeFDR, numa, synthetic
    numa.maybe_bind(0, default=True)
    base = tempfile.mkdtemp(prefix='h3d_gc_')
    kw = synthetic.write_genome(base, synthetic.MM10_BINS, seed=3, workers=16,
                                dmax=200)
    os.sync()
    design = pd.DataFrame(kw['design'], index=kw['reps'], columns=kw['conds'])
    stage = ['-']
    log = []
    t0 = [0.0]

    def cb(phase, info):
        if phase == 'start':
            t0[0] = time.perf_counter()
            if info['generation'] >= 1:
                young = collections.Counter(
                    type(o).__name__ for g in range(info['generation'] + 1)
                    for o in gc.get_objects(generation=g))
                log.append((stage[0], info['generation'], young.most_common(8)))
        else:
            dt = time.perf_counter() - t0[0]
            if dt > 1e-3:
                log.append((stage[0], info['generation'], 'took %.1f ms' % (dt * 1e3)))
    for run in range(2):
        gc.collect()
        gc.freeze()
        if run:
            gc.callbacks.append(cb)
        h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                      bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                      design=design, outdir=os.path.join(base, 'out%d' % run),
                      dist_thresh_max=200, loop_patterns=kw['loop_patterns'],
                      res=10000)
        for name, fn in (('prepare_data', lambda: h.prepare_data(verbose=False)),
                         ('estimate_disp', h.estimate_disp),
                         ('lrt', lambda: h.lrt(verbose=False)), ('bh', h.bh),
                         ('flush', h.flush)):
            stage[0] = name
            t = time.perf_counter()
            fn()
            print(run, name, '%.1f ms' % ((time.perf_counter() - t) * 1e3), flush=True)
        del h
    gc.callbacks.remove(cb)
    for row in log:
        print(row)


if __name__ == '__main__':
    main()
