"""The device's own spread on the headline chromosome (cfg2, seed 0; the
tests/golden/full_cfg2.npz workload) under pixel-order permutations of its
input: the product's prepare_data once, then disp_per_dist + tables + lrt per
permutation (k = 0: the reference's pixel order). Writes
gpurun_out/r04_dev_spread.npz (disp_per_dist, p on full_cfg2's sample and top
pixels per permutation) and prints the comparison with full_cfg2.npz.

    python tools/r04_dev_spread.py [--perms 6]
"""
import argparse
import os
import shutil
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--perms', type=int, default=6)
    args = ap.parse_args()
    import pandas as pd
    from hic3defdr_amd import HiC3DeFDR, _native, synthetic
    g = np.load(os.path.join(REPO, 'tests', 'golden', 'full_cfg2.npz'))
    tmp = tempfile.mkdtemp(prefix='h3d_spread_')
    try:
        kw = synthetic.write_dataset(tmp, {'chrB0': 20000},
                                     dist_thresh_max=250, seed=0)
        design = pd.DataFrame(kw['design'], index=kw['reps'],
                              columns=kw['conds'])
        h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                      bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                      design=design, outdir=os.path.join(tmp, 'out'),
                      dist_thresh_max=250)
        h.prepare_data(verbose=False)
        raw, f, dist, _ = h._f_and_dist()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    ctx = _native.context(0)
    cond = kw['design'].argmax(axis=1)
    C, D = kw['design'].shape[1], 251
    s, t = g['sample_idx'], g['top_idx']
    ref = g['disp_per_dist']
    fin = np.isfinite(ref)
    out = {}
    for k in range(args.perms):
        if k:
            perm = np.random.default_rng(k).permutation(len(raw))
        else:
            perm = np.arange(len(raw))
        dpd = ctx.disp_per_dist(raw[perm], f[perm], dist[perm], cond, C, D)
        tab = _native.disp_tables(dpd)
        p = ctx.lrt(raw, f, dist, tab, cond, want_disp=False)[0]
        out['disp_per_dist__%d' % k] = dpd
        out['p_sample__%d' % k] = p[s]
        out['p_top__%d' % k] = p[t]
        rel = np.abs(dpd[fin] - ref[fin]) / ref[fin]
        bad = np.flatnonzero(rel > 1e-6)
        segs = [(int(np.flatnonzero(fin.ravel())[b] // C),
                 int(np.flatnonzero(fin.ravel())[b] % C), float(rel[b]))
                for b in bad]
        print('perm %d: segments > 1e-6 rel vs reference %d %s; max rel %.3g; '
              'sample p max rel %.3g, top p %.3g' % (
                  k, len(bad), segs, rel.max(),
                  np.max(np.abs(p[s] - g['p']) / g['p']),
                  np.max(np.abs(p[t] - g['top_p']) / g['top_p'])), flush=True)
    os.makedirs(os.path.join(REPO, 'gpurun_out'), exist_ok=True)
    np.savez_compressed(os.path.join(REPO, 'gpurun_out', 'r04_dev_spread.npz'),
                        **out)


if __name__ == '__main__':
    main()
