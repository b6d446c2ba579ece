"""Which weighted-lowess mode agrees with the reference more often, measured
from the PRODUCT's own disp_per_dist.

For the five e2e fixtures and the full-size cfg1 / cfg2 workloads: the
product's run_to_qvalues gives disp_per_dist; both smoother modes are fitted
to it on the host (libh3d h3d_disp_tables: ``weighted=True`` -- the pinned
minimum weight, the default -- and ``weighted='reference'`` -- the
reference's ``w * (1/w)`` floor, lowess.py:195-204); each mode's table goes
through the product's LRT (GPU) and both are compared with the reference's
own run on the same inputs (tests/golden: e2e_<name>.npz, full_cfg1.npz,
full_cfg2.npz, lowess_mechanism.npz order 0):
- per condition, does the fitted function (core.DispFn, the disp_fn the
  outdir pickles) match the reference's disp_fn within 1e-6 at every
  present distance;
- the p-values compared: how many within 1e-6 relative, the max relative
  difference, identical calls at q < 0.05 (BH of the compared p).
Writes the JSON to stdout (committed as tests/golden/smoother_census.json;
tests/test_lowess_mechanism.py reads it). Runs on the GPU box:

    python tools/smoother_census.py > gpurun_out/smoother_census.json
"""
import json
import os
import shutil
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests'))

E2E = ('small2', 'c3r9', 'r18c3', 'r16c2', 'lwdrop')
MODES = (('pinned', True), ('reference', 'reference'))


def _run(kw, outdir, design, loop_patterns, res):
    import pandas as pd
    from hic3defdr_amd import HiC3DeFDR
    h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                  bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                  design=pd.DataFrame(design, index=kw['reps'],
                                      columns=kw['conds']),
                  outdir=outdir, dist_thresh_max=kw['dist_thresh_max'],
                  loop_patterns=loop_patterns, res=res)
    h.run_to_qvalues(verbose=False)
    h.flush()
    return h


def _compare(h, ref_tables, ref_p, idx_of):
    """ref_tables: (D, C) reference disp_fn at 0..D-1 (NaN: not compared);
    ref_p: chrom -> reference p at idx_of[chrom] (None: every disp pixel)."""
    from hic3defdr_amd import _native
    from hic3defdr_amd.analysis.core import DispFn
    dpd = h.load_data('disp_per_dist')
    raw, f, dist, offs = h._f_and_dist()
    design = np.asarray(h.design, dtype=bool)
    cond = design.argmax(axis=1)
    D, C = dpd.shape
    ctx = h._ctx()
    xs = np.arange(D)
    out = {}
    for name, mode in MODES:
        tab = _native.disp_tables(dpd, weighted=mode)
        fit = np.stack([DispFn(tab[:, c], dpd[:, c],
                               weighted=bool(mode))(xs) for c in range(C)],
                       axis=1)
        present = np.isfinite(dpd) & (xs[:, None] >= h.dist_thresh_min)
        t_rel = []
        for c in range(C):
            m = present[:, c] & np.isfinite(ref_tables[:, c])
            t_rel.append(float(np.max(np.abs(fit[m, c] - ref_tables[m, c])
                                      / np.abs(ref_tables[m, c]))))
        p, _, _, _, _ = ctx.lrt(raw, f, dist, tab, cond, want_disp=False)
        got, want = [], []
        for i, chrom in enumerate(h.chroms):
            pc = p[offs[i]:offs[i + 1]]
            sel = idx_of.get(chrom)
            got.append(pc if sel is None else pc[sel])
            want.append(ref_p[chrom])
        got, want = np.concatenate(got), np.concatenate(want)
        rel = np.abs(got - want) / np.maximum(want, 1e-300)
        rel[got == want] = 0.0
        qg, qw = _native.bh(got), _native.bh(want)
        out[name] = {
            'tables_rel': t_rel,
            'conditions_within_1e-6': int(sum(r <= 1e-6 for r in t_rel)),
            'conditions': C,
            'p_compared': int(len(got)),
            'p_within_1e-6': int(np.sum(rel <= 1e-6)),
            'p_max_rel': float(rel.max()),
            'identical_calls_q<0.05': bool(np.array_equal(qg < 0.05,
                                                          qw < 0.05))}
    return out


def main():
    import torch  # noqa: F401  (one HIP runtime: torch's first)
    from conftest import e2e_inputs, golden
    from hic3defdr_amd import synthetic
    res = {}
    base = tempfile.mkdtemp(prefix='h3d_census_')
    try:
        for name in E2E:
            g, kw = e2e_inputs(name)
            h = _run(kw, os.path.join(base, name), kw['design'],
                     kw['loop_patterns'], 10000)
            D = kw['dist_thresh_max'] + 1
            tabs = np.stack([g['disp_fn_table__%s' % c] for c in kw['conds']],
                            axis=1)[:D]
            ref_p = {c: g['pvalues__%s' % c] for c in kw['chroms']}
            res[name] = _compare(h, tabs, ref_p, {})
            print(name, json.dumps(res[name]), file=sys.stderr, flush=True)
        mech = golden('lowess_mechanism.npz')
        for cfg, shape, gname in (('cfg1', {'chr18': 9070, 'chr19': 6143},
                                   'full_cfg1.npz'),
                                  ('cfg2', {'chrB0': 20000}, 'full_cfg2.npz')):
            g = golden(gname)
            dmax = int(g['meta_dmax'])
            d = os.path.join(base, cfg)
            kw = synthetic.write_dataset(d, shape, dist_thresh_max=dmax,
                                         seed=int(g['meta_seed']))
            kw['dist_thresh_max'] = dmax
            loops = kw['loop_patterns'] if cfg == 'cfg1' else None
            h = _run(kw, os.path.join(d, 'out'), kw['design'], loops,
                     10000 if loops else None)
            tabs = np.stack([mech['%s__0__%d__table' % (cfg, c)]
                             for c in range(2)], axis=1)
            if cfg == 'cfg1':
                ref_p = {c: g['p__%s' % c] for c in shape}
                idx = {c: g['sample_idx__%s' % c] for c in shape}
            else:
                c0 = list(shape)[0]
                ref_p = {c0: np.concatenate([g['p'], g['top_p']])}
                idx = {c0: np.concatenate([g['sample_idx'], g['top_idx']])}
            res[cfg] = _compare(h, tabs, ref_p, idx)
            print(cfg, json.dumps(res[cfg]), file=sys.stderr, flush=True)
            shutil.rmtree(d, ignore_errors=True)
    finally:
        shutil.rmtree(base, ignore_errors=True)
    tot = {}
    for name, _ in MODES:
        tot[name] = {
            'conditions_within_1e-6': sum(r[name]['conditions_within_1e-6']
                                          for r in res.values()),
            'conditions': sum(r[name]['conditions'] for r in res.values()),
            'p_within_1e-6': sum(r[name]['p_within_1e-6']
                                 for r in res.values()),
            'p_compared': sum(r[name]['p_compared'] for r in res.values()),
            'datasets_identical_calls': sum(
                r[name]['identical_calls_q<0.05'] for r in res.values())}
    print(json.dumps({'datasets': res, 'totals': tot,
                      'source': 'tools/smoother_census.py (the product\'s '
                                'disp_per_dist, both smoother modes, the '
                                'product LRT; the reference goldens)'},
                     indent=1))


if __name__ == '__main__':
    main()
