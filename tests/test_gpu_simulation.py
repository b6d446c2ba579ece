"""The reference's simulation workflow (README.md:541-699) end to end on the
product: the GPU analysis of small2 -> simulate('ES') with the reference's
seed -> filter_sparse_rows_count + kr_balance -> a GPU analysis of the
simulated replicates -> evaluate(), against the reference doing the same
(tests/golden/sim_small2.npz)."""
import os
import shutil
import tempfile

import numpy as np
import pandas as pd
import pytest
import scipy.sparse as sparse

from conftest import e2e_inputs, golden, rel_err

pytestmark = pytest.mark.gpu
SIMREPS = ['A1', 'A2', 'B1', 'B2']


def test_simulate_balance_analyse_evaluate_matches_reference():
    from hic3defdr_amd import HiC3DeFDR
    from hic3defdr_amd.util.balancing import kr_balance
    from hic3defdr_amd.util.filtering import filter_sparse_rows_count
    g = golden('sim_small2.npz')
    _, kw = e2e_inputs('small2')
    tmp = tempfile.mkdtemp(prefix='h3d_gsim_')
    try:
        design = pd.DataFrame(kw['design'], index=kw['reps'],
                              columns=kw['conds'])
        h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                      bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                      design=design, outdir=os.path.join(tmp, 'out'),
                      dist_thresh_max=kw['dist_thresh_max'],
                      loop_patterns=kw['loop_patterns'])
        h.run_to_qvalues(verbose=False)
        sim = os.path.join(tmp, 'sim')
        np.random.seed(int(g['meta_seed']))
        h.simulate('ES', outdir=sim, verbose=False)
        for c in kw['chroms']:
            np.testing.assert_array_equal(
                np.loadtxt(os.path.join(sim, 'labels_%s.txt' % c), dtype='U7'),
                g['labels__%s' % c])
            for rep in SIMREPS:
                fn = os.path.join(sim, '%s_%s_raw.npz' % (rep, c))
                m = sparse.load_npz(fn).tocsr()
                np.testing.assert_array_equal(
                    m.data, g['sim__%s__%s__data' % (rep, c)])
                np.testing.assert_array_equal(
                    m.indices, g['sim__%s__%s__indices' % (rep, c)])
                _, bias, _ = kr_balance(filter_sparse_rows_count(m), fl=0)
                np.savetxt(fn.replace('_raw.npz', '_kr.bias'), bias)
        hs = HiC3DeFDR(
            raw_npz_patterns=[os.path.join(sim, '%s_<chrom>_raw.npz' % r)
                              for r in SIMREPS],
            bias_patterns=[os.path.join(sim, '%s_<chrom>_kr.bias' % r)
                           for r in SIMREPS],
            chroms=kw['chroms'], design=os.path.join(sim, 'design.csv'),
            outdir=os.path.join(tmp, 'simout'),
            dist_thresh_max=kw['dist_thresh_max'],
            loop_patterns={'ES': kw['loop_patterns']['ES']})
        hs.run_to_qvalues(verbose=False)
        assert rel_err(np.load(os.path.join(tmp, 'simout',
                                            'disp_per_dist.npy')),
                       g['simrun__disp_per_dist']) < 1e-6
        for c in kw['chroms']:
            for st, tol in (('pvalues', 1e-6), ('qvalues', 1e-6)):
                got = np.load(os.path.join(tmp, 'simout', '%s_%s.npy' % (st, c)))
                assert rel_err(got, g['simrun__%s__%s' % (st, c)]) < tol, st
        for a, b, rr in g['meta_evals']:
            a = None if a < 0 else int(a)
            b = None if b < 0 else int(b)
            hs.evaluate('ES', os.path.join(sim, 'labels_<chrom>.txt'),
                        min_dist=a, max_dist=b, rerun_bh=bool(rr))
            fn = 'eval' if a is None and b is None else 'eval_%s_%s' % (a, b)
            e = np.load(os.path.join(tmp, 'simout', fn + '.npz'))
            for k in ('fpr', 'tpr'):
                np.testing.assert_array_equal(e[k], g['eval__%s__%s' % (fn, k)])
            np.testing.assert_array_equal(np.isnan(e['fdr']),
                                          np.isnan(g['eval__%s__fdr' % fn]))
            assert rel_err(e['fdr'], g['eval__%s__fdr' % fn]) < 1e-12
            # thresholds are 1 - q: absolute q agreement
            assert np.max(np.abs(e['thresh'] - g['eval__%s__thresh' % fn])) \
                < 1e-6
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
