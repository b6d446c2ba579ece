"""End to end on the GPU: the product HiC3DeFDR.run_to_qvalues() on the
reference's inputs vs every outdir array the reference wrote (goldens)."""
import os
import pickle
import shutil
import tempfile

import numpy as np
import pandas as pd
import pytest

from conftest import e2e_inputs, golden, rel_err

pytestmark = pytest.mark.gpu


def _run(name, outdir):
    from hic3defdr_amd import HiC3DeFDR
    g, kw = e2e_inputs(name)
    design = pd.DataFrame(kw['design'], index=kw['reps'], columns=kw['conds'])
    h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                  bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                  design=design, outdir=outdir,
                  dist_thresh_max=kw['dist_thresh_max'],
                  loop_patterns=kw['loop_patterns'], res=10000)
    h.run_to_qvalues(verbose=False)
    return g, kw, h


@pytest.mark.parametrize('name', ['small2', 'c3r9'])
def test_run_to_qvalues_matches_reference(name):
    outdir = tempfile.mkdtemp(prefix='h3d_e2e_')
    try:
        g, kw, h = _run(name, outdir)
        dpd = np.load(os.path.join(outdir, 'disp_per_dist.npy'))
        np.testing.assert_array_equal(np.isnan(dpd), np.isnan(g['disp_per_dist']))
        np.testing.assert_allclose(dpd, g['disp_per_dist'], rtol=1e-6, atol=1e-12)
        for c in kw['chroms']:
            ld = lambda st: np.load(os.path.join(outdir, '%s_%s.npy' % (st, c)))
            for st in ('row', 'col', 'raw', 'disp_idx'):   # bit-exact
                a = ld(st)
                assert a.dtype == g['%s__%s' % (st, c)].dtype, st
                np.testing.assert_array_equal(a, g['%s__%s' % (st, c)])
            if kw['loop_patterns']:
                np.testing.assert_array_equal(ld('loop_idx'), g['loop_idx__%s' % c])
            assert rel_err(ld('size_factors'), g['size_factors__%s' % c]) < 1e-13
            assert rel_err(ld('scaled'), g['scaled__%s' % c]) < 1e-13
            assert rel_err(ld('disp'), g['disp__%s' % c]) < 1e-6
            assert rel_err(ld('pvalues'), g['pvalues__%s' % c]) < 1e-6
            assert rel_err(ld('qvalues'), g['qvalues__%s' % c]) < 1e-6
            assert rel_err(ld('mu_hat_null'), g['mu_hat_null__%s' % c]) < 1e-8
            assert rel_err(ld('mu_hat_alt'), g['mu_hat_alt__%s' % c]) < 1e-8
            # identical calls at the usual FDR thresholds
            for fdr in (0.01, 0.05, 0.1):
                np.testing.assert_array_equal(ld('qvalues') < fdr,
                                              g['qvalues__%s' % c] < fdr)
        # persistence contract: load() and the pickled disp_fn
        from hic3defdr_amd import HiC3DeFDR
        h2 = HiC3DeFDR.load(outdir)
        assert h2.chroms == kw['chroms']
        xs = g['disp_fn_xs']
        for cond in kw['conds']:
            fn = h2.load_disp_fn(cond)
            assert rel_err(fn(xs), g['disp_fn_cont__%s' % cond]) < 1e-6
        q_all, off = h2.load_data('qvalues', 'all')
        assert off[-1] == len(q_all)
        r, cc, v = h2.load_data('qvalues', kw['chroms'][0], coo=True)
        assert len(r) == len(cc) == len(v)
        # downstream calls on the GPU q-values: same clusters, same tables
        # as the reference (threshold -> classify -> collect)
        from test_calls import assert_calls_match
        ref = golden('calls_%s.npz' % name)
        h2.collect(fdr=[float(x) for x in ref['meta_fdrs']],
                   cluster_size=[int(x) for x in ref['meta_sizes']])
        assert_calls_match(outdir, name)
    finally:
        shutil.rmtree(outdir, ignore_errors=True)
