"""Every size-factor method prepare_data dispatches (util/scaling.py:10-149,
analysis/analysis.py:104-108) on the GPU, through the product's
run_to_qvalues(norm=...), vs the reference run on the same inputs
(tests/golden/norm_small2.npz). The per-replicate (1-D) methods exercise the
LRT's 1-D size-factor branch (analysis.py:274-275); their estimate_disp uses
the broadcast the reference's lrt uses (the reference's own estimate_disp
indexes a 1-D array with the pixel mask and raises, analysis.py:181 -- the
fixture pins the evident intent, see make_golden.py _PerRepFactors)."""
import os
import shutil
import tempfile

import numpy as np
import pandas as pd
import pytest

from conftest import e2e_inputs, golden, rel_err

NORMS = ['conditional_scaling', 'median_of_ratios', 'simple_scaling',
         'no_scaling']


@pytest.mark.gpu
@pytest.mark.parametrize('norm', NORMS)
def test_run_to_qvalues_norm_matches_reference(norm):
    from hic3defdr_amd import HiC3DeFDR
    g0, kw = e2e_inputs('small2')
    g = golden('norm_small2.npz')
    outdir = tempfile.mkdtemp(prefix='h3d_norm_')
    try:
        design = pd.DataFrame(kw['design'], index=kw['reps'],
                              columns=kw['conds'])
        h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                      bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                      design=design, outdir=outdir,
                      dist_thresh_max=kw['dist_thresh_max'],
                      loop_patterns=kw['loop_patterns'])
        h.run_to_qvalues(norm=norm, verbose=False)
        dpd = np.load(os.path.join(outdir, 'disp_per_dist.npy'))
        ref = g['%s__disp_per_dist' % norm]
        np.testing.assert_array_equal(np.isnan(dpd), np.isnan(ref))
        np.testing.assert_allclose(dpd, ref, rtol=1e-6, atol=1e-12)
        for c in kw['chroms']:
            def ld(st):
                return np.load(os.path.join(outdir, '%s_%s.npy' % (st, c)))
            sf = ld('size_factors')
            rsf = g['%s__size_factors__%s' % (norm, c)]
            assert sf.shape == rsf.shape
            assert rel_err(sf, rsf) < 1e-13
            np.testing.assert_array_equal(ld('disp_idx'),
                                          g['%s__disp_idx__%s' % (norm, c)])
            np.testing.assert_array_equal(ld('loop_idx'),
                                          g['%s__loop_idx__%s' % (norm, c)])
            for st, tol in (('disp', 1e-6), ('pvalues', 1e-6),
                            ('qvalues', 1e-6), ('mu_hat_null', 1e-8),
                            ('mu_hat_alt', 1e-8)):
                assert rel_err(ld(st), g['%s__%s__%s' % (norm, st, c)]) < tol, st
            for fdr in (0.01, 0.05, 0.1):
                np.testing.assert_array_equal(
                    ld('qvalues') < fdr, g['%s__qvalues__%s' % (norm, c)] < fdr)
    finally:
        shutil.rmtree(outdir, ignore_errors=True)


@pytest.mark.gpu
def test_size_factor_kernels_exact_distance_and_oracle():
    """conditional_scaling with exact distances (n_bins=0) and the global
    methods vs the CPU restatement on the same balanced matrix."""
    import oracle
    from hic3defdr_amd import _native
    ctx = _native.context(0)
    rng = np.random.default_rng(4)
    n, R = 20000, 6
    dist = rng.integers(0, 90, n).astype(np.int32)
    bal = np.exp(rng.normal(1, 1, (n, R))) * (rng.random((n, R)) > 0.05)
    assert rel_err(ctx.size_factors(bal, dist, 'conditional_scaling', 0),
                   oracle.conditional_scaling(bal, dist)) < 1e-13
    assert rel_err(ctx.size_factors(bal, dist, 'conditional_scaling', 17),
                   oracle.conditional_scaling(bal, dist, n_bins=17)) < 1e-13
    assert rel_err(ctx.size_factors(bal, None, 'median_of_ratios'),
                   oracle.median_of_ratios(bal)) < 1e-13
    assert rel_err(ctx.size_factors(bal, None, 'simple_scaling'),
                   oracle.simple_scaling(bal)) < 1e-13
    np.testing.assert_array_equal(ctx.size_factors(bal, None, 'no_scaling'),
                                  np.ones(R))


def test_oracle_norms_vs_reference():
    """The CPU restatement of every norm on the reference's balanced matrix
    (reconstructed from the committed inputs) vs the reference's factors."""
    import oracle
    g0, kw = e2e_inputs('small2')
    g = golden('norm_small2.npz')
    for c in kw['chroms']:
        npz = [p.replace('<chrom>', c) for p in kw['raw_npz_patterns']]
        bfs = [p.replace('<chrom>', c) for p in kw['bias_patterns']]
        prep = oracle.prepare_chrom(npz, bfs, kw['design'],
                                    dist_thresh_max=kw['dist_thresh_max'])
        bal = prep['raw'] / (oracle.load_bias(bfs)[prep['row']] *
                             oracle.load_bias(bfs)[prep['col']])
        dist = prep['col'] - prep['row']
        nb = int(kw['dist_thresh_max'] / 5)
        got = {'conditional_scaling': oracle.conditional_scaling(bal, dist,
                                                                 n_bins=nb),
               'median_of_ratios': oracle.median_of_ratios(bal),
               'simple_scaling': oracle.simple_scaling(bal),
               'no_scaling': oracle.no_scaling(bal)}
        for norm in NORMS:
            assert rel_err(got[norm], g['%s__size_factors__%s' % (norm, c)]) \
                < 1e-13, norm
