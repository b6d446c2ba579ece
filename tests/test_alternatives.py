"""Alternative models (reference analysis/alternatives.py, SURVEY.md §8(f)
#4) vs the reference's own outputs (tests/golden/alt_small2.npz, written by
tests/golden/make_golden.py running the reference): the oracle restatement on
the CPU, the product classes (Poisson / MME / one-segment qcml kernels) on the
GPU.

Parity bar: p / q within 1e-6 relative (north star), closed-form Poisson means
and MME dispersions to ~1e-13, loop_idx bit-exact, identical calls."""
import os
import shutil
import tempfile

import numpy as np
import pandas as pd
import pytest

import oracle
from conftest import e2e_inputs, golden, rel_err

CLASSES = ['Poisson3DeFDR', 'Unsmoothed3DeFDR', 'Global3DeFDR']


def _inputs(g, kw, chrom):
    bias = oracle.load_bias([p.replace('<chrom>', chrom)
                             for p in kw['bias_patterns']])
    di = g['disp_idx__%s' % chrom]
    row, col = g['row__%s' % chrom][di], g['col__%s' % chrom][di]
    f = bias[row] * bias[col] * g['size_factors__%s' % chrom][di]
    return g['raw__%s' % chrom][di], f, g['scaled__%s' % chrom][di]


def test_oracle_poisson_lrt_vs_reference():
    g, kw = e2e_inputs('small2')
    alt = golden('alt_small2.npz')
    for c in kw['chroms']:
        raw, f, _ = _inputs(g, kw, c)
        p, llr, m0, m1 = oracle.poisson_lrt(raw, f, kw['design'])
        assert rel_err(p, alt['Poisson3DeFDR__pvalues__%s' % c]) < 1e-12
        assert rel_err(llr, alt['Poisson3DeFDR__llr__%s' % c]) < 1e-12
        assert rel_err(m0, alt['Poisson3DeFDR__mu_hat_null__%s' % c]) < 1e-15
        assert rel_err(m1, alt['Poisson3DeFDR__mu_hat_alt__%s' % c]) < 1e-15


def test_oracle_mme_per_pixel_vs_reference():
    g, kw = e2e_inputs('small2')
    alt = golden('alt_small2.npz')
    design = kw['design']
    for c in kw['chroms']:
        _, _, scaled = _inputs(g, kw, c)
        disp = np.stack([np.maximum(oracle.mme_per_pixel(scaled[:, design[:, k]]),
                                    1e-7) for k in range(design.shape[1])], 1)
        assert rel_err(disp, alt['Unsmoothed3DeFDR__disp__%s' % c]) < 1e-15


@pytest.mark.gpu
@pytest.mark.parametrize('cls', CLASSES)
def test_alternative_run_to_qvalues_matches_reference(cls):
    from hic3defdr_amd.analysis import alternatives
    g, kw = e2e_inputs('small2')
    alt = golden('alt_small2.npz')
    outdir = tempfile.mkdtemp(prefix='h3d_alt_')
    try:
        design = pd.DataFrame(kw['design'], index=kw['reps'],
                              columns=kw['conds'])
        h = getattr(alternatives, cls)(
            raw_npz_patterns=kw['raw_npz_patterns'],
            bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
            design=design, outdir=outdir,
            dist_thresh_max=kw['dist_thresh_max'],
            loop_patterns=kw['loop_patterns'])
        h.run_to_qvalues(verbose=False)
        # Global: Brent on one pooled segment (qcml tolerance). Unsmoothed:
        # (var - mean) / mean^2 of the product's own scaled values, whose
        # ~1e-13 size-factor differences the var - mean cancellation
        # amplifies (measured 2.3e-12). Poisson: zeros.
        tol_disp = {'Global3DeFDR': 1e-6, 'Unsmoothed3DeFDR': 1e-9,
                    'Poisson3DeFDR': 1e-13}[cls]
        for c in kw['chroms']:
            def ld(st):
                return np.load(os.path.join(outdir, '%s_%s.npy' % (st, c)))
            ref = lambda st: alt['%s__%s__%s' % (cls, st, c)]  # noqa: E731
            np.testing.assert_array_equal(ld('loop_idx'), ref('loop_idx'))
            assert rel_err(ld('disp'), ref('disp')) < tol_disp
            if cls == 'Unsmoothed3DeFDR':
                # pixels floored at disp = 1e-7 (r = 1e7): logpmf's
                # lgamma(r + k) - lgamma(r) cancels ~1e8-sized terms, so llr
                # carries ~1e-8 absolute rounding in ANY implementation, and
                # p = chi2(1).sf(-2 llr) has an infinite slope at llr -> 0.
                # There: llr to 1e-6 absolute; elsewhere the 1e-6 p bar.
                ok = ref('disp').min(axis=1) > 1e-6
                assert np.max(np.abs(ld('llr') - ref('llr'))) < 1e-6
                assert rel_err(ld('pvalues')[ok], ref('pvalues')[ok]) < 1e-6
            else:
                assert rel_err(ld('pvalues'), ref('pvalues')) < 1e-6
                assert rel_err(ld('qvalues'), ref('qvalues')) < 1e-6
            assert rel_err(ld('mu_hat_null'), ref('mu_hat_null')) < 1e-8
            assert rel_err(ld('mu_hat_alt'), ref('mu_hat_alt')) < 1e-8
            for fdr in (0.01, 0.05, 0.1):
                np.testing.assert_array_equal(ld('qvalues') < fdr,
                                              ref('qvalues') < fdr)
        key = '%s__disp_per_dist' % cls
        if key in alt.files:
            dpd = np.load(os.path.join(outdir, 'disp_per_dist.npy'))
            assert rel_err(dpd, alt[key]) < tol_disp
    finally:
        shutil.rmtree(outdir, ignore_errors=True)


@pytest.mark.gpu
def test_poisson_lrt_refit_false_raises_like_reference():
    from hic3defdr_amd.analysis.alternatives import poisson_lrt
    with pytest.raises(ValueError):
        poisson_lrt(np.ones((3, 4), dtype=np.int64), np.ones((3, 4)),
                    np.array([[1, 0], [1, 0], [0, 1], [0, 1]], dtype=bool),
                    refit_mu=False)
