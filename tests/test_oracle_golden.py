"""Pins the CPU oracle (oracle/) to vectors produced by the reference itself
(tests/golden/make_golden.py) and to the reference's own doctests."""
import numpy as np
import pandas as pd
import pytest

import oracle
from oracle.lowess_sm import lowess as sm_lowess
from conftest import golden, e2e_inputs, rel_err


# -- reference doctests restated ------------------------------------------

def test_fit_mu_hat_doctests():
    """hic3defdr/util/scaled_nb.py:97-137."""
    x = np.array([[1, 2], [3, 4], [5, 6]])
    b = np.array([[0.9, 1.1], [0.8, 1.2], [0.7, 1.3]])
    alpha = np.array([[0.1, 0.2], [0.3, 0.4], [0.5, 0.6]])
    np.testing.assert_allclose(oracle.fit_mu_hat(x, b, alpha),
                               [1.47251127, 3.53879843, 5.86853465], rtol=1e-8)
    np.testing.assert_allclose(oracle.fit_mu_hat(x, b, np.array([0.1, 0.2])),
                               [1.47251127, 3.53749833, 5.85554075], rtol=1e-8)
    np.testing.assert_allclose(
        oracle.fit_mu_hat(x, b, np.array([0.1, 0.2, 0.3])[:, None]),
        [1.49544092, 3.51679438, 5.73129492], rtol=1e-8)
    x = np.array([[2, 3, 4, 2], [6, 9, 3, 1]])
    b = np.array([[0.45, 0.53, 0.088, 0.091], [0.70, 0.83, 0.14, 0.15]])
    alpha = np.array([[0.0071, 0.0071, 0.0073, 0.0073],
                      [0.0070, 0.0070, 0.0072, 0.0072]])
    np.testing.assert_allclose(oracle.fit_mu_hat(x, b, alpha),
                               [9.5900971, 10.45962955], rtol=1e-8)


def test_conditional_mor_doctest():
    """docs/median_of_ratios.rst:7-32 (also pins gmean pseudocount=1)."""
    data = np.arange(20, dtype=float).reshape((5, 4))
    dist = np.array([1, 1, 1, 2, 2])
    exp = np.array([[0.79394639, 0.93946738, 1.08498836, 1.23050934]] * 3 +
                   [[0.90390183, 0.96968472, 1.0354676, 1.10125049]] * 2)
    np.testing.assert_allclose(oracle.conditional_mor(data, dist), exp,
                               rtol=1e-8)


def test_sparse_union_doctest():
    """docs/sparse_union.rst:36-105."""
    import scipy.sparse as sparse
    rep1 = np.array([[0., 0., 3., 1.], [0., 6., 5., 0.], [0., 0., 0., 2.],
                     [0., 0., 0., 7.]])
    rep2 = np.array([[0., 1., 3., 2.], [0., 0., 0., 0.], [0., 0., 4., 2.],
                     [0., 0., 0., 3.]])
    mats = [sparse.csr_matrix(rep1), sparse.csr_matrix(rep2)]
    row, col = oracle.sparse_union(mats, dist_thresh=2)
    assert list(zip(row, col)) == [(0, 1), (0, 2), (1, 1), (1, 2), (2, 2),
                                   (2, 3), (3, 3)]
    data = np.zeros((len(row), 2))
    for i in range(2):
        data[:, i] = mats[i].tocsr()[row, col]
    np.testing.assert_array_equal(
        data, [[0, 1], [3, 3], [6, 0], [5, 0], [0, 4], [2, 2], [7, 3]])


# -- unit goldens ---------------------------------------------------------

def test_unit_nb_fit_mu_hat():
    g = golden('unit_nb.npz')
    mu = oracle.fit_mu_hat(g['fmh_x'], g['fmh_b'], g['fmh_alpha'])
    assert rel_err(mu, g['fmh_mu']) < 1e-9
    mu = oracle.fit_mu_hat(g['fmh_x'], g['fmh_b'], 0.05)
    assert rel_err(mu, g['fmh_mu_scalar_alpha']) < 1e-9


def test_unit_nb_q2q():
    g = golden('unit_nb.npz')
    out = oracle.q2qnbinom(g['q2q_x'], g['q2q_mu_in'].copy(),
                           g['q2q_mu_out'].copy(), g['q2q_alpha'])
    assert rel_err(out, g['q2q']) < 1e-10


def test_unit_nb_segments():
    g = golden('unit_nb.npz')
    for s in range(int(g['n_segs'])):
        data, f = g['seg%d_data' % s], g['seg%d_f' % s]
        assert rel_err(oracle.equalize(data, f, 0.02),
                       g['seg%d_equalize' % s]) < 1e-10
        # Brent (xatol 1e-5) on a flat NLL: agree to 1e-7 rel + 1e-10 abs
        np.testing.assert_allclose(oracle.cml(data.astype(float) / f),
                                   g['seg%d_cml' % s], rtol=1e-7, atol=1e-10)
        np.testing.assert_allclose(oracle.qcml(data, f=f), g['seg%d_qcml' % s],
                                   rtol=1e-7, atol=1e-10)
        assert rel_err(oracle.mme(data.astype(float), f=f),
                       g['seg%d_mme' % s]) < 1e-12


def test_unit_nb_logpmf_lrt():
    g = golden('unit_nb.npz')
    assert rel_err(oracle.logpmf(g['lp_k'], g['lp_m'], g['lp_phi']),
                   g['logpmf']) < 1e-12
    for pre, refit in (('lrt', True), ('lrtnr', False)):
        p, llr, m0, m1 = oracle.lrt(g['lrt_raw'], g['lrt_f'], g['lrt_disp'],
                                    g['lrt_design'], refit_mu=refit)
        assert rel_err(p, g[pre + '_p']) < 1e-7
        assert rel_err(m0, g[pre + '_mu0']) < 1e-9
        assert rel_err(m1, g[pre + '_mu1']) < 1e-9


def test_unit_lowess():
    g = golden('unit_lowess.npz')
    for t in range(6):
        r = sm_lowess(g['lo%d_y' % t], g['lo%d_x' % t],
                      frac=float(g['lo%d_frac' % t]),
                      delta=float(g['lo%d_delta' % t]))
        # bit-exact where x has no ties; ties are ordered by an unstable sort
        # in statsmodels, which only permutes summation order
        assert np.max(np.abs(r - g['lo%d_res' % t])) < 1e-12
        x, y = g['wl%d_x' % t], g['wl%d_y' % t]
        var = pd.Series(y).rolling(window=20, center=True).var().values
        np.testing.assert_array_equal(var, g['wl%d_rollvar' % t])
        fn = oracle.weighted_lowess_fit(x, y, left_boundary=y[0])
        tab = fn(np.arange(len(g['wl%d_table' % t])))
        assert rel_err(tab, g['wl%d_table' % t]) < 1e-12
        fn2 = oracle.lowess_fit(x, y, left_boundary=y[0])
        assert rel_err(fn2(np.arange(len(tab))), g['ul%d_table' % t]) < 1e-12


def test_unit_scaling():
    g = golden('unit_scaling.npz')
    for t in range(4):
        data, dist = g['cm%d_data' % t], g['cm%d_dist' % t]
        nb = int(g['cm%d_nbins' % t])
        np.testing.assert_array_equal(oracle.equal_bin(dist, nb),
                                      g['cm%d_eqbin' % t])
        assert rel_err(oracle.conditional_mor(data, dist, n_bins=nb),
                       g['cm%d_sf' % t]) < 1e-13
        assert rel_err(oracle.conditional_mor(data, dist),
                       g['cm%d_sf_exact' % t]) < 1e-13


def test_unit_special():
    import scipy.special as sc
    g = golden('unit_special.npz')
    a, x, p = g['a'], g['x'], g['p']
    assert rel_err(sc.gammainc(a, x), g['gammainc']) < 1e-12
    assert rel_err(sc.gammaincc(a, x), g['gammaincc']) < 1e-12
    assert rel_err(sc.gammaincinv(a, p), g['gammaincinv']) < 1e-11
    assert rel_err(sc.gammainccinv(a, p), g['gammainccinv']) < 1e-11
    assert rel_err(sc.ndtr(g['z']), g['ndtr']) < 1e-13
    assert rel_err(sc.ndtri(g['pq']), g['ndtri']) < 1e-13
    assert rel_err(sc.gammaln(g['g']), g['gammaln']) < 1e-14


# -- end to end -------------------------------------------------------------

FLOOR_DROP = {'r16c2', 'lwdrop'}


@pytest.mark.parametrize('name', ['small2', 'c3r9', 'r18c3', 'r16c2',
                                  'lwdrop'])
def test_e2e_oracle_matches_reference(name):
    g, kw = e2e_inputs(name)
    chroms = kw['chroms']
    npz = {c: [p.replace('<chrom>', c) for p in kw['raw_npz_patterns']]
           for c in chroms}
    bias = {c: [p.replace('<chrom>', c) for p in kw['bias_patterns']]
            for c in chroms}
    loops = None
    if kw['loop_patterns']:
        loops = {c: [p.replace('<chrom>', c)
                     for p in kw['loop_patterns'].values()] for c in chroms}
    out = oracle.run_to_qvalues(npz, bias, chroms, kw['design'],
                                dist_thresh_max=kw['dist_thresh_max'],
                                loop_files=loops)
    assert rel_err(out['disp_per_dist'], g['disp_per_dist']) < 1e-6
    drop = name in FLOOR_DROP
    for c in chroms:
        for st in ('row', 'col', 'raw', 'disp_idx'):
            np.testing.assert_array_equal(out[c][st], g['%s__%s' % (st, c)])
        if loops:
            np.testing.assert_array_equal(out[c]['loop_idx'],
                                          g['loop_idx__%s' % c])
        assert rel_err(out[c]['size_factors'],
                       g['size_factors__%s' % c]) < 1e-12
        assert rel_err(out[c]['scaled'], g['scaled__%s' % c]) < 1e-12
        if drop:
            # the reference's lowess dropped a distance here (floor of a
            # scaled weight, lowess.py:183-201); the oracle pins the intended
            # weight 1: measured bound, no call flips
            q, qr = out[c]['qvalues'], g['qvalues__%s' % c]
            assert np.nanmax(np.abs(q - qr)) < 0.02
            for fdr in (0.01, 0.05):
                np.testing.assert_array_equal(q < fdr, qr < fdr)
            continue
        assert rel_err(out[c]['disp'], g['disp__%s' % c]) < 1e-6
        assert rel_err(out[c]['pvalues'], g['pvalues__%s' % c]) < 1e-6
        assert rel_err(out[c]['qvalues'], g['qvalues__%s' % c]) < 1e-6
        assert rel_err(out[c]['mu_hat_null'], g['mu_hat_null__%s' % c]) < 1e-8
        assert rel_err(out[c]['mu_hat_alt'], g['mu_hat_alt__%s' % c]) < 1e-8


def test_oracle_lrt_on_cfg2_secant_failures():
    """The CPU restatement (fallback-fixed brentq) on the headline workload's
    secant-failure pixels vs the reference's lrt on them (hard_cfg2.npz)."""
    g = golden('hard_cfg2.npz')
    design = g['design'].astype(bool)
    p, llr, m0, m1 = oracle.lrt(g['raw'], g['f'],
                                np.dot(g['disp'], design.T), design)
    assert rel_err(p, g['p']) < 1e-6
    assert rel_err(m0, g['mu0']) < 1e-8
    assert rel_err(m1, g['mu1']) < 1e-8


@pytest.mark.parametrize('name,cond', [('r16c2', 'ES'), ('r16c2', 'NPC'),
                                       ('lwdrop', 'ES')])
def test_lowess_floor_drop_mechanism(name, cond):
    """Where the reference's table differs from the pinned one, the
    reference-faithful weight arithmetic (intended_min_weight=False) on the
    reference's own disp_per_dist reproduces it: the difference is exactly
    the floor(w * (1/min_w)) drop of lowess.py:183-201."""
    g = golden('e2e_%s.npz' % name)
    c = [str(x) for x in g['meta_conds']].index(cond)
    col = g['disp_per_dist'][:, c]
    fin = np.isfinite(col)
    x, y = np.arange(len(col))[fin], col[fin]
    ref = g['disp_fn_table__%s' % cond]
    xs = np.arange(len(col))
    faithful = oracle.weighted_lowess_fit(x, y, left_boundary=y[0],
                                          intended_min_weight=False)(xs)
    pinned = oracle.weighted_lowess_fit(x, y, left_boundary=y[0])(xs)
    assert rel_err(faithful, ref) < 1e-12
    assert rel_err(pinned, ref) > 1e-3
