"""The reference's own spread on the headline chromosome (CPU): its results
under six pixel orders of its input (tests/golden/cfg2_spread.npz, made by
make_golden.py run_cfg2_spread from the reference itself), which
test_gpu_scale.py's end-to-end bars are measured against."""
import numpy as np

from conftest import golden, rel_err


def _reference_orders():
    sp = golden('cfg2_spread.npz')
    return [{key: sp['%s__%d' % (key, k)] for key in (
        'disp_per_dist', 'p_sample', 'p_top', 'q_sample', 'q_top',
        'calls_0.01', 'calls_0.05', 'calls_0.1')} for k in sp['perms']]


def rel_err_arr(a, b):
    return np.abs(a - b) / np.abs(b)


def test_reference_order_spread_fixture():
    """What the reference itself does under a pixel-order permutation (the
    NLL of cml is a sum over pixels, dispersion.py:74-75; only np.sum's
    rounding sees the order): the same call sets, segment dispersions that
    move by up to 8.9e-5 (one bounded-Brent search taking the other side of
    a near-tie), and end-to-end p-values that move by up to 1.4e-3 (sample)
    / 1.4e-2 (top) -- the weighted lowess floors its weights
    (lowess.py:170-190), so a 1e-8 change of disp_per_dist can add or drop
    an expanded point. Pinned here so the bars below stay honest."""
    orders = _reference_orders()
    g = golden('full_cfg2.npz')
    np.testing.assert_array_equal(orders[0]['disp_per_dist'],
                                  g['disp_per_dist'])
    np.testing.assert_array_equal(orders[0]['p_sample'], g['p'])
    fin = np.isfinite(g['disp_per_dist'])
    seg = max(np.max(rel_err_arr(o['disp_per_dist'][fin],
                                 g['disp_per_dist'][fin])) for o in orders)
    p_spread = max(rel_err(o['p_sample'], g['p']) for o in orders)
    assert 5e-5 < seg < 2e-4 and 1e-4 < p_spread < 1e-2
    for o in orders:
        for fdr in (0.01, 0.05, 0.1):
            np.testing.assert_array_equal(o['calls_%g' % fdr],
                                          g['calls_%g' % fdr])


def test_cfg1_reference_order_spread_fixture():
    """The same on the cfg1 genome (two chromosomes, loop-pixel BH;
    cfg1_spread.npz, make_golden.py run_cfg1_spread): orders 1..5 of the
    reference's segments against its order 0 (full_cfg1.npz) move the
    sampled p-values by 1e-9 .. 4.3e-3 -- again the reference's own spread
    that test_gpu_cfg1.py's end-to-end bar is measured against."""
    g = golden('full_cfg1.npz')
    sp = golden('cfg1_spread.npz')
    chroms = [str(c) for c in g['meta_chroms']]
    spread = [max(rel_err(sp['p__%s__%d' % (c, k)], g['p__%s' % c])
                  for c in chroms) for k in sp['perms'][1:]]
    assert min(spread) < 1e-7 and 1e-4 < max(spread) < 1e-2, spread
    for k in sp['perms'][1:]:
        for c in chroms:
            assert sp['q__%s__%d' % (c, k)].shape == g['q__%s' % c].shape
