"""CPU checks of the C ABI: libh3d.so builds for gfx950, loads without a GPU,
exports every symbol include/h3d.h declares, and its host-side entry points
(the lowess smoother table and BH) match the oracle / reference goldens."""
import os
import re

import numpy as np
import pytest

import oracle
from conftest import REPO, golden, e2e_inputs, rel_err

from hic3defdr_amd import build as h3dbuild
from hic3defdr_amd import _native


@pytest.fixture(scope='module')
def lib():
    h3dbuild.build_native()
    return _native.load_library()


def declared_symbols():
    src = open(os.path.join(REPO, 'include', 'h3d.h')).read()
    return sorted(set(re.findall(r'\b(h3d_[a-z_]+)\s*\(', src)))


def test_exports_every_declared_symbol(lib):
    names = declared_symbols()
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(_native.EXPORTS)


def test_no_device_is_reported_not_faked(lib):
    if lib.h3d_device_count() > 0:
        pytest.skip('a GPU is visible')
    assert lib.h3d_open(0) is None
    with pytest.raises(_native.H3DError):
        _native.Context(0)


def test_disp_table_matches_reference_lowess_goldens(lib):
    g = golden('unit_lowess.npz')
    for t in range(6):
        x, y = g['wl%d_x' % t], g['wl%d_y' % t]
        D = len(g['wl%d_table' % t])
        col = np.full(D, np.nan)
        col[x] = y
        tab = _native.disp_table(col, weighted=True)
        assert rel_err(tab, g['wl%d_table' % t]) < 1e-12
        tab2 = _native.disp_table(col, weighted=False)
        assert rel_err(tab2, g['ul%d_table' % t]) < 1e-12


@pytest.mark.parametrize('name', ['small2', 'c3r9', 'r18c3'])
def test_disp_table_matches_e2e_disp_fn(lib, name):
    g, kw = e2e_inputs(name)
    for c, cond in enumerate(kw['conds']):
        tab = _native.disp_table(g['disp_per_dist'][:, c])
        assert rel_err(tab, g['disp_fn_table__%s' % cond]) < 1e-12


@pytest.mark.parametrize('name', ['small2', 'c3r9', 'r18c3'])
def test_disp_tables_all_conditions_in_one_call(lib, name):
    """h3d_disp_tables (conditions on concurrent host threads) = one
    h3d_disp_table per condition, bit for bit, and = the reference's disp_fn
    tables; a degenerate column's error names its condition."""
    g, kw = e2e_inputs(name)
    dpd = g['disp_per_dist']
    tabs = _native.disp_tables(dpd)
    for c, cond in enumerate(kw['conds']):
        np.testing.assert_array_equal(tabs[:, c],
                                      _native.disp_table(dpd[:, c]))
        assert rel_err(tabs[:, c], g['disp_fn_table__%s' % cond]) < 1e-12
    bad = dpd.copy()
    bad[:, -1] = np.nan
    with pytest.raises(_native.H3DError, match='condition %d' % (
            dpd.shape[1] - 1)):
        _native.disp_tables(bad)


@pytest.mark.parametrize('name', ['small2', 'c3r9', 'r18c3'])
def test_pickled_disp_fn_matches_reference_closure(lib, name):
    """DispFn (the product's picklable disp_fn) vs the reference's lowess
    closure evaluated at non-integer, negative and beyond-range distances."""
    import pickle
    from hic3defdr_amd.analysis.core import DispFn
    g, kw = e2e_inputs(name)
    xs = g['disp_fn_xs']
    for c, cond in enumerate(kw['conds']):
        col = g['disp_per_dist'][:, c]
        fn = pickle.loads(pickle.dumps(DispFn(_native.disp_table(col), col)))
        assert rel_err(fn(xs), g['disp_fn_cont__%s' % cond]) < 1e-12


def test_bh_matches_oracle(lib):
    rng = np.random.default_rng(0)
    p = np.concatenate([rng.uniform(0, 1, 5000) ** 3, [np.nan, 1.0, 0.0],
                        np.repeat(0.01, 20)])
    rng.shuffle(p)
    q = _native.bh(p)
    np.testing.assert_array_equal(np.isnan(q), np.isnan(p))
    np.testing.assert_array_equal(q, oracle.adjust_pvalues(p))


def test_bh_matches_reference_qvalues(lib):
    g, kw = e2e_inputs('small2')
    chroms = kw['chroms']
    p = np.concatenate([g['pvalues__%s' % c][g['loop_idx__%s' % c]]
                        for c in chroms])
    q = np.concatenate([g['qvalues__%s' % c] for c in chroms])
    assert rel_err(_native.bh(p), q) < 1e-15
