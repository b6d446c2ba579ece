"""The device smoother (h3d_disp_tables_dev, csrc/h3d_table.hip) against the
host one (h3d_disp_tables, pinned to the reference's lowess tables): the
same bits on the golden dispersion columns and on random ones (weighted /
unweighted, given / automatic frac, NaN holes, ties), the same errors, the
host hand-back for degenerate fits and for D > 1024, and the LRT over the
device table (h3d_lrt_dev_tab) equal to the LRT over the host table."""
import glob
import os

import numpy as np
import pytest

from table_emu import emu, random_column

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.fixture(scope='module')
def ctx():
    from hic3defdr_amd import _native
    return _native.context(0)


def _dev_tables(ctx, dpd, weighted=True, frac=None):
    import torch
    dev = torch.device('cuda', 0)
    t_in = torch.from_numpy(np.ascontiguousarray(dpd, dtype=np.float64)).to(dev)
    t_out = torch.full_like(t_in, -7.0)
    torch.cuda.synchronize()
    D, C = dpd.shape
    ctx.disp_tables_dev(t_in.data_ptr(), D, C, t_out.data_ptr(),
                        weighted=weighted, frac=frac)
    ctx.disp_tables_wait()
    return t_out.cpu().numpy()


def _host_tables(dpd, weighted=True, frac=None):
    from hic3defdr_amd import _native
    return _native.disp_tables(dpd, weighted=weighted, frac=frac)


def test_golden_columns_bit_equal(ctx):
    files = sorted(glob.glob(os.path.join(GOLDEN, 'e2e_*.npz'))) + \
        [os.path.join(GOLDEN, 'full_cfg2.npz')]
    for f in files:
        dpd = np.load(f)['disp_per_dist']
        for weighted in (True, False):
            got = _dev_tables(ctx, dpd, weighted)
            np.testing.assert_array_equal(got, _host_tables(dpd, weighted),
                                          err_msg=f)


def test_random_columns_bit_equal(ctx):
    """Column by column (the kernel runs one condition per workgroup), the
    degenerate ones included: those come back from the host smoother."""
    from hic3defdr_amd import _native
    rng = np.random.default_rng(11)
    n_deg = n_fail = 0
    for _ in range(120):
        col, weighted, frac = random_column(rng)
        frac = None if frac < 0 else frac
        dpd = col[:, None]
        try:
            ref = _host_tables(dpd, weighted, frac)
        except _native.H3DError:
            with pytest.raises(_native.H3DError):
                _dev_tables(ctx, dpd, weighted, frac)
            n_fail += 1
            continue
        n_deg += isinstance(emu(list(col), weighted,
                                -1. if frac is None else frac), str)
        np.testing.assert_array_equal(_dev_tables(ctx, dpd, weighted, frac),
                                      ref)
    assert n_deg >= 1        # the hand-back path ran
    assert n_fail >= 0


def test_many_conditions_and_large_d(ctx):
    rng = np.random.default_rng(3)
    for D, C in [(251, 2), (61, 3), (1024, 4), (1500, 2)]:
        d = np.arange(D)
        dpd = np.stack([0.05 + 0.3 * np.exp(-d / (10 + 7 * c)) +
                        rng.normal(0, 0.01, D) for c in range(C)], axis=1)
        dpd = np.abs(dpd)
        dpd[rng.random((D, C)) < 0.05] = np.nan
        np.testing.assert_array_equal(_dev_tables(ctx, dpd),
                                      _host_tables(dpd))


def test_errors_as_host(ctx):
    from hic3defdr_amd import _native
    dpd = np.full((40, 2), np.nan)
    dpd[3, :] = 0.1          # one finite point: the reference raises
    with pytest.raises(_native.H3DError):
        _host_tables(dpd)
    with pytest.raises(_native.H3DError):
        _dev_tables(ctx, dpd)
    # the ctx is usable afterwards
    ok = np.abs(0.1 + 0.01 * np.sin(np.arange(50.)))[:, None]
    np.testing.assert_array_equal(_dev_tables(ctx, ok), _host_tables(ok))


def test_lrt_over_device_table(ctx):
    """estimate_disp -> table on the device -> LRT (the bench step) equals the
    LRT over the host table, bit for bit."""
    import torch
    from hic3defdr_amd.synthetic import draw_band
    raw, f, dist = draw_band(3000, (2, 2), 60, seed=5)
    n, R = raw.shape
    cond = np.array([0, 0, 1, 1], dtype=np.int32)
    C, D = 2, 61
    dev = torch.device('cuda', 0)
    t_raw = torch.from_numpy(raw.astype(np.int32)).to(dev)
    t_f = torch.from_numpy(f).to(dev)
    t_d = torch.from_numpy(dist.astype(np.int32)).to(dev)
    torch.cuda.synchronize()
    dpd = ctx.disp_per_dist_dev(t_raw.data_ptr(), t_f.data_ptr(),
                                t_d.data_ptr(), n, R, cond, C, D)
    host_tab = _host_tables(dpd)

    def outs():
        t = torch.empty(n, dtype=torch.float64, device=dev)
        return [t, torch.empty_like(t), torch.empty_like(t),
                torch.empty((n, C), dtype=torch.float64, device=dev),
                torch.empty((n, C), dtype=torch.float64, device=dev)]
    a, b = outs(), outs()
    ctx.lrt_dev(t_raw.data_ptr(), t_f.data_ptr(), t_d.data_ptr(), host_tab,
                n, R, cond, *[x.data_ptr() for x in a])
    t_dpd = torch.from_numpy(dpd).to(dev)
    t_tab = torch.empty_like(t_dpd)
    torch.cuda.synchronize()
    ctx.disp_tables_dev(t_dpd.data_ptr(), D, C, t_tab.data_ptr())
    ctx.lrt_dev_tab(t_raw.data_ptr(), t_f.data_ptr(), t_d.data_ptr(),
                    t_tab.data_ptr(), D, n, R, cond,
                    *[x.data_ptr() for x in b])
    np.testing.assert_array_equal(t_tab.cpu().numpy(), host_tab)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())


def test_fused_estimate_disp_tables(ctx):
    """h3d_estimate_disp_dev: the same disp_per_dist as h3d_disp_per_dist_dev,
    the host smoother's tables on the device, the same LRT."""
    import torch
    from hic3defdr_amd.synthetic import draw_band
    raw, f, dist = draw_band(3000, (2, 3), 60, seed=6)
    n, R = raw.shape
    cond = np.array([0, 0, 1, 1, 1], dtype=np.int32)
    C, D = 2, 61
    dev = torch.device('cuda', 0)
    t_raw = torch.from_numpy(raw.astype(np.int32)).to(dev)
    t_f = torch.from_numpy(f).to(dev)
    t_d = torch.from_numpy(dist.astype(np.int32)).to(dev)
    t_tab = torch.full((D, C), -7.0, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ref = ctx.disp_per_dist_dev(t_raw.data_ptr(), t_f.data_ptr(),
                                t_d.data_ptr(), n, R, cond, C, D)
    got = ctx.estimate_disp_dev(t_raw.data_ptr(), t_f.data_ptr(),
                                t_d.data_ptr(), n, R, cond, C, D,
                                t_tab.data_ptr())
    np.testing.assert_array_equal(got, ref)
    outs = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
    outs += [torch.empty((n, C), dtype=torch.float64, device=dev)
             for _ in range(2)]
    ctx.lrt_dev_tab(t_raw.data_ptr(), t_f.data_ptr(), t_d.data_ptr(),
                    t_tab.data_ptr(), D, n, R, cond,
                    *[x.data_ptr() for x in outs])
    np.testing.assert_array_equal(t_tab.cpu().numpy(), _host_tables(ref))
    p_host = ctx.lrt(raw.astype(np.int64), f, dist,
                     _host_tables(ref), cond)[0]
    np.testing.assert_array_equal(outs[0].cpu().numpy(), p_host)
