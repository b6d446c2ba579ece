"""Operator-level drop-ins (reference util/lrt.py lrt, util/dispersion.py
qcml / cml / mme / mme_per_pixel) on the GPU vs the reference's own values
on the same inputs (tests/golden/unit_nb.npz)."""
import numpy as np
import pytest

from conftest import golden, rel_err

pytestmark = pytest.mark.gpu


def test_lrt_operator_matches_reference():
    from hic3defdr_amd.util.lrt import lrt
    g = golden('unit_nb.npz')
    for pre, refit in (('lrt', True), ('lrtnr', False)):
        p, llr, m0, m1 = lrt(g['lrt_raw'], g['lrt_f'], g['lrt_disp'],
                             g['lrt_design'], refit_mu=refit)
        assert rel_err(p, g[pre + '_p']) < 1e-7
        assert rel_err(m0, g[pre + '_mu0']) < 1e-9
        assert rel_err(m1, g[pre + '_mu1']) < 1e-9
        assert np.max(np.abs(llr - g[pre + '_llr'])) < 1e-8


def test_lrt_operator_broadcasts_disp_like_fit_mu_hat():
    from hic3defdr_amd.util.lrt import lrt
    g = golden('unit_nb.npz')
    raw, f, design = g['lrt_raw'], g['lrt_f'], g['lrt_design']
    wide = np.broadcast_to(0.05, raw.shape)
    a = lrt(raw, f, 0.05, design)
    b = lrt(raw, f, wide, design)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_dispersion_operators_match_reference():
    from hic3defdr_amd.util import dispersion
    g = golden('unit_nb.npz')
    for s in range(int(g['n_segs'])):
        data, f = g['seg%d_data' % s], g['seg%d_f' % s]
        assert rel_err(dispersion.qcml(data, f=f), g['seg%d_qcml' % s]) < 1e-6
        x = data.astype(float)
        assert rel_err(dispersion.cml(x / f), g['seg%d_cml' % s]) < 1e-6
        y = data.astype(float)
        assert rel_err(dispersion.mme(y, f=f.copy()), g['seg%d_mme' % s]) < 1e-12
    with pytest.raises(Exception):
        dispersion.cml(g['seg0_data'].copy(), f=g['seg0_f'])  # int /= float


def test_qcml_batch_equals_per_segment_calls():
    """qcml_batch: every segment in one driver call, bit-equal to the
    single-segment qcml calls (and to the reference's values); the per-call
    and batched costs printed (-rP) for INTEGRATION.md."""
    import time
    from hic3defdr_amd.synthetic import draw_band
    from hic3defdr_amd.util import dispersion
    g = golden('unit_nb.npz')
    segs = [(g['seg%d_data' % s], g['seg%d_f' % s])
            for s in range(int(g['n_segs']))]
    # plus the segments of a synthetic band: (distance, condition) blocks
    raw, f, dist = draw_band(2000, (2, 3), 60, seed=9)
    for d in range(4, 61, 3):
        m = dist == d
        segs += [(raw[m][:, :2], f[m][:, :2]), (raw[m][:, 2:], f[m][:, 2:])]
    batched = dispersion.qcml_batch(segs)
    t0 = time.perf_counter()
    single = [dispersion.qcml(d, f=ff) for d, ff in segs]
    t1 = time.perf_counter()
    dispersion.qcml_batch(segs)
    t2 = time.perf_counter()
    np.testing.assert_array_equal(np.array(batched), np.array(single))
    for s in range(int(g['n_segs'])):
        assert rel_err(batched[s], g['seg%d_qcml' % s]) < 1e-6
    print('qcml: %d segments, %.2f ms per single-segment call, %.2f ms for '
          'the batch' % (len(segs), (t1 - t0) / len(segs) * 1e3,
                         (t2 - t1) * 1e3))


def test_qcml_tol_vs_oracle():
    """qcml(tol=...) (dispersion.py:10-43: iterate while |disp - new disp|
    > tol) on the device state machine against the oracle's qcml at the
    same tol; the ctx's tolerance is back at the default afterwards (the
    next default call equals the reference's value)."""
    import oracle
    from hic3defdr_amd.util import dispersion
    g = golden('unit_nb.npz')
    for s in range(int(g['n_segs'])):
        data, f = g['seg%d_data' % s], g['seg%d_f' % s]
        for tol in (1e-2, 1e-3, 1e-6):
            got = dispersion.qcml(data, f=f, tol=tol)
            want = oracle.qcml(data.astype(float), f=f, tol=tol)
            assert rel_err(got, want) < 1e-6, (s, tol, got, want)
        got = dispersion.qcml_batch([(data, f)], tol=1e-2)[0]
        assert rel_err(got, oracle.qcml(data.astype(float), f=f, tol=1e-2)) < 1e-6
        assert rel_err(dispersion.qcml(data, f=f), g['seg%d_qcml' % s]) < 1e-6
    with pytest.raises(Exception):
        dispersion.qcml(g['seg0_data'], f=g['seg0_f'], tol=-1.0)
