"""cfg3 (BASELINE.json configs[2]): the whole mouse genome at 10 kb -- 20
mm10-sized chromosomes (265k bins), R = 4 (2 + 2), dist_thresh_max 200,
~46 M disp pixels -- through one genome-wide pooled estimate_disp
(analysis.py:169-206: every distance pools the pixels of all chromosomes),
the LRT and a genome-wide BH (analysis.py:286-303) on one GPU.

The reference would take days on this shape (its O(fail * N)
brentq fallback), so the whole genome is held to size-independent
properties; the reference-pinned checks of the same kernels are
test_gpu_scale.py (the full cfg2 chromosome) and the fixture-size goldens:
- every present distance has a finite dispersion in (0, 100), absent ones
  NaN; p in [0, 1]; positive finite means; llr <= 0 (nested models);
- the genome-wide BH is the CPU oracle's BH on the same p, bit for bit, and
  q is monotone in p;
- a second run is bit-identical (deterministic reductions at 46 M pixels:
  the 2^31-element scratch caps, the segment sums over 20 chromosomes).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DMAX = 200


@pytest.fixture(scope='module')
def cfg3():
    from hic3defdr_amd import synthetic
    parts = synthetic.draw_genome(synthetic.MM10_BINS, (2, 2), DMAX, seed=0)
    raw = np.concatenate([p[0] for p in parts])
    f = np.concatenate([p[1] for p in parts])
    dist = np.concatenate([p[2] for p in parts])
    del parts
    return raw, f, dist


def test_cfg3_whole_genome(cfg3):
    import oracle
    from hic3defdr_amd import _native
    ctx = _native.context(0)
    raw, f, dist = cfg3
    assert len(raw) > 40_000_000
    cond = np.array([0, 0, 1, 1], dtype=np.int32)
    C, D = 2, DMAX + 1
    runs = []
    for _ in range(2):
        dpd = ctx.disp_per_dist(raw, f, dist, cond, C, D)  # raises on flags
        tab = _native.disp_tables(dpd)
        p, llr, m0, m1, _ = ctx.lrt(raw, f, dist, tab, cond, want_disp=False)
        q = ctx.bh(p)
        runs.append((dpd, p, llr, m0, m1, q))
    dpd, p, llr, m0, m1, q = runs[0]
    present = np.isin(np.arange(D), dist)
    assert present[4:].all() and not present[:4].any()
    assert np.all(np.isfinite(dpd[present]))
    assert np.all(np.isnan(dpd[~present]))
    assert np.all((dpd[present] > 0) & (dpd[present] < 100.0))
    assert np.all(np.isfinite(p)) and np.all((p >= 0) & (p <= 1))
    assert np.all(np.isfinite(m0)) and np.all(m0 > 0)
    assert np.all(np.isfinite(m1)) and np.all(m1 > 0)
    assert np.all(llr <= 1e-9)
    # genome-wide BH: the oracle's (lib5c adjust_pvalues restated) bit for bit
    np.testing.assert_array_equal(q, oracle.adjust_pvalues(p))
    o = np.argsort(p, kind='stable')
    assert np.all(np.diff(q[o]) >= 0) and np.all(q >= p) and np.all(q <= 1)
    for a, b in zip(runs[0], runs[1]):
        np.testing.assert_array_equal(a, b)
