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
  the 2^31-element scratch caps, the segment sums over 20 chromosomes);
- six whole genome-wide segments (distances 4, 100, 200 in both conditions,
  each pooling ~160-260 k pixels of 20 chromosomes): the CPU oracle's qcml
  (dispersion.py:10-43, pinned to the reference's goldens) vs the GPU's
  disp_per_dist at 1e-6, at most one near-tied Brent comparison (within
  xatol in delta) as test_gpu_scale.py;
- 3,000 sampled pixels: the oracle's lrt (lrt.py:7-50) with the GPU's own
  tables vs the GPU's p and llr at 1e-6 relative.
The same comparison over every pixel of the genome -- the CPU restatement's
whole estimate_disp + lrt + BH against the GPU's, calls at three FDRs -- is
bench.py's other_configs.cfg3.vs_cpu_restatement.
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


COND = np.array([0, 0, 1, 1], dtype=np.int32)


@pytest.fixture(scope='module')
def cfg3_runs(cfg3):
    """Two GPU runs of the genome: (disp_per_dist, tables, p, llr, mu0,
    mu1, q) each."""
    from hic3defdr_amd import _native
    ctx = _native.context(0)
    raw, f, dist = cfg3
    C, D = 2, DMAX + 1
    runs = []
    for _ in range(2):
        dpd = ctx.disp_per_dist(raw, f, dist, COND, C, D)  # raises on flags
        tab = _native.disp_tables(dpd)
        p, llr, m0, m1, _ = ctx.lrt(raw, f, dist, tab, COND, want_disp=False)
        q = ctx.bh(p)
        runs.append((dpd, tab, p, llr, m0, m1, q))
    return runs


def test_cfg3_whole_genome(cfg3, cfg3_runs):
    import oracle
    raw, f, dist = cfg3
    assert len(raw) > 40_000_000
    C, D = 2, DMAX + 1
    runs = cfg3_runs
    dpd, _, p, llr, m0, m1, q = runs[0]
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


def test_cfg3_segments_vs_oracle(cfg3, cfg3_runs):
    """Whole genome-wide segments (every chromosome's pixels at one distance,
    one condition) through the oracle's qcml vs the GPU's disp_per_dist."""
    from concurrent.futures import ThreadPoolExecutor
    import oracle
    raw, f, dist = cfg3
    dpd = cfg3_runs[0][0]
    jobs, keys = [], []
    for d in (4, 100, 200):
        sel = np.flatnonzero(dist == d)
        for c in range(2):
            reps = COND == c
            jobs.append((raw[sel][:, reps].astype(float), f[sel][:, reps]))
            keys.append((d, c))
    # (numpy / scipy release the GIL: ~10 s for the six on the host)
    with ThreadPoolExecutor(6) as ex:
        want = np.array(list(ex.map(lambda a: oracle.qcml(*a), jobs)))
    got = np.array([dpd[d, c] for d, c in keys])
    rel = np.abs(got - want) / np.abs(want)
    ddelta = np.abs(got / (1 + got) - want / (1 + want))
    print('cfg3 segments vs the oracle: %s rel %s, |d delta| %s' % (
        keys, np.array2string(rel, precision=2),
        np.array2string(ddelta, precision=2)))
    # a near-tied Brent comparison can send one search to another point
    # inside its tolerance (xatol 1e-5 in delta; test_gpu_scale.py)
    assert np.sum(rel > 1e-6) <= 1, rel
    assert np.all(ddelta <= 1e-5), ddelta


def test_cfg3_lrt_sample_vs_oracle(cfg3, cfg3_runs):
    """3,000 pixels sampled over the genome through the oracle's lrt with
    the GPU's own tables (lrt.py:7-50) vs the GPU's p and llr."""
    import oracle
    raw, f, dist = cfg3
    _, tab, p, llr, _, _, _ = cfg3_runs[0]
    rng = np.random.default_rng(1)
    idx = np.sort(rng.choice(len(raw), 3000, replace=False))
    design = np.zeros((4, 2), dtype=bool)
    design[np.arange(4), COND] = True
    disp = tab[dist[idx]][:, COND]          # lrt.py's per-replicate disp
    p_o, llr_o, _, _ = oracle.lrt(raw[idx].astype(float), f[idx], disp, design)
    np.testing.assert_allclose(p[idx], p_o, rtol=1e-6, atol=1e-300)
    np.testing.assert_allclose(llr[idx], llr_o, rtol=1e-6, atol=1e-9)


def test_cfg3_through_the_class():
    """The same genome shape END TO END through the product route: the 20
    chromosomes written in the reference's input layout (NPZ + bias files,
    loop clusters; synthetic.write_genome), ``HiC3DeFDR.run_to_qvalues()``
    (analysis.py:305-364: per-chromosome prepare_data, the genome-wide pooled
    estimate_disp over the concatenated chromosomes with their offsets, the
    LRT over the resident session, the loop-pixel BH over the genome from
    the outdir files), then:
    - the properties above on every chromosome's outdir arrays;
    - the genome-wide BH of the files = the oracle's BH of the concatenated
      loop-pixel p-values, bit for bit;
    - the class's device-resident route = the host-array route on the same
      pixels (h._f_and_dist() from the outdir files -> ctx.disp_per_dist,
      the host smoother, ctx.lrt): disp_per_dist and every p bit for bit."""
    import shutil
    import tempfile
    import oracle
    import pandas as pd
    from hic3defdr_amd import HiC3DeFDR, _native, synthetic
    base = tempfile.mkdtemp(prefix='h3d_cfg3_class_')
    try:
        kw = synthetic.write_genome(base, synthetic.MM10_BINS, seed=3,
                                    workers=16, dmax=DMAX)
        design = pd.DataFrame(kw['design'], index=kw['reps'],
                              columns=kw['conds'])
        h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                      bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                      design=design, outdir=base + '/out', dist_thresh_max=DMAX,
                      loop_patterns=kw['loop_patterns'], res=10000)
        h.run_to_qvalues(verbose=False)
        C, D = 2, DMAX + 1
        dpd = h.load_data('disp_per_dist')
        p, offs = h.load_data('pvalues', 'all')
        assert len(p) > 40_000_000 and len(offs) == 21
        for st in ('llr', 'mu_hat_null', 'mu_hat_alt', 'disp'):
            a, o2 = h.load_data(st, 'all')
            np.testing.assert_array_equal(o2, offs)
        llr = h.load_data('llr', 'all')[0]
        m0 = h.load_data('mu_hat_null', 'all')[0]
        m1 = h.load_data('mu_hat_alt', 'all')[0]
        raw, f, dist, offsets = h._f_and_dist()
        np.testing.assert_array_equal(offsets, offs)
        present = np.isin(np.arange(D), dist)
        assert np.all(np.isfinite(dpd[present]))
        assert np.all(np.isnan(dpd[~present]))
        assert np.all((dpd[present] > 0) & (dpd[present] < 100.0))
        assert np.all(np.isfinite(p)) and np.all((p >= 0) & (p <= 1))
        assert np.all(np.isfinite(m0)) and np.all(m0 > 0)
        assert np.all(np.isfinite(m1)) and np.all(m1 > 0)
        assert np.all(llr <= 1e-9)
        # the genome-wide loop-pixel BH of the files
        li = h.load_data('loop_idx', 'all')[0]
        q = h.load_data('qvalues', 'all')[0]
        assert li.sum() > 1000 and len(q) == li.sum()
        np.testing.assert_array_equal(q, oracle.adjust_pvalues(p[li]))
        # the host-array route on the same pixels
        ctx = _native.context(0)
        cond = np.array([0, 0, 1, 1], dtype=np.int32)
        dpd_h = ctx.disp_per_dist(raw, f, dist, cond, C, D)
        np.testing.assert_array_equal(dpd_h, dpd)
        tab = _native.disp_tables(dpd_h)
        p_h, llr_h, m0_h, m1_h, _ = ctx.lrt(raw, f, dist, tab, cond,
                                            want_disp=False)
        np.testing.assert_array_equal(p_h, p)
        np.testing.assert_array_equal(llr_h, llr)
        np.testing.assert_array_equal(m1_h, m1)
        print('cfg3 through the class: %d disp pixels, %d loop pixels, '
              'q < 0.05: %d' % (len(p), int(li.sum()), int(np.sum(q < 0.05))))
    finally:
        shutil.rmtree(base, ignore_errors=True)
