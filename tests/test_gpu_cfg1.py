"""BASELINE configs[0]'s shape at full size through the product class: two
chromosomes of 9,070 + 6,143 bins (mm10 chr18 / chr19 at 10 kb, the Bonev
demo's), R = 4 as 2 + 2, dist_thresh_max 200, loop clusters, res 10 kb --
synthetic data of that shape (the demo data is not available offline),
regenerated here from its seed.

``HiC3DeFDR.run_to_qvalues()`` + ``collect()`` (per-chromosome prepare_data,
the outdir with its offsets, the genome-wide concatenation of estimate_disp,
analysis.py:169-172, the per-chromosome LRT, the loop-pixel BH over both
chromosomes, :286-303, threshold / classify / the results TSV, :366-572)
against the reference's own run on the same files (tests/golden/
full_cfg1.npz, make_golden.py run_full_cfg1: its prepare_data +
estimate_disp, its lrt in 20 k-pixel chunks, its bh and collect)."""
import json
import os
import shutil
import tempfile

import numpy as np
import pandas as pd
import pytest

from conftest import golden, rel_err

pytestmark = pytest.mark.gpu

CFG1 = {'chr18': 9070, 'chr19': 6143}


@pytest.fixture(scope='module')
def cfg1():
    from hic3defdr_amd import HiC3DeFDR, synthetic
    g = golden('full_cfg1.npz')
    tmp = tempfile.mkdtemp(prefix='h3d_cfg1_')
    try:
        kw = synthetic.write_dataset(tmp, CFG1,
                                     dist_thresh_max=int(g['meta_dmax']),
                                     seed=int(g['meta_seed']))
        design = pd.DataFrame(kw['design'], index=kw['reps'],
                              columns=kw['conds'])
        h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                      bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                      design=design, outdir=os.path.join(tmp, 'out'),
                      dist_thresh_max=int(g['meta_dmax']),
                      loop_patterns=kw['loop_patterns'], res=10000)
        h.run_to_qvalues(verbose=False)
        h.collect(fdr=[0.01, 0.05], cluster_size=[3, 4])
        h.flush()
        yield h, g
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def test_cfg1_disp_per_dist_vs_reference(cfg1):
    """The genome-wide pooled segments (both chromosomes' pixels per
    distance): as at cfg2 (test_gpu_scale.py), a bounded-Brent search
    follows the reference's trial points while no near-tied NLL comparison
    flips; the reference itself flips such comparisons under a pixel-order
    permutation (cfg2_spread.npz)."""
    h, g = cfg1
    dpd, ref = h.load_data('disp_per_dist'), g['disp_per_dist']
    np.testing.assert_array_equal(np.isnan(dpd), np.isnan(ref))
    fin = np.isfinite(ref)
    rel = np.abs(dpd[fin] - ref[fin]) / ref[fin]
    dd = np.abs(dpd[fin] / (1 + dpd[fin]) - ref[fin] / (1 + ref[fin]))
    print('cfg1 disp_per_dist: %d segments, %d > 1e-6 rel, max rel %.3g, '
          'max |d delta| %.3g' % (rel.size, int(np.sum(rel > 1e-6)),
                                  rel.max(), dd.max()))
    assert np.sum(rel > 1e-6) <= 2
    assert dd.max() <= 1e-5


def _reference_orders(g):
    """The reference's end-to-end p / q under six pixel orders of its
    segments: order 0 = full_cfg1.npz, 1..5 = cfg1_spread.npz (make_golden.py
    run_cfg1_spread). Measured: it moves itself by up to 4.3e-3 in p."""
    sp = golden('cfg1_spread.npz')
    out = [{c: (g['p__%s' % c], g['q__%s' % c]) for c in CFG1}]
    for k in sp['perms'][1:]:
        out.append({c: (sp['p__%s__%d' % (c, k)], sp['q__%s__%d' % (c, k)])
                    for c in CFG1})
    # and the reference run with numpy's C-library pow instead of its AVX-512
    # SVML pow (full_cfg1_glibc.npz; test_lowess_mechanism.py)
    gl = golden('full_cfg1_glibc.npz')
    out.append({c: (gl['p__%s' % c], gl['q__%s' % c]) for c in CFG1})
    return out


def test_cfg1_stages_vs_reference(cfg1):
    """Per chromosome: disp pixel and loop sets identical; the sampled p and
    every loop pixel's q within 1e-6 of the reference's end-to-end result
    under one of its pixel orders (measured r04b: the product's p equal the
    reference's orders 4 / 5 to ~1e-9 while those move 7.8e-5 from its
    order 0); the mean MLEs within 1e-4 of order 0 (they see the segment
    moves through disp); identical calls at q < 0.01 / 0.05 / 0.1."""
    h, g = cfg1
    orders = _reference_orders(g)
    ours = {}
    for chrom in CFG1:
        assert int(h.load_data('disp_idx', chrom).sum()) == \
            int(g['n_disp__%s' % chrom])
        np.testing.assert_array_equal(h.load_data('loop_idx', chrom),
                                      g['loop_idx__%s' % chrom])
        s = g['sample_idx__%s' % chrom]
        ours[chrom] = (h.load_data('pvalues', chrom)[s],
                       h.load_data('qvalues', chrom))
        m0 = h.load_data('mu_hat_null', chrom)[s]
        m1 = h.load_data('mu_hat_alt', chrom)[s]
        e0 = (rel_err(ours[chrom][0], g['p__%s' % chrom]),
              rel_err(ours[chrom][1], g['q__%s' % chrom]),
              rel_err(m0, g['mu0__%s' % chrom]),
              rel_err(m1, g['mu1__%s' % chrom]))
        print('cfg1 %s vs the reference: sample p rel %.3g, loop q rel %.3g, '
              'mu0 %.3g, mu1 %.3g' % ((chrom,) + e0))
        assert max(e0[2:]) < 1e-4
        for fdr in (0.01, 0.05, 0.1):
            np.testing.assert_array_equal(ours[chrom][1] < fdr,
                                          g['q__%s' % chrom] < fdr)
    near = [max(max(rel_err(ours[c][0], o[c][0]), rel_err(ours[c][1], o[c][1]))
                for c in CFG1) for o in orders]
    k = int(np.argmin(near))
    print('cfg1: p / q vs each reference order %s; nearest %d; vs the '
          "reference's own run (order 0) %.3g (bar 3e-4)" % (
              ['%.2g' % v for v in near], k, near[0]))
    assert near[k] < 1e-6
    # the reference's own run: one distance of condition 1 is dropped there
    # by the weighted lowess' floor of the minimum weight (w * (1 / w) =
    # 1 - 2^-53 with numpy 1.26's AVX-512 pow; lowess_mechanism.npz), which
    # the product's pinned minimum weight keeps: measured 1.9e-4
    assert near[0] < 3e-4


def test_cfg1_stage_isolated_vs_reference(cfg1):
    """The product's LRT, BH and collect() on the reference's OWN smoothed
    tables (lowess_mechanism.npz: the reference's weighted lowess on
    full_cfg1's disp_per_dist, i.e. its estimate_disp's tables, order 0):
    per chromosome the sampled p, llr and mean MLEs and every loop pixel's q
    within 1e-6 of the reference's run, the same calls, and the results TSVs
    identical row for row. (The product's smoother on that disp_per_dist:
    tests/test_lowess_mechanism.py.)"""
    from hic3defdr_amd import HiC3DeFDR, _native
    h, g = cfg1
    mech = golden('lowess_mechanism.npz')
    tabs = np.stack([mech['cfg1__0__%d__table' % c] for c in range(2)],
                    axis=1)
    ctx = _native.context(0)
    cond = np.asarray(h.design, dtype=bool).argmax(axis=1)
    raw, f, dist, offsets = h._f_and_dist()
    p, llr, m0, m1, _ = ctx.lrt(raw, f, dist, tabs, cond, want_disp=False)
    out2 = os.path.join(os.path.dirname(h.outdir), 'out_stage')
    os.makedirs(out2, exist_ok=True)
    h2 = HiC3DeFDR(raw_npz_patterns=h.raw_npz_patterns,
                   bias_patterns=h.bias_patterns, chroms=h.chroms,
                   design=h.design, outdir=out2,
                   dist_thresh_max=h.dist_thresh_max,
                   loop_patterns=h.loop_patterns, res=h.res)
    for i, chrom in enumerate(h.chroms):
        for st in ('row', 'col', 'disp_idx', 'loop_idx'):
            h2.save_data(h.load_data(st, chrom), st, chrom)
        a, b = offsets[i], offsets[i + 1]
        for st, v in (('pvalues', p), ('llr', llr), ('mu_hat_null', m0),
                      ('mu_hat_alt', m1)):
            h2.save_data(v[a:b], st, chrom)
    h2.bh()
    h2.collect(fdr=[0.01, 0.05], cluster_size=[3, 4])
    h2.flush()
    for i, chrom in enumerate(h.chroms):
        s = g['sample_idx__%s' % chrom]
        a = offsets[i]
        q = h2.load_data('qvalues', chrom)
        e = (rel_err(p[a + s], g['p__%s' % chrom]),
             rel_err(q, g['q__%s' % chrom]),
             rel_err(m0[a + s], g['mu0__%s' % chrom]),
             rel_err(m1[a + s], g['mu1__%s' % chrom]),
             np.max(np.abs(llr[a + s] - g['llr__%s' % chrom]) /
                    np.maximum(np.abs(g['llr__%s' % chrom]), 1.0)))
        print('cfg1 %s stage-isolated vs the reference: p %.3g, q %.3g, '
              'mu0 %.3g, mu1 %.3g, llr %.3g' % ((chrom,) + e))
        assert max(e) < 1e-6
        for fdr in (0.01, 0.05, 0.1):
            np.testing.assert_array_equal(q < fdr, g['q__%s' % chrom] < fdr)
    for fdr in (0.01, 0.05):
        for size in (3, 4):
            with open(os.path.join(out2, 'results_%g_%i.tsv' % (fdr, size))) \
                    as fh:
                ours = _rows(fh.read())
            ref = _rows(str(g['results_%g_%i' % (fdr, size)]))
            assert ours == ref
            with open(os.path.join(out2, 'results_%g_%i.tsv' % (fdr, size))) \
                    as fh:
                assert fh.read() == str(g['results_%g_%i' % (fdr, size)])


def _rows(text):
    lines = text.rstrip('\n').split('\n')
    head = lines[0].split('\t')
    k = head.index('cluster')
    out = []
    for ln in lines[1:]:
        f = ln.split('\t')
        # the cluster column lists a Python set of pixels in hash-table
        # order (cluster_table.py:67 list(cluster)): compared as a set
        f[k] = frozenset(map(tuple, json.loads(f[k])))
        out.append(f)
    return head, out


def test_cfg1_results_tsv_identical(cfg1):
    """collect()'s results_<fdr>_<size>.tsv -- the loop calls with their
    classification -- the reference's, row for row and field for field, and
    the file byte for byte."""
    h, g = cfg1
    for fdr in (0.01, 0.05):
        for size in (3, 4):
            with open(os.path.join(h.outdir, 'results_%g_%i.tsv' % (fdr, size))) \
                    as fh:
                ours = _rows(fh.read())
            ref = _rows(str(g['results_%g_%i' % (fdr, size)]))
            print('results_%g_%i.tsv: %d rows' % (fdr, size, len(ref[1])))
            assert ours[0] == ref[0]
            assert len(ours[1]) == len(ref[1])
            for a, b in zip(ours[1], ref[1]):
                assert a == b, (a, b)
            # and the file itself, byte for byte (each cluster's pixels in
            # the reference's Python-set order, where the goldens' interpreter
            # is one whose set table h3d_calls.cpp replays)
            with open(os.path.join(h.outdir, 'results_%g_%i.tsv' % (fdr, size))) \
                    as fh:
                same = fh.read() == str(g['results_%g_%i' % (fdr, size)])
            if not same:
                from test_calls import _order_mismatch
                _order_mismatch(('results_%g_%i.tsv' % (fdr, size),
                                 'cluster pixel order'))
