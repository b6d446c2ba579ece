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
    print('cfg1: p / q vs each reference order %s; nearest %d' % (
        ['%.2g' % v for v in near], k))
    assert near[k] < 1e-6


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
    classification -- the reference's, row for row and field for field (the
    cluster column as the set of pixels it lists)."""
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
