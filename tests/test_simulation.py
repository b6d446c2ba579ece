"""simulate() / kr_balance / filter_sparse_rows_count / evaluate() vs the
reference (tests/golden/sim_small2.npz, made by make_golden.py run_sim: the
reference simulating from its own small2 analysis with np.random.seed(0),
balancing the simulated replicates, analysing them, evaluating).

CPU: the product's simulate() is fed the reference's stage arrays (the
simulation is host code drawing from the reference's global numpy stream,
so the simulated counts must come out identical); the balancing and the
evaluation run on the reference's simulated matrices / q-values. The GPU
end-to-end chain is in tests/test_gpu_simulation.py."""
import os
import shutil
import tempfile

import numpy as np
import pandas as pd
import pytest
import scipy.sparse as sparse

from conftest import e2e_inputs, golden, rel_err

SIMREPS = ['A1', 'A2', 'B1', 'B2']


def _sim_matrix(g, rep, chrom, n):
    return sparse.csr_matrix(
        (g['sim__%s__%s__data' % (rep, chrom)],
         g['sim__%s__%s__indices' % (rep, chrom)],
         g['sim__%s__%s__indptr' % (rep, chrom)]), shape=(n, n))


def _analysis_from_goldens(outdir):
    """A HiC3DeFDR whose outdir holds the reference's small2 stage arrays and
    the product's disp_fn of the reference's disp_per_dist."""
    from hic3defdr_amd import HiC3DeFDR, _native
    from hic3defdr_amd.analysis.core import DispFn
    g, kw = e2e_inputs('small2')
    design = pd.DataFrame(kw['design'], index=kw['reps'], columns=kw['conds'])
    h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                  bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                  design=design, outdir=outdir,
                  dist_thresh_max=kw['dist_thresh_max'],
                  loop_patterns=kw['loop_patterns'])
    for c in kw['chroms']:
        for st in ('row', 'col', 'size_factors', 'scaled', 'disp_idx'):
            h.save_data(g['%s__%s' % (st, c)], st, c)
    for i, cond in enumerate(kw['conds']):
        col = g['disp_per_dist'][:, i]
        h.save_disp_fn(cond, DispFn(_native.disp_table(col), col))
    return h, kw


def test_simulate_matches_reference_counts():
    g = golden('sim_small2.npz')
    tmp = tempfile.mkdtemp(prefix='h3d_sim_')
    try:
        h, kw = _analysis_from_goldens(os.path.join(tmp, 'out'))
        sim = os.path.join(tmp, 'sim')
        np.random.seed(int(g['meta_seed']))
        h.simulate('ES', outdir=sim, verbose=False)
        assert open(os.path.join(sim, 'design.csv'), 'rb').read() == \
            g['sim_design_csv'].tobytes()
        for c in kw['chroms']:
            labels = np.loadtxt(os.path.join(sim, 'labels_%s.txt' % c),
                                dtype='U7')
            np.testing.assert_array_equal(labels, g['labels__%s' % c])
            for rep in SIMREPS:
                m = sparse.load_npz(os.path.join(sim, '%s_%s_raw.npz' % (rep, c)))
                ref = _sim_matrix(g, rep, c, m.shape[0])
                assert (m != ref).nnz == 0, (rep, c)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def test_filter_and_kr_balance_match_reference():
    from hic3defdr_amd.util.balancing import kr_balance
    from hic3defdr_amd.util.filtering import filter_sparse_rows_count
    g = golden('sim_small2.npz')
    _, kw = e2e_inputs('small2')
    sizes = {'chrA': 420, 'chrB': 300}
    for c in kw['chroms']:
        for rep in SIMREPS:
            m = _sim_matrix(g, rep, c, sizes[c])
            filt = filter_sparse_rows_count(m)
            assert filt.nnz == int(g['filt__%s__%s__nnz' % (rep, c)])
            np.testing.assert_array_equal(
                np.asarray(filt.sum(axis=1)).ravel(),
                g['filt__%s__%s__rowsum' % (rep, c)])
            _, bias, _ = kr_balance(filt, fl=0)
            ref = g['bias__%s__%s' % (rep, c)]
            np.testing.assert_array_equal(bias == 0, ref == 0)
            assert rel_err(bias, ref) < 1e-9


def test_filter_dense_equals_sparse():
    from hic3defdr_amd.util.filtering import filter_sparse_rows_count
    rng = np.random.default_rng(2)
    a = np.triu(rng.poisson(0.3, (120, 120)))
    d = filter_sparse_rows_count(a, min_nnz=5, k=20)
    s = filter_sparse_rows_count(sparse.csr_matrix(a), min_nnz=5, k=20)
    np.testing.assert_array_equal(d, s.toarray())


@pytest.mark.parametrize('which', [0, 1, 2, 3])
def test_evaluate_matches_reference(which):
    """evaluate() on the reference's simulated-analysis q-values: every
    eval npz array identical."""
    from hic3defdr_amd import HiC3DeFDR
    g = golden('sim_small2.npz')
    _, kw = e2e_inputs('small2')
    a, b, rr = (int(v) for v in g['meta_evals'][which])
    a = None if a < 0 else a
    b = None if b < 0 else b
    tmp = tempfile.mkdtemp(prefix='h3d_eval_')
    try:
        lab = os.path.join(tmp, 'labels_<chrom>.txt')
        design = pd.DataFrame({'A': [1, 1, 0, 0], 'B': [0, 0, 1, 1]},
                              dtype=bool, index=SIMREPS)
        h = HiC3DeFDR(raw_npz_patterns=['x_<chrom>'] * 4,
                      bias_patterns=['y_<chrom>'] * 4, chroms=kw['chroms'],
                      design=design, outdir=os.path.join(tmp, 'out'),
                      dist_thresh_max=kw['dist_thresh_max'],
                      loop_patterns={'ES': kw['loop_patterns']['ES']})
        for c in kw['chroms']:
            np.savetxt(lab.replace('<chrom>', c), g['labels__%s' % c], fmt='%s')
            for st in ('pvalues', 'qvalues', 'disp_idx', 'loop_idx', 'row',
                       'col'):
                h.save_data(g['simrun__%s__%s' % (st, c)], st, c)
        h.evaluate('ES', lab, min_dist=a, max_dist=b, rerun_bh=bool(rr))
        fn = 'eval' if a is None and b is None else 'eval_%s_%s' % (a, b)
        e = np.load(os.path.join(tmp, 'out', fn + '.npz'))
        for k in ('fdr', 'fpr', 'tpr', 'thresh'):
            ref = g['eval__%s__%s' % (fn, k)]
            np.testing.assert_array_equal(np.isnan(e[k]), np.isnan(ref))
            np.testing.assert_allclose(e[k], ref, rtol=1e-12, atol=0)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def test_oracle_evaluate_matches_reference():
    """The oracle's evaluate / make_y_true (the reference's own loops,
    oracle/restatement.py) pinned to the reference's eval.npz on its own
    simulated-analysis q-values: the checker test_gpu_sim_scale.py uses at
    the genome's scale."""
    import oracle
    g = golden('sim_small2.npz')
    _, kw = e2e_inputs('small2')
    ys, qs = [], []
    for c in kw['chroms']:
        di = g['simrun__disp_idx__%s' % c]
        li = g['simrun__loop_idx__%s' % c]
        sel = np.flatnonzero(di)[li]
        row = g['simrun__row__%s' % c][sel]
        col = g['simrun__col__%s' % c][sel]
        cl = oracle.load_clusters(kw['loop_patterns']['ES'].replace('<chrom>', c))
        ys.append(oracle.make_y_true(row, col, cl, g['labels__%s' % c]))
        qs.append(g['simrun__qvalues__%s' % c])
    e = oracle.evaluate(np.concatenate(ys), np.concatenate(qs))
    for k, v in zip(('fdr', 'fpr', 'tpr', 'thresh'), e):
        ref = g['eval__eval__%s' % k]
        np.testing.assert_array_equal(np.isnan(v), np.isnan(ref))
        np.testing.assert_allclose(v, ref, rtol=1e-12, atol=0)
