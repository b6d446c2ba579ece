"""GPU parity: libh3d.so kernels on a real MI355X vs the reference goldens and
the CPU oracle. Tolerances (north star): p/q within 1e-6 relative; integer
outputs (union pixels, raw counts, disp_idx, loop_idx) bit-exact."""
import numpy as np
import pytest
import scipy.sparse as sparse

import oracle
from conftest import e2e_inputs, rel_err

pytestmark = pytest.mark.gpu

RTOL_PQ = 1e-6      # north-star tolerance on p- and q-values
RTOL_DISP = 1e-6    # per-distance qcml (Brent xatol 1e-5 on a flat NLL)
RTOL_MU = 1e-8      # MLE of mu (reference secant tol 1.48e-8 absolute)


@pytest.fixture(scope='module')
def ctx():
    from hic3defdr_amd import _native
    return _native.context(0)


def _stage_inputs(name):
    """raw / f / dist of the disp pixels exactly as the reference's
    estimate_disp builds them (analysis.py:169-183), from the goldens."""
    g, kw = e2e_inputs(name)
    raws, fs, dists = [], [], []
    for c in kw['chroms']:
        bias = oracle.load_bias([p.replace('<chrom>', c)
                                 for p in kw['bias_patterns']])
        di = g['disp_idx__%s' % c]
        row, col = g['row__%s' % c][di], g['col__%s' % c][di]
        raws.append(g['raw__%s' % c][di])
        fs.append(bias[row] * bias[col] * g['size_factors__%s' % c][di])
        dists.append(col - row)
    return g, kw, np.concatenate(raws), np.concatenate(fs), \
        np.concatenate(dists)


@pytest.mark.parametrize('name', ['small2', 'c3r9', 'r18c3', 'r16c2'])
def test_disp_per_dist_vs_reference(ctx, name):
    g, kw, raw, f, dist = _stage_inputs(name)
    design = kw['design']
    C = design.shape[1]
    D = kw['dist_thresh_max'] + 1
    out = ctx.disp_per_dist(raw, f, dist, design.argmax(axis=1), C, D)
    ref = g['disp_per_dist']
    np.testing.assert_array_equal(np.isnan(out), np.isnan(ref))
    np.testing.assert_allclose(out, ref, rtol=RTOL_DISP, atol=1e-12)


@pytest.mark.parametrize('name', ['small2', 'c3r9', 'r18c3', 'r16c2'])
def test_lrt_vs_reference(ctx, name):
    from hic3defdr_amd import _native
    g, kw, raw, f, dist = _stage_inputs(name)
    design = kw['design']
    # the reference's own fitted table (disp_fn at every integer distance),
    # so this checks the LRT alone (the smoother is checked in test_abi)
    tab = np.stack([g['disp_fn_table__%s' % cond] for cond in kw['conds']],
                   axis=1)
    p, llr, m0, m1, disp = ctx.lrt(raw, f, dist, tab, design.argmax(axis=1))
    pr = np.concatenate([g['pvalues__%s' % c] for c in kw['chroms']])
    m0r = np.concatenate([g['mu_hat_null__%s' % c] for c in kw['chroms']])
    m1r = np.concatenate([g['mu_hat_alt__%s' % c] for c in kw['chroms']])
    dr = np.concatenate([g['disp__%s' % c] for c in kw['chroms']])
    assert rel_err(disp, dr) < 1e-12
    assert rel_err(p, pr) < RTOL_PQ
    assert rel_err(m0, m0r) < RTOL_MU
    assert rel_err(m1, m1r) < RTOL_MU


def test_lrt_refit_false_vs_oracle(ctx):
    g, kw, raw, f, dist = _stage_inputs('small2')
    design = kw['design']
    from hic3defdr_amd import _native
    tab = np.stack([_native.disp_table(g['disp_per_dist'][:, c])
                    for c in range(design.shape[1])], axis=1)
    p, llr, m0, m1, _ = ctx.lrt(raw, f, dist, tab, design.argmax(axis=1),
                                refit_mu=False)
    disp = tab[dist]
    rp, rllr, rm0, rm1 = oracle.lrt(raw, f, np.dot(disp, design.T), design,
                                    refit_mu=False)
    assert rel_err(p, rp) < RTOL_PQ
    assert rel_err(m0, rm0) < 1e-14
    assert rel_err(m1, rm1) < 1e-14


@pytest.mark.parametrize('R,C', [(9, 2), (12, 3), (18, 3), (24, 5), (32, 8)])
@pytest.mark.parametrize('refit', [True, False])
def test_lrt_wide_designs_vs_oracle(ctx, R, C, refit):
    """R > 8 runs k_lrt8 (one 8-lane group per pixel, h3d_lrt_group.h):
    unequal condition sizes, interleaved replicate order, numpy's tail
    association (R % 8 != 0) and the compacted means of refit_mu=False."""
    rng = np.random.default_rng(R * 10 + C)
    n = 600
    cond = np.sort(np.r_[np.arange(C), rng.integers(0, C, R - C)])
    rng.shuffle(cond)
    design = np.eye(C, dtype=bool)[cond]
    f = np.exp(rng.normal(0, 0.3, (n, R)))
    mu = rng.gamma(2.0, 20.0, n)[:, None] * f
    raw = rng.negative_binomial(10, 10 / (10 + mu)).astype(np.int64)
    for c in range(C):   # no all-zero condition row (the MLE has no root)
        first = np.flatnonzero(cond == c)[0]
        raw[raw[:, cond == c].sum(axis=1) == 0, first] = 1
    dist = rng.integers(0, 50, n).astype(np.int32)
    tab = rng.uniform(0.01, 0.3, (50, C))
    p, llr, m0, m1, _ = ctx.lrt(raw, f, dist, tab, cond, refit_mu=refit)
    disp_wide = np.dot(tab[dist], design.T)
    rp, rllr, rm0, rm1 = oracle.lrt(raw, f, disp_wide, design, refit_mu=refit)
    assert rel_err(p, rp) < RTOL_PQ
    # llr is a difference of two R-term sums: near 0 its error is absolute
    # (the MLE tolerance times the slope), measured 7e-14 at |llr| 4e-7
    np.testing.assert_allclose(llr, rllr, rtol=1e-7, atol=1e-10)
    tol = RTOL_MU if refit else 1e-14
    assert rel_err(m0, rm0) < tol
    assert rel_err(m1, rm1) < tol
    # lrt.py's own (n, R) dispersion argument: the same numbers, bit for bit
    wp, wllr, wm0, wm1 = ctx.lrt_wide(raw, f, disp_wide, cond, C,
                                      refit_mu=refit)
    np.testing.assert_array_equal(wp, p)
    np.testing.assert_array_equal(wllr, llr)
    np.testing.assert_array_equal(wm1, m1)


@pytest.mark.parametrize('name', ['small2', 'c3r9', 'r18c3', 'r16c2'])
def test_union_and_size_factors_vs_reference(ctx, name):
    g, kw = e2e_inputs(name)
    for c in kw['chroms']:
        bias = oracle.load_bias([p.replace('<chrom>', c)
                                 for p in kw['bias_patterns']])
        mats = []
        for p in kw['raw_npz_patterns']:
            m = sparse.load_npz(p.replace('<chrom>', c)).tocsr()
            m.sum_duplicates()
            mats.append(m)
        row, col, raw, bal = ctx.sparse_union(mats, bias,
                                              kw['dist_thresh_max'])
        np.testing.assert_array_equal(row, g['row__%s' % c])
        np.testing.assert_array_equal(col, g['col__%s' % c])
        np.testing.assert_array_equal(raw, g['raw__%s' % c])
        nb = int(kw['dist_thresh_max'] / 5)
        sf = ctx.size_factors_cmor(bal, col - row, nb)
        assert rel_err(sf, g['size_factors__%s' % c]) < 1e-13
        sf0 = ctx.size_factors_cmor(bal, col - row, 0)
        assert rel_err(sf0, oracle.conditional_mor(bal, col - row)) < 1e-13


def test_disp_and_lrt_vs_oracle_larger(ctx):
    """A 900-bin synthetic chromosome: GPU vs the CPU oracle end to end from
    the same prepared inputs (the oracle finishes in seconds)."""
    import tempfile
    from hic3defdr_amd import synthetic, _native
    with tempfile.TemporaryDirectory() as tmp:
        kw = synthetic.write_dataset(tmp, {'chrX': 900}, dist_thresh_max=80,
                                     seed=7)
        design = kw['design']
        chrom = 'chrX'
        npz = [p.replace('<chrom>', chrom) for p in kw['raw_npz_patterns']]
        bfs = [p.replace('<chrom>', chrom) for p in kw['bias_patterns']]
        prep = oracle.prepare_chrom(npz, bfs, design, dist_thresh_max=80)
        bias = oracle.load_bias(bfs)
        di = prep['disp_idx']
        row, col = prep['row'][di], prep['col'][di]
        raw = prep['raw'][di]
        f = bias[row] * bias[col] * prep['size_factors'][di]
        dist = col - row
        disp, dpd, _ = oracle.estimate_disp([prep], [bias], design,
                                            dist_thresh_max=80)
        out = ctx.disp_per_dist(raw, f, dist, design.argmax(axis=1), 2, 81)
        np.testing.assert_allclose(out, dpd, rtol=RTOL_DISP, atol=1e-12)
        tab = np.stack([_native.disp_table(out[:, c]) for c in range(2)],
                       axis=1)
        p, llr, m0, m1, d = ctx.lrt(raw, f, dist, tab, design.argmax(axis=1))
        rp, _, rm0, rm1 = oracle.lrt(raw, f, np.dot(disp, design.T), design)
        assert rel_err(p, rp) < RTOL_PQ
        assert rel_err(m0, rm0) < RTOL_MU


def test_disp_dev_with_noop_reduce_matches_single_rank(ctx):
    """The multi-rank branch of the device driver (per-pass k_disp_work NLL
    sums, k_seg_reduce, the reduce hook on the ctx stream, k_seg_update
    step=1, termination on the live-segment count) with an identity
    all-reduce vs the single-rank driver (k_brent): same dispersions, both
    deterministic."""
    import torch
    from hic3defdr_amd import _native
    g, kw, raw, f, dist = _stage_inputs('small2')
    design = kw['design']
    C, D = design.shape[1], kw['dist_thresh_max'] + 1
    cond = design.argmax(axis=1)
    dev = torch.device('cuda', 0)
    t_raw = torch.from_numpy(raw.astype(np.int32)).to(dev).contiguous()
    t_f = torch.from_numpy(f).to(dev).contiguous()
    t_d = torch.from_numpy(dist.astype(np.int32)).to(dev).contiguous()
    torch.cuda.synchronize()
    calls = []

    def noop(ptr, count):
        calls.append(count)

    args = (t_raw.data_ptr(), t_f.data_ptr(), t_d.data_ptr(), len(raw),
            raw.shape[1], cond, C, D)
    one = ctx.disp_per_dist_dev(*args)      # in-kernel Brent (k_brent)
    multi = ctx.disp_per_dist_dev(*args, reduce=noop)
    assert len(calls) > 10
    again = ctx.disp_per_dist_dev(*args, reduce=noop)
    np.testing.assert_array_equal(multi, again)   # deterministic
    np.testing.assert_array_equal(one, ctx.disp_per_dist_dev(*args))
    # the two drivers sum the NLL terms in different orders
    np.testing.assert_allclose(one, multi, rtol=1e-7, atol=1e-12)
    np.testing.assert_allclose(multi, g['disp_per_dist'], rtol=RTOL_DISP,
                               atol=1e-12)


@pytest.mark.parametrize('case', ['random', 'ties', 'nan', 'one', 'allnan',
                                  'empty', 'large'])
def test_bh_gpu_bit_identical(ctx, case):
    """h3d_bh_ctx (GPU radix sort + min-scan) == h3d_bh (host) == the
    oracle's statsmodels fdrcorrection restatement, bit for bit."""
    from hic3defdr_amd import _native
    rng = np.random.default_rng(7)
    p = {'random': rng.random(10007),
         'ties': np.round(rng.random(5000), 2),
         'nan': np.where(rng.random(3000) < 0.2, np.nan, rng.random(3000)),
         'one': np.array([0.3]),
         'allnan': np.full(17, np.nan),
         'empty': np.empty(0),
         'large': rng.random(3_000_000) ** 3}[case]
    q = ctx.bh(p)
    np.testing.assert_array_equal(q, _native.bh(p))
    np.testing.assert_array_equal(q, oracle.adjust_pvalues(p))


def test_union_whole_matrix_keeps_only_the_band(ctx):
    """Whole-chromosome CSRs (entries at every distance, both triangles,
    explicit zeros, zero-bias bins): only in-band entries are staged on the
    device, and the union equals the reference's
    wipe_distances + sum (oracle.sparse_union)."""
    rng = np.random.default_rng(11)
    n_bins, R, dmax = 400, 3, 12
    mats = []
    for r in range(R):
        m = sparse.random(n_bins, n_bins, density=0.08, random_state=r + 1,
                          data_rvs=lambda k: rng.integers(0, 6, k)).tocsr()
        m.sort_indices()
        mats.append(m)
    bias = np.exp(rng.normal(0, 0.2, (n_bins, R)))
    bias[rng.random((n_bins, R)) < 0.03] = 0.0
    row, col, raw, bal = ctx.sparse_union(mats, bias, dmax)
    with np.errstate(divide='ignore', invalid='ignore'):
        rr, rc = oracle.sparse_union(mats, dist_thresh=dmax,
                                     bias=bias.copy())
    np.testing.assert_array_equal(row, rr)
    np.testing.assert_array_equal(col, rc)
    dense = np.stack([m.toarray()[row, col] for m in mats], axis=1)
    # the reference gathers raw at every union pixel whatever the replicate's
    # bias there (analysis.py:91-101): counts on zero-bias bins stay, and
    # balanced is v / 0 = inf (or 0 / 0 = nan) exactly as numpy divides
    np.testing.assert_array_equal(raw, dense)
    with np.errstate(divide='ignore', invalid='ignore'):
        bal_ref = dense / (bias[row] * bias[col])
    np.testing.assert_array_equal(bal, bal_ref)
    assert np.any(np.isinf(bal)) and np.any(bias[row] * bias[col] == 0)
    assert np.all((col - row >= 0) & (col - row <= dmax))

