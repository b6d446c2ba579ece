"""The device numerics (csrc/h3d_special.h, h3d_model.h) vs scipy / the
oracle / reference goldens, through two builds of the same source behind one
test ABI (h3dt_*):

- ``host``:   g++ (libh3d_hosttest.so), runs on the CPU;
- ``gfx950``: hipcc for gfx950 (libh3d_selftest.so, csrc/h3d_selftest.hip):
  every call runs the device code in a kernel on the MI355X -- OCML
  exp/log, the contracted NLL lgamma -- so the unit goldens hold the
  kernels' own numerics (marked gpu).

Same tolerances for both."""
import ctypes
import os

import numpy as np
import pytest
import scipy.special as sc

import oracle
from conftest import golden, rel_err

from hic3defdr_amd import build as h3dbuild

D = ctypes.POINTER(ctypes.c_double)
I = ctypes.POINTER(ctypes.c_int32)


@pytest.fixture(scope='module',
                params=['host', pytest.param('gfx950', marks=pytest.mark.gpu)])
def lib(request):
    if request.param == 'host':
        return ctypes.CDLL(h3dbuild.build_hosttest())
    # one HIP runtime per process: torch's first, as _native.load_library
    # does (the selftest library loaded first leaves torch without devices
    # for the GPU tests that run after this module)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    # prebuilt in-tree by build() (the GPU box does not compile)
    path = os.path.join(h3dbuild.LIBDIR, 'libh3d_selftest.so')
    if not os.path.exists(path):
        raise RuntimeError('libh3d_selftest.so missing: run build()')
    lib = ctypes.CDLL(path)
    assert lib.h3dt_device_ok() == 1, 'no HIP device for the gfx950 self-test'
    return lib


def _p(a, t=D):
    return a.ctypes.data_as(t)


def unary(lib, name, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    getattr(lib, 'h3dt_' + name)(ctypes.c_int64(x.size), _p(x), _p(out))
    return out


def binary(lib, name, a, x):
    a = np.ascontiguousarray(a, dtype=np.float64)
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    getattr(lib, 'h3dt_' + name)(ctypes.c_int64(x.size), _p(a), _p(x), _p(out))
    return out


def igam_err(got, ref, a, x):
    """Largest error of an incomplete-gamma value in units of its tolerance
    1e-12 + 2 ulp x |a ln x| + |x| + |lgamma a|: the regularised prefactor
    exp(a ln x - x - lgamma a) turns the rounding of that exponent (~1e4 at a
    = 2e3) into relative error, for scipy's evaluation as much as for this
    one, so two correct libms (glibc on the host, OCML on gfx950) differ by
    that much (measured on gfx950: 1.8e-12 at a ~ 2e3)."""
    got, ref = np.asarray(got), np.asarray(ref)
    with np.errstate(all='ignore'):
        scale = np.abs(a * np.log(x)) + np.abs(x) + np.abs(sc.gammaln(a))
        tol = 1e-12 + 2 * 2.2e-16 * np.where(np.isfinite(scale), scale, 0)
        err = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300)
    err[(got == ref) | (np.isnan(got) & np.isnan(ref))] = 0
    return float(np.max(err / tol))


def test_special_vs_reference_goldens(lib):
    g = golden('unit_special.npz')
    a, x, p = g['a'], g['x'], g['p']
    assert igam_err(binary(lib, 'igam', a, x), g['gammainc'], a, x) < 1
    assert igam_err(binary(lib, 'igamc', a, x), g['gammaincc'], a, x) < 1
    assert rel_err(binary(lib, 'igami', a, p), g['gammaincinv']) < 1e-11
    assert rel_err(binary(lib, 'igamci', a, p), g['gammainccinv']) < 1e-11
    assert rel_err(unary(lib, 'ndtr', g['z']), g['ndtr']) < 1e-13
    assert rel_err(unary(lib, 'ndtri', g['pq']), g['ndtri']) < 1e-13
    assert rel_err(unary(lib, 'lgam', g['g']), g['gammaln']) < 1e-14
    df1 = binary(lib, 'chi2_sf', np.ones_like(g['llr']), -2 * g['llr'])
    df2 = binary(lib, 'chi2_sf', 2 * np.ones_like(g['llr']), -2 * g['llr'])
    assert rel_err(df1, g['chi2_sf_df1']) < 1e-12
    assert rel_err(df2, g['chi2_sf_df2']) < 1e-12


def test_special_dense_grids(lib):
    rng = np.random.default_rng(3)
    # shapes/arguments met in q2qnbinom: a = mu/(1+alpha mu) in [1e-3, 2e3]
    a = np.concatenate([10 ** rng.uniform(-3, 3.3, 20000)])
    x = a * np.exp(rng.normal(0, 0.5, a.size))
    assert igam_err(binary(lib, 'igam', a, x), sc.gammainc(a, x), a, x) < 1
    assert igam_err(binary(lib, 'igamc', a, x), sc.gammaincc(a, x), a, x) < 1
    q = np.clip(rng.uniform(0, 1, a.size) ** 4, 1e-300, 1 - 1e-16)
    assert rel_err(binary(lib, 'igami', a, q), sc.gammaincinv(a, q)) < 1e-11
    assert rel_err(binary(lib, 'igamci', a, q), sc.gammainccinv(a, q)) < 1e-11
    z = rng.uniform(-37, 8, 20000)
    assert rel_err(unary(lib, 'ndtr', z), sc.ndtr(z)) < 1e-13
    pq = np.concatenate([10 ** rng.uniform(-307, -0.3, 20000),
                         rng.uniform(0, 1, 20000)])
    assert rel_err(unary(lib, 'ndtri', pq), sc.ndtri(pq)) < 1e-13
    v = np.concatenate([10 ** rng.uniform(-3, 6, 20000),
                        rng.uniform(0.01, 40, 20000)])
    assert rel_err(unary(lib, 'lgam', v), sc.gammaln(v)) < 1e-14
    s = rng.uniform(-0.49, 2, 5000)
    # gammaln(1 + s) itself cancels near s = 0, 1: compare absolutely (the
    # cephes Taylor series stops at n = 41: ~1e-14 at |s| = 0.5, as scipy)
    assert np.max(np.abs(unary(lib, 'lgam1p', s) - sc.gammaln(1 + s))) < 5e-14


def test_igam_plain_prefactor_near_the_mode(lib):
    """igam_fac_l forms x^a e^-x / Gamma(a) by the plain exponent for every
    a < 50 (csrc/h3d_special.h), also where |x - a| <= 0.4 a and cephes
    (scipy, the reference's igam) switches to the log1pmx / Stirling form at
    a > 10: there the exponent's rounding becomes relative error of a well
    conditioned value. A deliberate trade, pinned: at a in [10, 50) near the
    mode within 3e-13 relative of scipy (measured 8e-14 on the host), above
    a = 50 (the log1pmx form) within 1e-13 (measured 2.8e-14)."""
    rng = np.random.default_rng(7)
    for lo, hi, bar in ((10.0, 50.0, 3e-13), (50.0, 200.0, 1e-13)):
        a = rng.uniform(lo, hi, 40000)
        x = a * (1 + rng.uniform(-0.4, 0.4, a.size))
        assert rel_err(binary(lib, 'igam', a, x), sc.gammainc(a, x)) < bar
        assert rel_err(binary(lib, 'igamc', a, x), sc.gammaincc(a, x)) < bar


def test_fit_mu_vs_goldens(lib):
    g = golden('unit_nb.npz')
    x = np.ascontiguousarray(g['fmh_x'], dtype=np.int32)
    b = np.ascontiguousarray(g['fmh_b'])
    for al, ref in ((g['fmh_alpha'], g['fmh_mu']),
                    (np.full(b.shape, 0.05), g['fmh_mu_scalar_alpha'])):
        al = np.ascontiguousarray(al)
        mu = np.empty(len(x))
        st = lib.h3dt_fit_mu(ctypes.c_int64(len(x)), 4, _p(x, I), _p(b),
                             _p(al), _p(mu))
        assert st == 0
        assert rel_err(mu, ref) < 1e-9


def test_fit_mu_is_converged_to_full_precision(lib):
    """fit_mu's Halley steps stop once a step is <= 1e-5 in log mu (cubic
    convergence: ~1e-15 after it). The root of the score S(mu)
    (scaled_nb.py:143-147) must lie within 1e-12 relative of the returned
    mu, over counts from 0 to 1e5, dispersions 1e-6 .. 10 and size factors
    1e-3 .. 1e3 (some replicates zero)."""
    rng = np.random.default_rng(5)
    n = 40000
    lam = 10 ** rng.uniform(-1, 5, (n, 1))
    b = 10 ** rng.uniform(-1.5, 1.5, (n, 4)) * 10 ** rng.uniform(-1.5, 1.5, (n, 1))
    al = 10 ** rng.uniform(-6, 1, (n, 4))
    x = rng.poisson(lam * b).astype(np.int32)
    x[rng.random((n, 4)) < 0.1] = 0
    x[x.sum(1) == 0, 0] = 1
    mu = np.empty(n)
    st = lib.h3dt_fit_mu(ctypes.c_int64(n), 4, _p(x, I), _p(b), _p(al), _p(mu))
    assert st == 0 and np.all(mu > 0)
    # a pixel whose only non-zero replicate has a far smaller dispersion
    # than the zero ones can have S > 0 for every mu (the MLE at infinity)
    fin = np.isfinite(mu)
    assert fin.sum() >= n - 5
    x, b, al, mu = x[fin], b[fin], al[fin], mu[fin]

    def score(m):
        mb = m[:, None] * b
        return ((x - mb) / (m[:, None] + al * m[:, None] * mb)).sum(1)
    lo, hi = score(mu * (1 - 1e-12)), score(mu * (1 + 1e-12))
    # S decreases through the root: S(mu (1 - eps)) >= 0 >= S(mu (1 + eps))
    assert np.all(lo >= 0) and np.all(hi <= 0)


def test_nll_term_forms_agree(lib):
    """The Brent kernels' NLL term (dispersion.py:67-70) by its general form
    and by the mid (r >= 10: no shift products) and large (r >= 20: 5-term
    Stirling) forms: within 1e-14 of the term's largest lgamma of each other
    and of scipy's gammaln (the term is a difference of lgammas)."""
    from scipy.special import gammaln
    rng = np.random.default_rng(11)
    for r in (2, 4):
        pd = np.ascontiguousarray(np.concatenate([
            rng.gamma(0.7, 3.0, (4000, r)), rng.gamma(2.0, 60.0, (4000, r)),
            np.zeros((50, r))]))
        n = len(pd)
        for delta, modes in ((0.09, (0, 1)), (0.0476, (0, 1, 2)),
                             (0.01, (0, 1, 2)), (0.3, (0,))):
            rr = 1.0 / delta - 1.0
            want = (gammaln(pd + rr).sum(1) + gammaln(r * rr)
                    - gammaln(pd.sum(1) + r * rr) - r * gammaln(rr))
            got = {}
            for m in modes:
                out = np.empty(n)
                assert lib.h3dt_nll_terms(ctypes.c_int64(n), r, _p(pd),
                                          ctypes.c_double(delta), m, _p(out)) == 0
                got[m] = out
                scale = np.maximum(1.0, gammaln(pd.sum(1) + r * rr))
                err = np.max(np.abs(out - want) / scale)
                assert err < 1e-14, (r, delta, m, err)
            for m in modes[1:]:
                assert np.max(np.abs(got[m] - got[0]) / scale) < 1e-14


def test_fit_mu_doctest_brentq_case(lib):
    """scaled_nb.py:129-137: the second pixel needs the brentq fallback."""
    x = np.array([[2, 3, 4, 2], [6, 9, 3, 1]], dtype=np.int32)
    b = np.array([[0.45, 0.53, 0.088, 0.091], [0.70, 0.83, 0.14, 0.15]])
    al = np.array([[0.0071, 0.0071, 0.0073, 0.0073],
                   [0.0070, 0.0070, 0.0072, 0.0072]])
    mu = np.empty(2)
    lib.h3dt_fit_mu(ctypes.c_int64(2), 4, _p(x, I), _p(b), _p(al), _p(mu))
    np.testing.assert_allclose(mu, [9.5900971, 10.45962955], rtol=1e-8)


def test_q2q_vs_goldens(lib):
    g = golden('unit_nb.npz')
    out = np.empty_like(g['q2q_x'])
    lib.h3dt_q2q(ctypes.c_int64(out.size), _p(np.ascontiguousarray(g['q2q_x'])),
                 _p(np.ascontiguousarray(g['q2q_mu_in'])),
                 _p(np.ascontiguousarray(g['q2q_mu_out'])),
                 _p(np.ascontiguousarray(g['q2q_alpha'])), _p(out))
    # x = 0 with both means clamped maps to 0 +- 1e-17 rounding noise
    np.testing.assert_allclose(out, g['q2q'], rtol=1e-10, atol=1e-12)


def test_equalize_and_qcml_vs_goldens(lib):
    g = golden('unit_nb.npz')
    lib.h3dt_qcml.restype = ctypes.c_double
    for s in range(int(g['n_segs'])):
        data = np.ascontiguousarray(g['seg%d_data' % s], dtype=np.int32)
        f = np.ascontiguousarray(g['seg%d_f' % s])
        n, r = data.shape
        out = np.empty((n, r))
        st = lib.h3dt_equalize(ctypes.c_int64(n), r, _p(data, I), _p(f),
                               ctypes.c_double(0.02), _p(out))
        assert st == 0
        np.testing.assert_allclose(out, g['seg%d_equalize' % s], rtol=1e-9,
                                   atol=1e-12)
        stat = ctypes.c_int(0)
        q = lib.h3dt_qcml(ctypes.c_int64(n), r, _p(data, I), _p(f),
                          ctypes.byref(stat))
        assert stat.value == 0
        np.testing.assert_allclose(q, g['seg%d_qcml' % s], rtol=1e-6,
                                   atol=1e-10)


def test_lrt_vs_goldens(lib):
    g = golden('unit_nb.npz')
    raw = np.ascontiguousarray(g['lrt_raw'], dtype=np.int32)
    f = np.ascontiguousarray(g['lrt_f'])
    disp = np.ascontiguousarray(g['lrt_disp'])
    cor = np.ascontiguousarray(g['lrt_design'].argmax(axis=1), dtype=np.int32)
    n = len(raw)
    for pre, refit in (('lrt', 1), ('lrtnr', 0)):
        p, llr, m0 = np.empty(n), np.empty(n), np.empty(n)
        m1 = np.empty((n, 2))
        st = lib.h3dt_lrt(ctypes.c_int64(n), 4, 2, _p(raw, I), _p(f), _p(disp),
                          _p(cor, I), refit, _p(p), _p(llr), _p(m0), _p(m1))
        assert st == 0
        assert rel_err(p, g[pre + '_p']) < 1e-7
        assert rel_err(m0, g[pre + '_mu0']) < 1e-9
        assert rel_err(m1, g[pre + '_mu1']) < 1e-9


def test_lrt_vs_oracle_r9c3(lib):
    rng = np.random.default_rng(9)
    n, R, C = 500, 9, 3
    design = np.zeros((R, C), dtype=bool)
    design[np.arange(R), np.arange(R) // 3] = True
    mu = 10 ** rng.uniform(0, 2.5, n)
    f = np.exp(rng.normal(0, 0.3, (n, R)))
    disp = np.repeat(10 ** rng.uniform(-2, -0.5, (n, C)), 3, axis=1)
    raw = rng.negative_binomial(1 / disp, 1 / (1 + disp * mu[:, None] * f))
    for c in range(C):
        raw[raw[:, design[:, c]].sum(axis=1) == 0, 3 * c] = 1
    rp, rllr, rm0, rm1 = oracle.lrt(raw, f, disp, design)
    raw32 = np.ascontiguousarray(raw, dtype=np.int32)
    cor = np.ascontiguousarray(design.argmax(axis=1), dtype=np.int32)
    p, llr, m0, m1 = np.empty(n), np.empty(n), np.empty(n), np.empty((n, C))
    st = lib.h3dt_lrt(ctypes.c_int64(n), R, C, _p(raw32, I), _p(f),
                      _p(np.ascontiguousarray(disp)), _p(cor, I), 1, _p(p),
                      _p(llr), _p(m0), _p(m1))
    assert st == 0
    assert rel_err(p, rp) < 1e-7
    assert rel_err(m1, rm1) < 1e-9


def test_lrt_llr_against_long_double(lib):
    """llr = sum(null logpmf row) - sum(alt logpmf row) (lrt.py:42-48) as the
    rows' difference term by term (one log per replicate): against a
    long-double evaluation of the rows at the product's own MLEs it is within
    5e-12 absolute (measured 1.1e-12; numpy's row sums, the reference's
    form, carry ~8.5e-12 of cancellation)."""
    rng = np.random.default_rng(3)
    n, R, C = 20000, 4, 2
    design = np.zeros((R, C), dtype=bool)
    design[np.arange(R), np.arange(R) // 2] = True
    mu = 10 ** rng.uniform(0, 3, n)
    f = np.exp(rng.normal(0, 0.3, (n, R)))
    disp = np.repeat(10 ** rng.uniform(-2, -0.5, (n, C)), 2, axis=1)
    raw = rng.negative_binomial(1 / disp, 1 / (1 + disp * mu[:, None] * f))
    for c in range(C):
        raw[raw[:, design[:, c]].sum(axis=1) == 0, 2 * c] = 1
    raw32 = np.ascontiguousarray(raw, dtype=np.int32)
    cor = np.ascontiguousarray(design.argmax(axis=1), dtype=np.int32)
    p, llr, m0, m1 = np.empty(n), np.empty(n), np.empty(n), np.empty((n, C))
    assert lib.h3dt_lrt(ctypes.c_int64(n), R, C, _p(raw32, I), _p(f),
                        _p(np.ascontiguousarray(disp)), _p(cor, I), 1, _p(p),
                        _p(llr), _p(m0), _p(m1)) == 0
    L = np.longdouble
    x, ff, r = raw.astype(L), f.astype(L), 1 / disp.astype(L)
    a0 = m0.astype(L)[:, None] * ff
    a1 = m1.astype(L)[:, cor] * ff
    want = ((x * np.log(a0) - (r + x) * np.log(r + a0)).sum(1)
            - (x * np.log(a1) - (r + x) * np.log(r + a1)).sum(1))
    assert np.max(np.abs(llr - want.astype(float))) < 5e-12


def test_log1pmx_fixed_length_form(lib):
    # the atanh form replaces cephes' convergent Taylor loop on |x| < 0.5;
    # reference: log1p(x) - x in extended precision via the series itself
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(-0.4999, 0.4999, 20000),
                        10 ** rng.uniform(-12, -0.31, 5000),
                        -(10 ** rng.uniform(-12, -0.31, 5000))])
    ref = np.array([float(sum((-1) ** (n + 1) * np.longdouble(v) ** n / n
                              for n in range(2, 200)))
                    for v in x[:3000]])
    got = unary(lib, 'log1pmx', x)
    assert rel_err(got[:3000], ref) < 4e-16 * 8
    big = np.abs(x) > 1e-3  # where log1p(x) - x itself is still accurate
    assert rel_err(got[big], np.log1p(x[big]) - x[big]) < 1e-10


def test_lgam_nll_and_log_fast(lib):
    # the NLL-sum lgamma: absolute error bound (each term joins a sum of
    # thousands), checked against scipy gammaln over the NLL argument range
    # d + r, r = 1/delta - 1 in [0.0101, 9999]
    rng = np.random.default_rng(11)
    x = np.concatenate([10 ** rng.uniform(np.log10(0.0101), 6, 40000),
                        rng.uniform(0.0101, 14, 40000)])
    got = unary(lib, 'lgam_nll', x)
    ref = sc.gammaln(x)
    # 1.2e-14: the fixed 5/10-step shift (y in [10, 15)) leaves ~3 ulp of
    # (y - 1/2) ln y - ln P ~ 17 where the two cancel near x = 1, 2
    assert np.max(np.abs(got - ref) / np.maximum(1.0, np.abs(ref))) < 1.2e-14
    assert np.isinf(unary(lib, 'lgam_nll', np.array([np.inf])))[0]
    v = 10 ** rng.uniform(-300, 300, 40000)
    # the gfx950 build forms its quotient with v_rcp_f64 + one Newton step
    # (one more ulp); the NLL sums need absolute accuracy only
    assert rel_err(unary(lib, 'log_fast', v), np.log(v)) < 6e-16
