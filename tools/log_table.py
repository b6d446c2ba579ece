"""Generates h3d_special.h's kLogTab (the NLL log_fast table) with numpy's
80-bit long double and checks the scheme's accuracy against it.

    python tools/log_table.py
"""
import numpy as np

LD = np.longdouble


def table():
    rows = []
    half = np.sqrt(LD(0.5))
    for i in range(129):
        mi = LD(0.5) + LD(i) / LD(256)
        c = np.float64(LD(1) / mi)
        lc = -np.log(LD(c))          # ln(1 / c) ~ ln m_i
        if mi < half:               # exponent taken one lower: ln(2 m_i)
            lc = lc + np.log(LD(2))
        rows.append((c, np.float64(lc), mi < half))
    return rows


def log_fast(xs, rows):
    c = np.array([r[0] for r in rows])
    el = np.array([r[1] for r in rows])
    sh = np.array([r[2] for r in rows], dtype=int)
    m, e = np.frexp(xs)
    i = np.floor((m - 0.5) * 256 + 0.5).astype(int)
    t = (m.astype(LD) * c[i].astype(LD) - 1).astype(np.float64)  # fma
    q = 1 / 7
    for k in (-1 / 6, 1 / 5, -1 / 4, 1 / 3, -1 / 2):
        q = q * t + k
    lp = (q.astype(LD) * (t * t) + t).astype(np.float64)
    de = (e - sh[i]).astype(float)
    return de * 6.93147180369123816490e-01 + (
        de * 1.90821492927058770002e-10 + (el[i] + lp))


if __name__ == '__main__':
    rows = table()
    assert sum(r[2] for r in rows) == 54  # kLogTabShifted = 53
    for c, el, _ in rows:
        print('    {%r, %r},' % (float(c), float(el)))
    rng = np.random.default_rng(0)
    for xs in (10 ** rng.uniform(-300, 300, 400000),
               rng.uniform(0.3, 3, 400000)):
        ref = np.log(xs.astype(LD))
        err = np.abs(log_fast(xs, rows) - ref)
        rel = np.where(ref != 0, err / np.abs(ref), err)
        print('# max abs %.3g, max rel %.3g' % (err.max(), rel.max()))
