"""Restatement of statsmodels' lowess (``statsmodels.nonparametric.
_smoothers_lowess``, Cleveland 1979), the smoother that lib5c's ``lowess``
wraps (reference ``hic3defdr/util/lowess.py:72``). TEST INFRASTRUCTURE ONLY.

statsmodels is not installed in the product interpreter; its algorithm
(statsmodels 0.12.2, the version the goldens were made with) is restated
here: local linear fits with tricube distance weights over the k = int(frac*n
+ 1e-10) nearest neighbours, ``delta`` skipping with linear interpolation,
tie copying, and ``it`` bisquare robustness iterations on 6*median|resid|.
Pinned by ``tests/golden/unit_lowess.npz`` (lo*_res).
"""
import numpy as np


def _cube(v):
    return v * (v * v)


def _tricube(t):
    # bit-exact with statsmodels: in-place cube, 1 - ., clip, cube
    return _cube(np.maximum(1 - _cube(np.abs(t)), 0.0))


def _bisquare(t):
    t = np.abs(t)
    out = np.zeros_like(t)
    m = t < 1
    out[m] = (1 - t[m] ** 2) ** 2
    return out


def lowess_sorted(y, x, frac=2. / 3, it=3, delta=0.0):
    """x sorted ascending; returns fitted y (same order)."""
    n = x.shape[0]
    k = int(frac * n + 1e-10)
    k = min(max(k, 2), n)
    resid_w = np.ones(n)
    y_fit = np.zeros(n)
    for robiter in range(it + 1):
        y_fit = np.zeros(n)
        i = 0
        last_fit_i = -1
        left_end, right_end = 0, k
        while True:
            xval = x[i]
            while right_end < n and xval > (x[left_end] + x[right_end]) / 2.0:
                left_end += 1
                right_end += 1
            radius = max(xval - x[left_end], x[right_end - 1] - xval)
            xs = x[left_end:right_end]
            w = _tricube(np.abs(xs - xval) / radius) if radius > 0 else \
                np.where(xs == xval, 1.0, 0.0)
            if robiter > 0:
                w = w * resid_w[left_end:right_end]
            sw = np.sum(w)  # numpy pairwise summation, as statsmodels
            if sw <= 0:
                y_fit[i] = y[i]
            else:
                w = w / sw
                swx = 0.0
                for j in range(w.size):
                    swx += w[j] * xs[j]
                sq = 0.0
                for j in range(w.size):
                    sq += w[j] * (xs[j] - swx) ** 2
                acc = 0.0
                for j in range(w.size):
                    p = w[j] * (1.0 + (xval - swx) * (xs[j] - swx) / sq) \
                        if sq > 0 else w[j]
                    acc += p * y[left_end + j]
                y_fit[i] = acc
            if last_fit_i < i - 1:
                a = (x[last_fit_i + 1:i] - x[last_fit_i]) / \
                    (x[i] - x[last_fit_i])
                y_fit[last_fit_i + 1:i] = a * y_fit[i] + \
                    (1.0 - a) * y_fit[last_fit_i]
            last_fit_i = i
            cut = x[i] + delta
            # python for-loop semantics: on exhaustion k keeps the last value
            kk = last_fit_i
            for kk in range(last_fit_i + 1, n):
                if x[kk] > cut:
                    break
                if x[kk] == x[last_fit_i]:
                    y_fit[kk] = y_fit[last_fit_i]
                    last_fit_i = kk
            i = max(kk - 1, last_fit_i + 1)
            if last_fit_i >= n - 1:
                break
        if robiter < it:
            res = y - y_fit
            s = np.median(np.abs(res))
            resid_w = _bisquare(res / (6.0 * s)) if s > 0 else \
                np.where(res == 0, 1.0, 0.0)
    return y_fit


def lowess(endog, exog, frac=2. / 3, it=3, delta=0.0):
    """statsmodels ``lowess(endog, exog, ...)`` with return_sorted=True."""
    y = np.asarray(endog, float)
    x = np.asarray(exog, float)
    m = np.isfinite(x) & np.isfinite(y)
    x, y = x[m], y[m]
    order = np.argsort(x, kind='stable')
    x, y = x[order], y[order]
    return np.column_stack([x, lowess_sorted(y, x, frac, it, delta)])
