"""Operator-level drop-ins for the reference's dispersion estimators
(hic3defdr/util/dispersion.py): same signatures; computed on the GPU.

- ``qcml(data, f)``: one (distance, condition) segment through the
  estimate_disp device driver (equalize + bounded Brent, k_disp_work /
  k_brent) -- the estimator ``estimate_disp(estimator='qcml')`` calls;
  ``qcml_batch`` runs many segments in one driver call (a single-segment
  call pays the driver's whole setup: sort, tables, launches, polls);
- ``cml(data, f)``: one bounded-Brent search (h3d_cml);
- ``mme_per_pixel`` / ``mme``: the per-pixel method-of-moments kernel.

As in the reference, ``cml`` / ``mme`` / ``mme_per_pixel`` divide ``data``
by ``f`` IN PLACE (dispersion.py:67-68, 101-102, 129-130): float data is
modified, integer data raises numpy's casting error (which is why the
reference's estimate_disp cannot use them on raw counts)."""
import numpy as np

from hic3defdr_amd import _native


def _tol_scope(ctx, tol):
    """The ctx's qcml tolerance set to ``tol`` for one call, restored to
    the estimate_disp default (1e-4) after it."""
    import contextlib

    @contextlib.contextmanager
    def scope():
        ctx.set_qcml_tol(tol)
        try:
            yield
        finally:
            ctx.set_qcml_tol(1e-4)
    return scope()


def qcml(data, f=None, max_iter=10, tol=1e-4):
    """dispersion.py:10-43. ``max_iter`` is accepted and, as in the
    reference (whose loop counter is never incremented), has no effect;
    ``tol``: iterate while |disp - new disp| > tol (the device state
    machine's own tolerance, h3d_set_qcml_tol)."""
    data = np.asarray(data)
    if data.ndim != 2:
        raise ValueError('data must be (pixels, replicates)')
    if data.size and not np.all(data == np.floor(data)):
        raise ValueError('qcml takes integer counts')
    n, r = data.shape
    f = np.ones((n, r)) if f is None else np.broadcast_to(f, (n, r))
    ctx = _native.context()
    with _tol_scope(ctx, tol):
        out = ctx.disp_per_dist(data.astype(np.int64), f,
                                np.zeros(n, np.int32), np.zeros(r, np.int32),
                                1, 1)
    return float(out[0, 0])


def qcml_batch(segments, max_iter=10, tol=1e-4):
    """qcml over many segments in ONE estimate_disp driver call: ``segments``
    is a list of (data, f) pairs as qcml takes them (f may be None); returns
    the list of dispersions, each the qcml of its own pixels -- equal to
    qcml(data, f) up to the summation order of the NLL, which depends on the
    whole call (the gang slice size follows the call's pixel count, and one
    workgroup per segment or gangs are chosen by the live-segment count), so
    a segment can land elsewhere inside Brent's tolerance (xatol 1e-5 in
    delta = disp / (1 + disp)), as the reference itself does under a pixel
    permutation (tests/golden/cfg2_spread.npz). The reference's
    estimate_disp calls qcml once per (distance,
    condition) (analysis.py:198-246 -> dispersion.py:10-43): a caller
    patching that loop gathers its segments first and makes this one call
    instead of several hundred single-segment driver runs."""
    out = [np.nan] * len(segments)
    by_r = {}
    for i, (data, f) in enumerate(segments):
        data = np.asarray(data)
        if data.ndim != 2:
            raise ValueError('data must be (pixels, replicates)')
        if data.size and not np.all(data == np.floor(data)):
            raise ValueError('qcml takes integer counts')
        n, r = data.shape
        f = np.ones((n, r)) if f is None else np.broadcast_to(f, (n, r))
        by_r.setdefault(r, []).append((i, data, f))
    ctx = _native.context()
    for r, group in by_r.items():
        # one pseudo-distance per segment, one condition of r replicates
        raw = np.concatenate([d for _, d, _ in group]).astype(np.int64)
        ff = np.concatenate([f for _, _, f in group]).astype(np.float64)
        dist = np.concatenate([np.full(len(d), j, np.int32)
                               for j, (_, d, _) in enumerate(group)])
        with _tol_scope(ctx, tol):
            res = ctx.disp_per_dist(raw.reshape(-1, r), ff.reshape(-1, r),
                                    dist, np.zeros(r, np.int32), 1,
                                    len(group))
        for j, (i, _, _) in enumerate(group):
            out[i] = float(res[j, 0])
    return out


def cml(data, f=None):
    """dispersion.py:46-80."""
    if f is not None:
        data /= f   # in place, as the reference
    return _native.context().cml(np.asarray(data, dtype=np.float64))


def mme_per_pixel(data, f=None):
    """dispersion.py:83-105."""
    if f is not None:
        data /= f
    data = np.asarray(data, dtype=np.float64)
    ctx = _native.context()
    return ctx.mme_per_pixel(data, None, np.zeros(data.shape[1], np.int32),
                             1)[:, 0]


def mme(data, f=None):
    """dispersion.py:108-131."""
    if f is not None:
        data /= f
    return np.nanmean(mme_per_pixel(data))
