"""Operator-level drop-in for the reference's ``hic3defdr.util.lrt.lrt``
(lrt.py:7-50): same signature, arguments and return values, computed by
the fused gfx950 LRT kernel (libh3d h3d_lrt_wide)."""
import numpy as np

from hic3defdr_amd import _native


def lrt(raw, f, disp, design, refit_mu=True):
    """Likelihood ratio test of a common mean across conditions vs one mean
    per condition (negative binomial, dispersion fixed).

    raw, f : (pixels, replicates) counts and scaling factors.
    disp : dispersions broadcastable to raw's shape, as fit_mu_hat accepts
        them (scaled_nb.py:139-147: scalar, (R,), (N, 1) or (N, R)); the
        pipeline passes np.dot(disp, design.T).
    design : (replicates, conditions) boolean; every replicate in exactly one
        condition.
    Returns pvalues, llr, mu_hat_null (N,), mu_hat_alt (N, C).
    Raises H3DError where the reference raises (no MLE: an all-zero pixel;
    non-positive or non-finite disp / f)."""
    raw = np.asarray(raw)
    if raw.ndim != 2:
        raise ValueError('raw must be (pixels, replicates)')
    design = np.asarray(design, dtype=bool)
    if not np.all(design.sum(axis=1) == 1):
        raise ValueError('every replicate must belong to exactly one condition')
    if raw.size and not np.all(raw == np.floor(raw)):
        raise ValueError('raw must hold integer counts')
    dw = np.broadcast_to(np.asarray(disp, dtype=np.float64), raw.shape)
    fw = np.broadcast_to(np.asarray(f, dtype=np.float64), raw.shape)
    ctx = _native.context()
    return ctx.lrt_wide(raw.astype(np.int64), fw, dw,
                        design.argmax(axis=1).astype(np.int32),
                        design.shape[1], refit_mu=refit_mu)
