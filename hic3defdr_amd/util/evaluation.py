"""Evaluation of q-values against simulated truth (reference
hic3defdr/util/evaluation.py:15-100)."""
import numpy as np

from hic3defdr_amd.util.clusters import pixel_membership


def make_y_true(row, col, clusters, labels):
    """True for pixels inside a cluster whose label is not 'constit'
    (evaluation.py:15-41); vectorised pixel-key membership."""
    labels = np.asarray(labels)
    sig = [c for c, lab in zip(clusters, labels) if lab != 'constit']
    return pixel_membership(np.asarray(row), np.asarray(col), [sig])


def compute_fdr(y_true, y_pred):
    """fp / (fp + tp) (evaluation.py:82-100)."""
    y_true = np.asarray(y_true, dtype=bool)
    y_pred = np.asarray(y_pred, dtype=bool)
    fp = np.count_nonzero(y_pred & ~y_true)
    tp = np.count_nonzero(y_pred & y_true)
    return fp / float(fp + tp)


def evaluate(y_true, qvalues, n_fdr_points=100):
    """ROC (sklearn roc_curve on 1 - q, as the reference) plus the observed
    FDR at about ``n_fdr_points`` thresholds (evaluation.py:44-79). The FDR
    points are counted for all thresholds at once from one sort of the
    scores instead of a confusion matrix per threshold."""
    from sklearn.metrics import roc_curve
    y_true = np.asarray(y_true, dtype=bool)
    y_pred = 1 - np.asarray(qvalues)
    fpr, tpr, thresh = roc_curve(y_true, y_pred)
    if len(thresh) and np.isinf(thresh[0]):
        # scikit-learn >= 1.3 opens the curve at +inf; the reference's
        # scikit-learn (0.24, the version its outputs were produced with)
        # at the largest score + 1 -- kept, so eval.npz files compare
        thresh = thresh.copy()
        thresh[0] = thresh[1] + 1 if len(thresh) > 1 else 1.0
    fdr = np.ones_like(fpr) * np.nan
    rate = max(int(len(thresh) / n_fdr_points), 1)
    idx = np.arange(np.argmax(tpr > 0), len(thresh), rate)
    if idx.size:
        order = np.sort(y_pred)
        pos = np.sort(y_pred[y_true])
        # predicted positive at threshold t: y_pred >= t
        n_pred = len(order) - np.searchsorted(order, thresh[idx], side='left')
        tp = len(pos) - np.searchsorted(pos, thresh[idx], side='left')
        fdr[idx] = (n_pred - tp) / (n_pred).astype(float)
    return fdr, fpr, tpr, thresh
