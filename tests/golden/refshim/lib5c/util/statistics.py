import numpy as np
from statsmodels.stats.multitest import multipletests


def adjust_pvalues(pvalues, method='fdr_bh'):
    q = np.ones_like(pvalues, dtype=float) * np.nan
    idx = np.isfinite(pvalues)
    if idx.any():
        q[idx] = multipletests(pvalues[idx], method=method)[1]
    return q
