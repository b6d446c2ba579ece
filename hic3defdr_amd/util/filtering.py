"""Sparse-bin filtering before balancing (reference
hic3defdr/util/filtering.py:7-72, used by the README's simulation workflow
ahead of kr_balance)."""
import numpy as np
import scipy.sparse as sparse


def filter_sparse_rows_count(matrix, min_nnz=25, k=300):
    """Zeroes (rows and columns of) every bin that has fewer than
    ``min_nnz`` nonzero contacts with its ``k`` nearest upstream bins AND
    fewer than ``min_nnz`` with its ``k`` nearest downstream bins, counted on
    the upper triangle (the reference symmetrises its upper band,
    filtering.py:52-55). CSR input comes back CSR without the wiped entries;
    a dense array is wiped in place of a copy."""
    dense = isinstance(matrix, np.ndarray)
    if min_nnz == 0 or k == 0:
        return matrix.copy()
    m = sparse.coo_matrix(matrix)
    m.sum_duplicates()
    n = m.shape[0]
    off = m.col - m.row
    band = (off >= 1) & (off <= min(n, k)) & (m.data > 0)
    # bin j: contacts (j, j+1..j+k) downstream, (j-k..j-1, j) upstream
    down = np.bincount(m.row[band], minlength=n)
    up = np.bincount(m.col[band], minlength=n)
    wipe = (up < min_nnz) & (down < min_nnz)
    if dense:
        out = matrix.copy()
        out[:, wipe] = 0
        out[wipe, :] = 0
        return out
    keep = sparse.diags([~wipe], [0], dtype=int)
    return keep.dot(sparse.csr_matrix(matrix)).dot(keep)
