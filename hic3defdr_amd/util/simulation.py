"""Simulated differential-loop data (reference hic3defdr/util/simulation.py).

Host code with the reference's random-number semantics -- the legacy global
numpy stream, drawn in the reference's order (one ``np.random.choice`` for
the cluster classes, then one ``negative_binomial`` array per replicate) --
so a seeded simulation reproduces the reference's matrices count for count.
"""
import numpy as np
import scipy.ndimage as ndimage
import scipy.sparse as sparse

from hic3defdr_amd.util.printing import eprint

CLASSES = np.array(['constit', 'up A', 'down A', 'up B', 'down B'], dtype='U7')


def _footprint(rs, cs, r0, c0, shape):
    """The cluster's pixels at weight 1, their 8-neighbourhood ring at 1/2
    (simulation.py:47-53: (mask + dilation(mask)) / 2)."""
    fp = np.zeros(shape, dtype=float)
    fp[rs - r0, cs - c0] = 1
    fp += ndimage.binary_dilation(fp, structure=np.ones((3, 3), dtype=bool))
    return fp / 2


def perturb_cluster(matrix, cluster, effect, respect_zeros=True):
    """Scales the pixels under a cluster footprint by (1 + effect x weight),
    in place (simulation.py:12-67). On a sparse matrix with respect_zeros
    only stored entries change."""
    rs, cs = (np.array(v) for v in zip(*cluster))
    r0, r1 = max(rs.min() - 1, 0), min(rs.max() + 1, matrix.shape[0] - 1)
    c0, c1 = max(cs.min() - 1, 0), min(cs.max() + 1, matrix.shape[1] - 1)
    fp = _footprint(rs, cs, r0, c0, (r1 - r0 + 1, c1 - c0 + 1))
    rsl, csl = slice(r0, r1 + 1), slice(c0, c1 + 1)
    if isinstance(matrix, sparse.spmatrix) and respect_zeros:
        sub = matrix[rsl, csl]
        coo = sub.tocoo()
        delta = sub.toarray() * fp * effect
        matrix[coo.row + r0, coo.col + c0] += delta[coo.row, coo.col]
    else:
        matrix[rsl, csl] += matrix[rsl, csl].toarray() * fp * effect


def _nb_params(mean, var):
    """lib5c freeze_distribution(nbinom, mean, var): n = mean^2 / (var -
    mean), p = mean / var."""
    return mean ** 2 / (var - mean), mean / var


def simulate(row, col, mean, disp_fn, bias, size_factors, clusters, beta=0.5,
             p_diff=0.4, trend='mean', verbose=True):
    """Reference simulation.py:70-204: class labels per cluster, the perturbed
    A / B mean matrices, and a generator of simulated CSR replicates (the
    first half condition A, the second B)."""
    eprint('  assigning cluster classes', skip=not verbose)
    p = [1 - p_diff] + [p_diff / 4] * 4 if isinstance(p_diff, float) \
        else [1 - sum(p_diff)] + list(p_diff)
    classes = np.random.choice(CLASSES, size=len(clusters), p=p)
    pos = mean > 0
    row, col, mean = row[pos], col[pos], mean[pos]
    eprint('  perturbing clusters', skip=not verbose)
    n = bias.shape[0]
    mats = {c: sparse.coo_matrix((mean, (row, col)), shape=(n, n)).tocsr()
            for c in 'AB'}
    effects = {'up A': ('A', beta), 'down A': ('A', -beta),
               'up B': ('B', beta), 'down B': ('B', -beta)}
    for i, cluster in enumerate(clusters):
        if classes[i] in effects:
            which, eff = effects[classes[i]]
            perturb_cluster(mats[which], cluster, eff)
    means = {}
    for c in 'AB':
        coo = mats.pop(c).tocoo()
        assert np.array_equal(coo.row, row) and np.array_equal(coo.col, col)
        assert np.all(coo.data > 0)
        means[c] = coo.data
    eprint('  renaming cluster classes', skip=not verbose)
    classes[(classes == 'up A') | (classes == 'down B')] = 'A'
    classes[(classes == 'up B') | (classes == 'down A')] = 'B'
    n_sim = size_factors.shape[-1]
    half = n_sim // 2
    dist = col - row

    def gen():
        for j in range(n_sim):
            eprint('  biasing and simulating rep %i/%i' % (j + 1, n_sim),
                   skip=not verbose)
            m = means['A'] if j < half else means['B']
            sf = size_factors[j] if size_factors.ndim == 1 \
                else size_factors[dist, j]
            f = bias[row, j] * bias[col, j] * sf
            assert np.all(f > 0)
            bm = m * f
            assert np.all(bm > 0)
            cov = bm if trend == 'mean' else dist
            var = bm + bm ** 2 * disp_fn(cov)   # scaled_nb.mvr
            nb_n, nb_p = _nb_params(bm, var)
            x = np.random.negative_binomial(nb_n, nb_p)
            yield sparse.coo_matrix((x, (row, col)), shape=(n, n)).tocsr()

    return classes, gen()
