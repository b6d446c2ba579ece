"""Classification (reference hic3defdr/util/classification.py)."""
import numpy as np

from hic3defdr_amd.util.clusters import ClusterList, pixel_in


def classify_clusters(row, col, value, clusters):
    """``ClusterList`` form of ``classify`` (classification.py:7-49): the
    pixels of ``clusters`` (matched against (row, col)) get the class
    argmax(value[pixel]) (first maximum; NaN wins as in np.argmax), then each
    class's pixels are re-clustered in (row, col) order. Returns one
    ``ClusterList`` per column of ``value``."""
    row = np.asarray(row, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    value = np.asarray(value)
    if not isinstance(clusters, ClusterList):
        clusters = ClusterList.from_sets(clusters)
    pr, pc = clusters.pixels()
    idx = pixel_in(row, col, pr, pc)
    classes = np.argmax(value[idx, :], axis=1) if idx.any() else \
        np.zeros(0, dtype=np.int64)
    r, c = row[idx], col[idx]
    return [ClusterList.find(r[classes == k], c[classes == k])
            for k in range(value.shape[1])]


def classify(row, col, value, clusters):
    """Reference ``classification.py:7-49``: list (per class) of lists of
    sets of (i, j)."""
    return [cl.to_sets() for cl in classify_clusters(row, col, value,
                                                     clusters)]
