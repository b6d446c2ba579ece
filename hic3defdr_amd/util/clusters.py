"""Sparse cluster JSON I/O (reference hic3defdr/util/clusters.py).

Format: a JSON list of clusters, each a list of ``[i, j]`` pixel indices.
"""
import json

import numpy as np


def load_clusters(infile):
    """Reference ``clusters.py:176-193``: list of sets of (i, j) tuples."""
    with open(infile, 'r') as handle:
        return [set([tuple(e) for e in cluster]) for cluster in
                json.load(handle)]


def save_clusters(clusters, outfile):
    """Reference ``clusters.py:116-136``."""
    with open(outfile, 'w') as handle:
        json.dump([[[int(i), int(j)] for i, j in cluster]
                   for cluster in clusters], handle)


def pixel_membership(row, col, clusters_lists, n_bins=None):
    """Boolean vector: (row[k], col[k]) in the union of all clusters
    (reference ``analysis.py:117-125``, a Python set lookup per pixel),
    vectorised with 64-bit pixel keys."""
    pixels = set().union(*sum(clusters_lists, []))
    if not pixels or len(row) == 0:
        return np.zeros(len(row), dtype=bool)
    pix = np.array(sorted(pixels), dtype=np.int64)
    base = int(max(pix.max(), int(np.max(row)), int(np.max(col)))) + 1
    keys = np.asarray(row, dtype=np.int64) * base + np.asarray(col, np.int64)
    pk = pix[:, 0] * base + pix[:, 1]
    return np.isin(keys, pk)
