"""Thresholding (reference hic3defdr/util/thresholding.py)."""
import numpy as np

from hic3defdr_amd.util.clusters import ClusterList


def threshold_clusters(qvalues, row, col, fdr):
    """``ClusterList`` form of ``threshold_and_cluster``: pixels with
    q < fdr and with q >= fdr (NaN in neither), each clustered in pixel
    order (thresholding.py:7-41)."""
    q = np.asarray(qvalues)
    row = np.asarray(row)
    col = np.asarray(col)
    sig = q < fdr
    insig = q >= fdr
    return (ClusterList.find(row[sig], col[sig]),
            ClusterList.find(row[insig], col[insig]))


def threshold_and_cluster(qvalues, row, col, fdr):
    """Reference ``thresholding.py:7-41``: lists of sets of (i, j)."""
    sig, insig = threshold_clusters(qvalues, row, col, fdr)
    return sig.to_sets(), insig.to_sets()


def size_filter(clusters, cluster_size):
    """Reference ``thresholding.py:44-61``."""
    if isinstance(clusters, ClusterList):
        return clusters.size_filter(cluster_size)
    return [c for c in clusters if len(c) >= cluster_size]
