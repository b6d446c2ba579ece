"""Clusters of pixels (reference hic3defdr/util/clusters.py).

Two forms:

- the reference's: a list of sets of ``(i, j)`` tuples (``find_clusters``,
  ``load_clusters``, ``save_clusters`` keep that API);
- ``ClusterList``: the same clusters as arrays (pixel coordinates, a member
  permutation and cluster start offsets), which the pipeline steps use so a
  chromosome with millions of thresholded pixels never becomes millions of
  Python tuples. Cluster numbering follows the reference's group order, and
  within a cluster the pixels come in the iteration order of the reference's
  Python set (h3d_find_clusters_ordered replays CPython's set table over the
  DirectedDisjointSet's adds and merges), so the JSON / TSV text is the
  reference's byte for byte.

Clustering itself is ``h3d_find_clusters`` in libh3d (host C++ restatement of
the DirectedDisjointSet, clusters.py:15-97).
"""
import json
import re

import numpy as np

from hic3defdr_amd import _native


class ClusterList(object):
    """Cluster k = pixels ``(row[m], col[m])`` for
    ``m in members[starts[k]:starts[k + 1]]``."""

    def __init__(self, row, col, members, starts):
        self.row = np.asarray(row, dtype=np.int64)
        self.col = np.asarray(col, dtype=np.int64)
        self.members = np.asarray(members, dtype=np.int64)
        self.starts = np.asarray(starts, dtype=np.int64)

    @classmethod
    def empty(cls):
        z = np.zeros(0, dtype=np.int64)
        return cls(z, z, z, np.zeros(1, dtype=np.int64))

    @classmethod
    def from_labels(cls, row, col, labels, n_clusters):
        """Group pixels by label (stable: input order inside a cluster)."""
        members = np.argsort(labels, kind='stable')
        counts = np.bincount(labels, minlength=n_clusters)
        starts = np.zeros(n_clusters + 1, dtype=np.int64)
        np.cumsum(counts, out=starts[1:])
        return cls(row, col, members, starts)

    @classmethod
    def find(cls, row, col, connectivity=1):
        """Clusters of the pixel list (row, col) in the reference's order
        (``find_clusters`` on the COO of these pixels)."""
        row = np.asarray(row, dtype=np.int64)
        col = np.asarray(col, dtype=np.int64)
        if len(row) == 0:
            return cls.empty()
        try:
            lab, nc, order = _native.cluster_order(row, col, connectivity)
        except _native.H3DError:
            # repeated pixels (a COO with duplicates): the sets' order is not
            # defined by the pixel list; input order inside each cluster
            lab, nc = _native.cluster_labels(row, col, connectivity)
            return cls.from_labels(row, col, lab, nc)
        counts = np.bincount(lab, minlength=nc)
        starts = np.zeros(nc + 1, dtype=np.int64)
        np.cumsum(counts, out=starts[1:])
        return cls(row, col, order, starts)

    @classmethod
    def from_sets(cls, clusters):
        """From the reference form (list of iterables of (i, j))."""
        rows, cols, sizes = [], [], []
        for c in clusters:
            c = list(c)
            sizes.append(len(c))
            for i, j in c:
                rows.append(int(i))
                cols.append(int(j))
        starts = np.zeros(len(sizes) + 1, dtype=np.int64)
        np.cumsum(sizes, out=starts[1:])
        return cls(np.array(rows, dtype=np.int64),
                   np.array(cols, dtype=np.int64),
                   np.arange(len(rows), dtype=np.int64), starts)

    def __len__(self):
        return len(self.starts) - 1

    def sizes(self):
        return np.diff(self.starts)

    def select(self, keep):
        """Sub-list of the clusters where ``keep`` (bool per cluster)."""
        keep = np.asarray(keep, dtype=bool)
        sz = self.sizes()[keep]
        idx = np.repeat(keep, self.sizes())
        starts = np.zeros(len(sz) + 1, dtype=np.int64)
        np.cumsum(sz, out=starts[1:])
        return ClusterList(self.row, self.col, self.members[idx], starts)

    def size_filter(self, cluster_size):
        """thresholding.py:44-61: keep clusters with >= cluster_size pixels."""
        return self.select(self.sizes() >= cluster_size)

    def pixels(self):
        """(row, col) of all member pixels, cluster by cluster."""
        return self.row[self.members], self.col[self.members]

    def bounds(self):
        """Per-cluster (min row, max row, min col, max col)."""
        if not len(self):
            z = np.zeros(0, dtype=np.int64)
            return z, z, z, z
        r, c = self.pixels()
        s = self.starts[:-1]
        return (np.minimum.reduceat(r, s), np.maximum.reduceat(r, s),
                np.minimum.reduceat(c, s), np.maximum.reduceat(c, s))

    def texts(self):
        """Per-cluster text ``[[i, j], [i, j]]`` as a list of str."""
        if not len(self):
            return []
        buf, ends = _native.format_clusters(self.row, self.col, self.members,
                                            self.starts)
        b = np.concatenate([[0], ends])
        s = buf.decode('ascii')
        return [s[b[k]:b[k + 1]] for k in range(len(self))]

    def json_text(self):
        """save_clusters text (clusters.py:129-130, json.dump defaults)."""
        if not len(self):
            return '[]'
        buf, _ = _native.format_clusters(self.row, self.col, self.members,
                                         self.starts)
        # clusters are adjacent "[...]" blocks: join them with ", "
        return '[' + buf.decode('ascii').replace(']][[', ']], [[') + ']'

    def to_sets(self):
        r, c = self.pixels()
        return [set(zip(r[a:b].tolist(), c[a:b].tolist()))
                for a, b in zip(self.starts[:-1], self.starts[1:])]


def find_clusters(sig_points, connectivity=1):
    """Reference ``clusters.py:73-97``: clusters of the True entries of a
    boolean matrix (scipy sparse or dense), as a list of sets of tuples."""
    import scipy.sparse as sparse
    m = sparse.coo_matrix(sig_points)
    return ClusterList.find(m.row, m.col, connectivity).to_sets()


def load_clusters(infile):
    """Reference ``clusters.py:176-193``: list of sets of (i, j) tuples."""
    with open(infile, 'r') as handle:
        return [set([tuple(e) for e in cluster]) for cluster in
                json.load(handle)]


_PIXEL_TEXT = bytes.maketrans(b'[]', b'  ')
_PAIR = rb'\[\d+,\d+\]'
_CLUSTER = rb'\[(?:%s(?:,%s)*)?\]' % (_PAIR, _PAIR)
_CLUSTER_FILE = re.compile(rb'\[(?:%s(?:,%s)*)?\]' % (_CLUSTER, _CLUSTER))


def load_cluster_pixels(infile):
    """Every pixel of a cluster JSON (reference clusters.py:176-193's file:
    a list of clusters, each a list of [i, j]) as one (k, 2) int64 array,
    parsed in C (numpy's text reader over the numbers) instead of as
    Python sets of tuples -- what prepare_data's loop_idx needs (the union
    of the clusters' pixels, analysis.py:117-125). Files that are not pure
    nested lists of integer pairs go through json (load_clusters)."""
    with open(infile, 'rb') as handle:
        text = handle.read()
    compact = text.translate(None, b' \t\r\n')
    if _CLUSTER_FILE.fullmatch(compact):
        body = compact.translate(_PIXEL_TEXT).replace(b',', b' ').strip()
        if not body:
            return np.zeros((0, 2), dtype=np.int64)
        return np.fromstring(body.decode('ascii'), dtype=np.int64,
                             sep=' ').reshape(-1, 2)
    # anything else as the reference reads it; a pixel with a non-integer
    # coordinate can match no (row, col) of the union
    pix = np.array([p for cl in load_clusters(infile) for p in cl],
                   dtype=np.float64).reshape(-1, 2)
    pix = pix[np.all(pix == np.floor(pix), axis=1)]
    return pix.astype(np.int64)


def load_cluster_list(infile):
    """A cluster JSON as a ``ClusterList`` (file order kept)."""
    with open(infile, 'r') as handle:
        data = json.load(handle)
    return ClusterList.from_sets(data)


def save_clusters(clusters, outfile):
    """Reference ``clusters.py:116-136`` (list of sets or a ClusterList)."""
    with open(outfile, 'w') as handle:
        if isinstance(clusters, ClusterList):
            handle.write(clusters.json_text())
        else:
            json.dump([[[int(i), int(j)] for i, j in cluster]
                       for cluster in clusters], handle)


def cluster_to_loop_id(cluster, chrom, resolution):
    """Reference ``clusters.py:300-330``: "chr:start-end_chr:start-end"."""
    x, y = zip(*cluster)
    return '%s:%s-%s_%s:%s-%s' % (chrom, min(x) * resolution,
                                  (max(x) + 1) * resolution, chrom,
                                  min(y) * resolution,
                                  (max(y) + 1) * resolution)


def cluster_from_string(cluster_string):
    """Reference ``clusters.py:333-360``."""
    return json.loads(cluster_string.replace('(', '[').replace('{', '[')
                      .replace(')', ']').replace('}', ']'))


def pixel_membership(row, col, clusters_lists, n_bins=None, mask=None):
    """Boolean vector: (row[k], col[k]) in the union of all clusters
    (reference ``analysis.py:117-125``, a Python set lookup per pixel),
    vectorised with 64-bit pixel keys. ``clusters_lists``: per condition a
    list of pixel sets (load_clusters) or a (k, 2) pixel array
    (load_cluster_pixels)."""
    arrs = [c for c in clusters_lists if isinstance(c, np.ndarray)]
    sets = [c for c in clusters_lists if not isinstance(c, np.ndarray)]
    if sets:
        pixels = set().union(*sum(sets, []))
        if pixels:
            arrs.append(np.array(sorted(pixels), dtype=np.int64))
    arrs = [a.reshape(-1, 2) for a in arrs if len(a)]
    if not arrs or len(row) == 0:
        return np.zeros(len(row) if mask is None else
                        int(np.count_nonzero(mask)), dtype=bool)
    pix = np.concatenate(arrs)
    return pixel_in(row, col, pix[:, 0], pix[:, 1], mask=mask)


def pixel_in(row, col, prow, pcol, mask=None):
    """(row[k], col[k]) in the pixel set {(prow, pcol)} (vectorised), for
    the k where ``mask`` (when given) is set -- the keys are formed over all
    of row / col in place and masked once (prepare_data's loop_idx over the
    disp pixels of a chromosome's union)."""
    row = np.asarray(row)
    col = np.asarray(col)
    if mask is not None and len(row):
        n_out = int(np.count_nonzero(mask))
    else:
        n_out = len(row)
    if n_out == 0 or len(prow) == 0:
        return np.zeros(n_out, dtype=bool)
    prow = np.asarray(prow, dtype=np.int64)
    pcol = np.asarray(pcol, dtype=np.int64)
    base = int(max(pcol.max(), col.max())) + 1
    keys = row.astype(np.int64)
    keys *= base
    keys += col
    if mask is not None:
        keys = keys[mask]
    pk = prow * base + pcol
    if len(keys) > 1 and not np.all(keys[1:] > keys[:-1]):
        return np.isin(keys, pk)
    # the union's pixels come in (row, col) order with unique keys: each set
    # pixel is found by binary search (no sort of the chromosome's keys)
    out = np.zeros(len(keys), dtype=bool)
    pos = np.searchsorted(keys, pk)
    ok = pos < len(keys)
    pos, pk = pos[ok], pk[ok]
    out[pos[keys[pos] == pk]] = True
    return out
