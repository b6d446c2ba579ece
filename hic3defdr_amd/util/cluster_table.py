"""Cluster tables (reference hic3defdr/util/cluster_table.py).

``ClusterTable`` holds a table as columns (bounding boxes, sizes, cluster
text, optional classification) and reads / writes the reference's TSV layout
directly, so ``threshold`` / ``classify`` / ``collect`` never build a pandas
frame per cluster. ``clusters_to_table`` / ``sort_cluster_table`` /
``load_cluster_table`` keep the reference's DataFrame API.

TSV layout (pandas ``to_csv(sep='\\t')`` of the reference's frame): header
``loop_id us_chrom us_start us_end ds_chrom ds_start ds_end cluster_size
cluster [classification]``; loop_id = ``chr:start-end_chr:start-end``;
``cluster`` = ``[[i, j], [i, j], ...]``. Rows sorted by (natural chromosome
order, us_start, us_end, ds_start, ds_end), stable (pandas multi-column
sort_values is a lexsort).
"""
import re

import numpy as np

from hic3defdr_amd.util.clusters import ClusterList, cluster_from_string

COLUMN_ORDER = ['loop_id', 'us_chrom', 'us_start', 'us_end', 'ds_chrom',
                'ds_start', 'ds_end', 'cluster_size', 'cluster']


def natural_sort_key(s):
    """lib5c.util.primers.natural_sort_key (digits compare as numbers)."""
    return [int(t) if t.isdigit() else t.lower()
            for t in re.split(r'(\d+)', s)]


class ClusterTable(object):
    """Columns of a cluster table (one row per cluster)."""

    def __init__(self, us_chrom, us_start, us_end, ds_chrom, ds_start, ds_end,
                 size, cluster, classification=None):
        self.us_chrom = list(us_chrom)
        self.us_start = np.asarray(us_start, dtype=np.int64)
        self.us_end = np.asarray(us_end, dtype=np.int64)
        self.ds_chrom = list(ds_chrom)
        self.ds_start = np.asarray(ds_start, dtype=np.int64)
        self.ds_end = np.asarray(ds_end, dtype=np.int64)
        self.size = np.asarray(size, dtype=np.int64)
        self.cluster = list(cluster)
        self.classification = None if classification is None else \
            list(classification)

    def __len__(self):
        return len(self.cluster)

    @classmethod
    def from_clusters(cls, clusters, chrom, res):
        """cluster_table.py:14-77 clusters_to_table (sorted)."""
        if not isinstance(clusters, ClusterList):
            clusters = ClusterList.from_sets(clusters)
        rmin, rmax, cmin, cmax = clusters.bounds()
        n = len(clusters)
        t = cls([chrom] * n, rmin * res, (rmax + 1) * res, [chrom] * n,
                cmin * res, (cmax + 1) * res, clusters.sizes(),
                clusters.texts())
        return t.sorted()

    def loop_ids(self):
        return ['%s:%d-%d_%s:%d-%d' % v for v in zip(
            self.us_chrom, self.us_start.tolist(), self.us_end.tolist(),
            self.ds_chrom, self.ds_start.tolist(), self.ds_end.tolist())]

    def with_classification(self, label):
        t = self.take(np.arange(len(self)))
        t.classification = [label] * len(self)
        return t

    def take(self, idx):
        idx = np.asarray(idx, dtype=np.int64)
        return ClusterTable(
            [self.us_chrom[i] for i in idx], self.us_start[idx],
            self.us_end[idx], [self.ds_chrom[i] for i in idx],
            self.ds_start[idx], self.ds_end[idx], self.size[idx],
            [self.cluster[i] for i in idx],
            None if self.classification is None else
            [self.classification[i] for i in idx])

    def sorted(self):
        """cluster_table.py:80-140 sort_cluster_table."""
        if not len(self):
            return self
        names = sorted(set(self.us_chrom) | set(self.ds_chrom),
                       key=natural_sort_key)
        rank = {c: i for i, c in enumerate(names)}
        us = np.array([rank[c] for c in self.us_chrom], dtype=np.int64)
        ds = np.array([rank[c] for c in self.ds_chrom], dtype=np.int64)
        order = np.lexsort((self.ds_end, self.ds_start, ds, self.us_end,
                            self.us_start, us))
        return self.take(order)

    @staticmethod
    def concat(tables):
        tables = list(tables)
        cls_ = [t.classification for t in tables]
        has = any(c is not None for c in cls_)
        return ClusterTable(
            sum((t.us_chrom for t in tables), []),
            np.concatenate([t.us_start for t in tables] or [[]]),
            np.concatenate([t.us_end for t in tables] or [[]]),
            sum((t.ds_chrom for t in tables), []),
            np.concatenate([t.ds_start for t in tables] or [[]]),
            np.concatenate([t.ds_end for t in tables] or [[]]),
            np.concatenate([t.size for t in tables] or [[]]),
            sum((t.cluster for t in tables), []),
            sum(((c if c is not None else [''] * len(t))
                 for c, t in zip(cls_, tables)), []) if has else None)

    def to_tsv(self, path):
        cols = COLUMN_ORDER + (['classification']
                               if self.classification is not None else [])
        lines = ['\t'.join(cols)]
        ids = self.loop_ids()
        for k in range(len(self)):
            f = [ids[k], self.us_chrom[k], str(self.us_start[k]),
                 str(self.us_end[k]), self.ds_chrom[k], str(self.ds_start[k]),
                 str(self.ds_end[k]), str(self.size[k]), self.cluster[k]]
            if self.classification is not None:
                f.append(self.classification[k])
            lines.append('\t'.join(f))
        with open(path, 'w') as fh:
            fh.write('\n'.join(lines) + '\n')

    @classmethod
    def read_tsv(cls, path):
        """A TSV written by ``to_tsv`` (or the reference); the cluster text
        is kept verbatim."""
        with open(path, 'r') as fh:
            lines = fh.read().split('\n')
        header = lines[0].split('\t')
        rows = [ln.split('\t') for ln in lines[1:] if ln]
        col = {h: i for i, h in enumerate(header)}

        def ints(name):
            return np.array([int(r[col[name]]) for r in rows], dtype=np.int64)
        return cls([r[col['us_chrom']] for r in rows], ints('us_start'),
                   ints('us_end'), [r[col['ds_chrom']] for r in rows],
                   ints('ds_start'), ints('ds_end'), ints('cluster_size'),
                   [r[col['cluster']] for r in rows],
                   [r[col['classification']] for r in rows]
                   if 'classification' in col else None)

    def to_frame(self):
        import pandas as pd
        df = pd.DataFrame({
            'loop_id': self.loop_ids(), 'us_chrom': self.us_chrom,
            'us_start': self.us_start, 'us_end': self.us_end,
            'ds_chrom': self.ds_chrom, 'ds_start': self.ds_start,
            'ds_end': self.ds_end, 'cluster_size': self.size,
            'cluster': [cluster_from_string(c) for c in self.cluster]},
            columns=COLUMN_ORDER)
        if self.classification is not None:
            df['classification'] = self.classification
        return df.set_index('loop_id')


def clusters_to_table(clusters, chrom, res):
    """Reference ``cluster_table.py:14-77`` (DataFrame indexed by loop_id)."""
    return ClusterTable.from_clusters(clusters, chrom, res).to_frame()


def sort_cluster_table(cluster_table):
    """Reference ``cluster_table.py:80-140`` (not in place)."""
    names = sorted(set(cluster_table['us_chrom'].unique()) |
                   set(cluster_table['ds_chrom'].unique()),
                   key=natural_sort_key)
    rank = {c: i for i, c in enumerate(names)}
    keys = (cluster_table['ds_end'].values, cluster_table['ds_start'].values,
            cluster_table['ds_chrom'].map(rank).values,
            cluster_table['us_end'].values, cluster_table['us_start'].values,
            cluster_table['us_chrom'].map(rank).values)
    return cluster_table.iloc[np.lexsort(keys)]


def load_cluster_table(table_filename):
    """Reference ``cluster_table.py:143-176``."""
    import pandas as pd
    df = pd.read_csv(table_filename, sep='\t', index_col=0)
    df['cluster'] = df['cluster'].apply(cluster_from_string)
    return df
