"""Simulation / evaluation mixin (reference hic3defdr/analysis/simulation.py).

simulate(): per chromosome, the mean of a condition's scaled data, perturbed
at that condition's loop clusters into two synthetic conditions A and B,
re-biased with the real replicates' bias vectors and size factors, NB-drawn
with the fitted dispersion function (host, the reference's global numpy
random stream). evaluate(): ROC / FDR of this analysis' q-values (the GPU
pipeline's) against the simulation's true cluster labels.
"""
import os

import numpy as np
import pandas as pd
import scipy.sparse as sparse

from hic3defdr_amd import _native
from hic3defdr_amd.util.clusters import load_clusters
from hic3defdr_amd.util.evaluation import evaluate, make_y_true
from hic3defdr_amd.util.printing import eprint
from hic3defdr_amd.util.simulation import simulate


class SimulatingHiC3DeFDR(object):

    def simulate(self, cond, chrom=None, beta=0.5, p_diff=0.4,
                 skip_bias=False, loop_pattern=None, outdir='sim',
                 n_threads=-1, verbose=True):
        """Reference ``simulation.py:22-144``. Writes
        ``<outdir>/<A|B><k>_<chrom>_raw.npz``, ``labels_<chrom>.txt`` and
        ``design.csv``. Chromosomes run in order (the random stream is
        consumed chromosome by chromosome, as the reference's serial path)."""
        if chrom is None:
            for c in self.chroms:
                self.simulate(cond, chrom=c, beta=beta, p_diff=p_diff,
                              skip_bias=skip_bias, loop_pattern=loop_pattern,
                              outdir=outdir, verbose=verbose)
            return
        eprint('simulating data for chrom %s' % chrom)
        loop_pattern = loop_pattern or self.loop_patterns[cond]
        reps = np.asarray(self.design[cond], dtype=bool)
        bias = self.load_bias(chrom)[:, reps]
        sf = self.load_data('size_factors', chrom)
        sf = sf[:, reps] if sf.ndim == 2 else sf[reps]
        row = self.load_data('row', chrom)
        col = self.load_data('col', chrom)
        mean = np.mean(self.load_data('scaled', chrom)[:, reps], axis=1)
        disp_fn = self.load_disp_fn(cond)
        clusters = load_clusters(loop_pattern.replace('<chrom>', chrom))
        os.makedirs(outdir, exist_ok=True)
        k = sf.shape[-1]
        repnames = ['%s%i' % (c, i + 1) for c in 'AB' for i in range(k)]
        design_file = '%s/design.csv' % outdir
        if not os.path.isfile(design_file):
            pd.DataFrame({'A': [1] * k + [0] * k, 'B': [0] * k + [1] * k},
                         dtype=bool, index=repnames).to_csv(design_file)
        if sf.ndim == 2:
            # per-distance factors: the first pixel at each distance
            # (simulation.py:119-127; argmax of an all-False mask is 0)
            eprint('  converting size factors', skip=not verbose)
            dist = col - row
            first = np.array([np.argmax(dist == d)
                              for d in range(dist.max() + 1)])
            sf = sf[first, :]
        if skip_bias:
            bias = np.ones_like(bias)
            sf = np.ones_like(sf)
        classes, reps_iter = simulate(
            row, col, mean, disp_fn, np.tile(bias, 2), np.tile(sf, 2),
            clusters, beta=beta, p_diff=p_diff, trend='dist', verbose=verbose)
        np.savetxt('%s/labels_%s.txt' % (outdir, chrom), classes, fmt='%s')
        for rep, csr in zip(repnames, reps_iter):
            sparse.save_npz('%s/%s_%s_raw.npz' % (outdir, rep, chrom), csr)

    def evaluate(self, cluster_pattern, label_pattern, min_dist=None,
                 max_dist=None, rerun_bh=False, outfile=None):
        """Reference ``simulation.py:146-239``: ``<outdir>/eval.npz`` (or
        ``eval_<min>_<max>.npz``) with fdr, fpr, tpr, thresh."""
        if outfile is None:
            outfile = 'eval.npz' if min_dist is None and max_dist is None \
                else 'eval_%s_%s.npz' % (min_dist, max_dist)
        if self.loop_patterns and cluster_pattern in self.loop_patterns:
            cluster_pattern = self.loop_patterns[cluster_pattern]
        restrict = min_dist is not None or max_dist is not None
        y_true, pvalues, qvalues = [], [], []
        for chrom in self.chroms:
            disp_idx = self.load_data('disp_idx', chrom)
            loop_idx = self.load_data('loop_idx', chrom)
            row = self.load_data('row', chrom, idx=(disp_idx, loop_idx))
            col = self.load_data('col', chrom, idx=(disp_idx, loop_idx))
            clusters = load_clusters(cluster_pattern.replace('<chrom>', chrom))
            labels = np.loadtxt(label_pattern.replace('<chrom>', chrom),
                                dtype='U7')
            dist = col - row
            keep = np.ones(len(dist), dtype=bool)
            if min_dist is not None:
                keep[dist < min_dist] = False
            if max_dist is not None:
                keep[dist > max_dist] = False
            y_true.append(make_y_true(row[keep], col[keep], clusters,
                                      np.atleast_1d(labels)))
            if restrict:
                if rerun_bh:
                    pvalues.append(self.load_data('pvalues', chrom,
                                                  idx=(loop_idx, keep)))
                else:
                    qvalues.append(self.load_data('qvalues', chrom, idx=keep))
        y_true = np.concatenate(y_true)
        if pvalues:
            qvalues = _native.bh(np.concatenate(pvalues))
        elif qvalues:
            qvalues = np.concatenate(qvalues)
        else:
            qvalues, _ = self.load_data('qvalues', 'all')
        fdr, fpr, tpr, thresh = evaluate(y_true, qvalues)
        np.savez('%s/%s' % (self.outdir, outfile),
                 **{'fdr': fdr, 'fpr': fpr, 'tpr': tpr, 'thresh': thresh})
