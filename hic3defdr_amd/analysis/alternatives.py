"""Variants of the HiC3DeFDR model for benchmarking (reference
hic3defdr/analysis/alternatives.py), on the GPU:

  Poisson3DeFDR      zero dispersion; Poisson LRT (h3d_lrt_poisson)
  Unsmoothed3DeFDR   per-pixel method-of-moments dispersion, no distance
                     pooling or smoothing (h3d_mme_per_pixel), then the NB LRT
  Global3DeFDR       one qcml dispersion per condition over the loop pixels
                     (h3d_disp_per_dist with a single distance segment), then
                     the NB LRT

Same class names, methods and outdir files as the reference.
"""
import numpy as np

from hic3defdr_amd import _native
from hic3defdr_amd.analysis.constructor import HiC3DeFDR
from hic3defdr_amd.analysis.analysis import NATIVE_ESTIMATORS
from hic3defdr_amd.util.clusters import load_clusters, pixel_membership
from hic3defdr_amd.util.printing import eprint


class ZeroDispFn(object):
    """Picklable ``disp_fn`` of Poisson3DeFDR (alternatives.py:63-64)."""

    def __call__(self, mean):
        return np.zeros_like(mean)


class ConstDispFn(object):
    """Picklable ``disp_fn`` of Global3DeFDR (alternatives.py:174-175)."""

    def __init__(self, value):
        self.value = float(value)

    def __call__(self, mean):
        return np.ones_like(mean) * self.value


def poisson_lrt(raw, f, design, refit_mu=True):
    """Reference ``alternatives.py:25-42`` on the GPU. Returns pvalues, llr,
    mu_hat_null (n,), mu_hat_alt (n, C).

    The reference's ``refit_mu=False`` branch stacks mu_hat_alt as (C, n) and
    then fails in ``np.dot(mu_hat_alt, design.T)``; it raises here too."""
    design = np.asarray(design, dtype=bool)
    if not refit_mu:
        raise ValueError('poisson_lrt(refit_mu=False): the reference builds '
                         'mu_hat_alt as (C, n) and np.dot fails on it '
                         '(alternatives.py:33-37)')
    cond = design.argmax(axis=1).astype(np.int32)
    return _native.context().lrt_poisson(raw, f, cond, design.shape[1])


class Poisson3DeFDR(HiC3DeFDR):
    """Reference ``alternatives.py:45-115``."""

    def estimate_disp(self, estimator='qcml', frac=None, auto_frac_factor=15.,
                      weighted_lowess=True, n_threads=-1):
        # note: all kwargs are ignored (as in the reference)
        eprint('estimating dispersion')
        eprint('  loading data')
        disp_idx, _ = self.load_data('disp_idx', 'all')
        _, offsets = self.load_data('row', 'all', idx=disp_idx)
        C = self.design.shape[1]
        disp_per_dist = np.zeros((self.dist_thresh_max + 1, C))
        disp = np.zeros((int(disp_idx.sum()), C))
        for cond in self.design.columns:
            self.save_disp_fn(cond, ZeroDispFn())
        eprint('  saving estimated dispersions to disk')
        self.save_data(disp, 'disp', offsets)
        self.save_data(disp_per_dist, 'disp_per_dist')

    def lrt(self, chrom=None, refit_mu=True, n_threads=-1, verbose=True):
        if chrom is None:
            for c in self.chroms:
                self.lrt(chrom=c, refit_mu=refit_mu, verbose=verbose)
            return
        eprint('running LRT for chrom %s' % chrom)
        bias = self.load_bias(chrom)
        size_factors = self.load_data('size_factors', chrom)
        row = self.load_data('row', chrom)
        col = self.load_data('col', chrom)
        raw = self.load_data('raw', chrom)
        disp_idx = self.load_data('disp_idx', chrom)
        f = bias[row, :][disp_idx, :] * bias[col, :][disp_idx, :] * \
            size_factors[disp_idx, :]
        # the reference always refits here (alternatives.py:98-99)
        pvalues, llr, mu_hat_null, mu_hat_alt = poisson_lrt(
            raw[disp_idx, :], f, self.design.values, refit_mu=True)
        if self.loop_patterns:
            cl = [load_clusters(p.replace('<chrom>', chrom))
                  for p in self.loop_patterns.values()]
            loop_idx = pixel_membership(row[disp_idx], col[disp_idx], cl)
            self.save_data(loop_idx, 'loop_idx', chrom)
        self.save_data(pvalues, 'pvalues', chrom)
        self.save_data(llr, 'llr', chrom)
        self.save_data(mu_hat_null, 'mu_hat_null', chrom)
        self.save_data(mu_hat_alt, 'mu_hat_alt', chrom)


class Unsmoothed3DeFDR(HiC3DeFDR):
    """Reference ``alternatives.py:118-137``: disp = max(mme_per_pixel(scaled
    of the condition), 1e-7); no disp_per_dist / disp_fn are written."""

    def estimate_disp(self, estimator='qcml', frac=None, auto_frac_factor=15.,
                      weighted_lowess=True, n_threads=-1):
        eprint('estimating dispersion')
        eprint('  loading data')
        disp_idx, _ = self.load_data('disp_idx', 'all')
        _, offsets = self.load_data('row', 'all', idx=disp_idx)
        scaled, _ = self.load_data('scaled', 'all', idx=disp_idx)
        eprint('  computing pixel-wise mean per condition')
        disp = _native.context().mme_per_pixel(scaled, None,
                                               self._cond_of_rep(),
                                               self.design.shape[1],
                                               min_disp=1e-7)
        eprint('  saving estimated dispersions to disk')
        self.save_data(disp, 'disp', offsets)


class Global3DeFDR(HiC3DeFDR):
    """Reference ``alternatives.py:140-181``: one dispersion per condition,
    estimated over the loop pixels of every chromosome."""

    def estimate_disp(self, estimator='qcml', frac=None, auto_frac_factor=15.,
                      weighted_lowess=True, n_threads=-1):
        # note: all kwargs except estimator are ignored (as in the reference)
        eprint('estimating dispersion')
        eprint('  loading data')
        raw, f, _, offsets = self._f_and_dist()
        loop_idx, _ = self.load_data('loop_idx', 'all')
        design = np.asarray(self.design, dtype=bool)
        C = design.shape[1]
        raw_l, f_l = raw[loop_idx], f[loop_idx]
        if callable(estimator):
            global_disp = np.array([estimator(raw_l[:, design[:, c]],
                                              f=f_l[:, design[:, c]])
                                    for c in range(C)])
        elif estimator in NATIVE_ESTIMATORS:
            # every loop pixel in one segment: distance 0 of a D = 1 table
            global_disp = self._ctx().disp_per_dist(
                raw_l, f_l, np.zeros(len(raw_l), dtype=np.int32),
                self._cond_of_rep(), C, 1, estimator=estimator)[0]
        else:
            raise NotImplementedError(
                'estimator=%r: the reference divides its int64 raw slice in '
                'place for cml/mme (dispersion.py:76,129) and raises; the GPU '
                'path implements %s' % (estimator, NATIVE_ESTIMATORS))
        disp = np.zeros((len(raw), C))
        disp_per_dist = np.zeros((self.dist_thresh_max + 1, C))
        for c, cond in enumerate(self.design.columns):
            eprint('  estimating dispersion for condition %s' % cond)
            disp[:, c] = global_disp[c]
            disp_per_dist[:, c] = global_disp[c]
            self.save_disp_fn(cond, ConstDispFn(global_disp[c]))
        eprint('  saving estimated dispersions to disk')
        self.save_data(disp, 'disp', offsets)
        self.save_data(disp_per_dist, 'disp_per_dist')
