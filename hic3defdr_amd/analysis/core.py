"""Persistence mixin (reference hic3defdr/analysis/core.py): the outdir is the
contract between stages — ``<outdir>/<name>_<chrom>.npy`` per chromosome,
``disp_per_dist.npy``, ``disp_fn_<cond>.pickle`` and ``pickle``."""
import pickle

import numpy as np


def _interp_extrap(xp, yp, x):
    """scipy interp1d(kind='linear', fill_value='extrapolate')."""
    idx = np.clip(np.searchsorted(xp, x), 1, len(xp) - 1)
    lo, hi = idx - 1, idx
    return (yp[hi] - yp[lo]) / (xp[hi] - xp[lo]) * (x - xp[lo]) + yp[lo]


class DispFn(object):
    """Picklable fitted dispersion function of one condition.

    The reference pickles the lowess closure (``core.py:220-253``,
    ``lowess.py:76-92`` / ``229-242``). The smoothed part is piecewise linear
    with knots on integer distances (lowess outputs at the expanded integer
    x), so its tabulation on d = 0..D-1 (``h3d_disp_table``, native) with
    linear interpolation / extrapolation over the integer knots reproduces
    it. The weighted fit replaces it below ``x[inc_idx]`` by linear
    interpolation of the raw (distance, dispersion) points, and below the
    first fitted distance by ``y[0]``; those points are kept here too.
    """

    def __init__(self, table, disp_per_dist_col, weighted=True):
        self.table = np.asarray(table, dtype=float)
        col = np.asarray(disp_per_dist_col, dtype=float)
        fin = np.isfinite(col)
        self.x = np.arange(len(col), dtype=float)[fin]
        self.y = col[fin]
        self.weighted = bool(weighted)
        self.inc_idx = int(np.argmax(np.diff(self.y) > 0) + 1) \
            if self.weighted else 0

    def __call__(self, x_star):
        x = np.asarray(x_star, dtype=float)
        t = self.table
        d = np.arange(len(t), dtype=float)
        xi = np.rint(x)
        on_knot = (xi == x) & (xi >= 0) & (xi < len(t))
        out = np.empty(x.shape, dtype=float)
        out[on_knot] = t[xi[on_knot].astype(np.int64)]
        off = ~on_knot
        if off.any():
            out[off] = _interp_extrap(d, t, x[off])
        if self.weighted:
            below = x < self.x[self.inc_idx]
            if below.any():
                v = _interp_extrap(self.x, self.y, x[below])
                v[x[below] < self.x[0]] = self.y[0]
                out[below] = v
        return out


class CoreHiC3DeFDR(object):
    """Mixin providing saving and loading (reference ``core.py:10-291``)."""

    @property
    def picklefile(self):
        return '%s/pickle' % self.outdir

    @classmethod
    def load(cls, outdir):
        """Reference ``core.py:15-33``."""
        with open('%s/pickle' % outdir, 'rb') as handle:
            return cls(outdir=outdir, **pickle.load(handle))

    def load_bias(self, chrom):
        """Reference ``core.py:35-60``: (n_bins, R); bins failing
        ``bias_thresh`` in any replicate are zeroed."""
        bias = np.array([np.loadtxt(pattern.replace('<chrom>', chrom))
                         for pattern in self.bias_patterns]).T
        bias[(np.any(bias < self.bias_thresh, axis=1)) |
             (np.any(bias > 1. / self.bias_thresh, axis=1)), :] = 0
        return bias

    def load_data(self, name, chrom=None, idx=None, rep=None, cond=None,
                  coo=False):
        """Reference ``core.py:62-196``. Deviation: the reference's
        ``loop_idx`` short-circuit calls ``np.load_data`` (``core.py:105``, an
        AttributeError); here it returns the all-True vector it intends."""
        if name == 'loop_idx' and self.loop_patterns is None and idx is None \
                and chrom != 'all':
            disp_idx = self.load_data('disp_idx', chrom)
            return np.ones(disp_idx.sum(), dtype=bool)
        col_idx = self.design.index.tolist().index(rep) if rep is not None \
            else self.design.columns.tolist().index(cond) if cond is not None \
            else None
        if coo:
            if chrom == 'all' or idx is not None:
                raise ValueError("cannot pass coo=True with chrom='all' or idx")
            if name in ['row', 'col', 'bias', 'cov_per_bin', 'disp_per_bin']:
                raise ValueError('data with name %s cannot be loaded as COO'
                                 % name)
            if name in ['raw', 'size_factors', 'scaled', 'disp_idx']:
                row = self.load_data('row', chrom)
                col = self.load_data('col', chrom)
            elif name in ['loop_idx', 'disp', 'mu_hat_null', 'mu_hat_alt',
                          'llr', 'pvalues']:
                disp_idx = self.load_data('disp_idx', chrom)
                row = self.load_data('row', chrom, idx=disp_idx)
                col = self.load_data('col', chrom, idx=disp_idx)
            elif name in ['qvalues']:
                disp_idx = self.load_data('disp_idx', chrom)
                loop_idx = self.load_data('loop_idx', chrom)
                row = self.load_data('row', chrom, idx=(disp_idx, loop_idx))
                col = self.load_data('col', chrom, idx=(disp_idx, loop_idx))
            else:
                raise ValueError('data name %s not recognized' % name)
            data = self.load_data(name, chrom)
            if col_idx is not None:
                return row, col, data[:, col_idx]
            return row, col, data
        if type(idx) == tuple:
            big_idx, small_idx = idx
            big_idx = big_idx.copy()
            big_idx[np.where(big_idx)[0][~small_idx]] = False
            idx = big_idx
        if chrom is None:
            fname = '%s/%s.npy' % (self.outdir, name)
        elif chrom != 'all':
            fname = '%s/%s_%s.npy' % (self.outdir, name, chrom)
        else:
            fname = None
        if fname is not None:
            if idx is None:
                data = np.load(fname)
                return data[:, col_idx] if col_idx is not None else data
            data = np.load(fname, mmap_mode='r')
            if col_idx is not None:
                return data[idx, col_idx]
            return data[idx]
        idx_offset = 0
        all_data = []
        offset = 0
        offsets = [0]
        for c in self.chroms:
            fname = '%s/%s_%s.npy' % (self.outdir, name, c)
            if idx is not None:
                data = np.load(fname, mmap_mode='r')
                full = data.shape[0]
                data = data[idx[idx_offset:idx_offset + full]]
                idx_offset += full
            else:
                data = np.load(fname)
            offset += data.shape[0]
            offsets.append(offset)
            all_data.append(data)
        all_data = np.concatenate(all_data)
        if col_idx is not None:
            return all_data[:, col_idx], np.array(offsets)
        return all_data, np.array(offsets)

    def save_data(self, data, name, chrom=None):
        """Reference ``core.py:198-218``."""
        if chrom is None:
            np.save('%s/%s.npy' % (self.outdir, name), data)
        elif isinstance(chrom, np.ndarray):
            for i, c in enumerate(self.chroms):
                self.save_data(data[chrom[i]:chrom[i + 1]], name, c)
        else:
            np.save('%s/%s_%s.npy' % (self.outdir, name, chrom), data)

    def load_disp_fn(self, cond):
        """Reference ``core.py:220-236``."""
        with open('%s/disp_fn_%s.pickle' % (self.outdir, cond), 'rb') as h:
            return pickle.load(h)

    def save_disp_fn(self, cond, disp_fn):
        """Reference ``core.py:238-253``."""
        with open('%s/disp_fn_%s.pickle' % (self.outdir, cond), 'wb') as h:
            pickle.dump(disp_fn, h, -1)
