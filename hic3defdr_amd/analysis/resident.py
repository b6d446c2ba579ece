"""The product path's device-resident copy of a HiC3DeFDR object's stage data.

The reference's stages hand their data over through the outdir only
(prepare_data writes row / col / raw / size_factors / disp_idx,
``analysis.py:128-133``; estimate_disp reads them back and rebuilds
``f = bias[row] * bias[col] * size_factors``, ``:169-183``; lrt reads them
and ``disp`` again and rebuilds ``f``, ``:261-275``). The outdir contract is
kept -- every file is written (core.py's write-behind queue) -- but within
one object the data also stays in HBM:

* prepare_data leaves each chromosome's union (row, col, raw as int32, size
  factors, disp_idx) in device buffers (``h3d_union_fill_dev``,
  ``h3d_size_factors_dev``), so nothing is re-read or re-uploaded;
* estimate_disp builds the disp pixels of all its chromosomes on the device
  (``h3d_disp_pixels_dev``: compaction by disp_idx, f in numpy's product
  order) -- from the resident union, or uploaded from the outdir files when
  another process prepared them -- and runs qcml, the smoother and
  ``disp = table[dist]`` there (``h3d_estimate_disp_dev``,
  ``h3d_table_gather_dev``);
* lrt runs over estimate_disp's resident pixels and device tables in one
  launch (``h3d_lrt_dev_tab``) while the disp files it would read are the
  ones estimate_disp wrote; otherwise per chromosome from the files;
* bh runs on lrt's device p-values (``h3d_bh_dev``) while the pvalues files
  it would read are the ones lrt wrote.

A resident entry is used only while the outdir files it mirrors are the
ones it was made from (core.CoreHiC3DeFDR.is_current, or the file stamps
taken when it was loaded from disk) and the bias files are unchanged, so
edits of the outdir are always seen. Device buffers are torch tensors (the
allocator); every computation on them is libh3d's.
"""
import os

import numpy as np

from hic3defdr_amd import _native
from hic3defdr_amd.analysis.d2h import to_host_async


def _stamp(fname):
    try:
        st = os.stat(fname)
    except OSError:
        return None
    return (st.st_ino, st.st_size, st.st_mtime_ns, st.st_ctime_ns)


def bias_stamps(bias_patterns, chrom):
    """{bias file: ('disk', stamp)} of one chromosome's bias files."""
    return {f: ('disk', _stamp(f)) for f in
            (p.replace('<chrom>', chrom) for p in bias_patterns)}


class ChromDev(object):
    """One chromosome's union pixels on the device."""

    def __init__(self, row, col, raw, sf, sf_per_rep, disp_idx, n_disp, bias,
                 files):
        self.row, self.col, self.raw = row, col, raw
        self.sf, self.sf_per_rep = sf, sf_per_rep
        self.disp_idx, self.n_disp = disp_idx, n_disp
        self.bias = bias      # host (n_bins, R), bias_thresh-filtered
        self.files = files    # fname -> ('ours', generation) / ('disk', stamp)
        self.n = int(row.shape[0])


class Resident(object):
    """The device copy of one object's stages (see the module docstring)."""

    STAGES = ('row', 'col', 'raw', 'size_factors', 'disp_idx')

    def __init__(self, h):
        import torch
        self.torch = torch
        self.h = h
        self.ctx = h._ctx()
        self.dev = torch.device('cuda', self.ctx.device)
        self.chroms = {}
        self.session = None
        self.pvals = None

    # -- validity --------------------------------------------------------
    def _current(self, files):
        for fname, (kind, tok) in files.items():
            if kind == 'ours':
                if self.h.write_generation(fname) != tok or \
                        not self.h.is_current(fname):
                    return False
            elif _stamp(fname) != tok:
                return False
        return True

    def _token(self, fname):
        """('ours', generation) for an outdir file this object wrote and
        that is still that write, else ('disk', file stamp)."""
        if self.h.is_current(fname):
            return ('ours', self.h.write_generation(fname))
        return ('disk', _stamp(fname))

    def _bias_stamps(self, chrom):
        return bias_stamps(self.h.bias_patterns, chrom)

    # -- prepare_data ----------------------------------------------------
    def union_alloc(self, holder):
        """device_alloc for Context.sparse_union: the union's device
        buffers, kept in ``holder``."""
        torch = self.torch

        def alloc(n, R):
            try:
                holder['row'] = torch.empty(n, dtype=torch.int32,
                                            device=self.dev)
                holder['col'] = torch.empty(n, dtype=torch.int32,
                                            device=self.dev)
                holder['raw'] = torch.empty((n, R), dtype=torch.int32,
                                            device=self.dev)
                holder['bal'] = torch.empty((n, R), dtype=torch.float64,
                                            device=self.dev)
            except RuntimeError as e:   # torch.OutOfMemoryError included
                holder.clear()
                raise _native.H3DError(
                    'allocating the device copy of a %d x %d pixel union: %s'
                    % (n, R, e), code=-4)
            return tuple(holder[k].data_ptr() if n else None
                         for k in ('row', 'col', 'raw', 'bal'))
        return alloc

    def size_factors(self, holder, dist, norm, n_bins):
        """Size factors on the resident balanced, the device copy kept in
        ``holder['sf']``: returns (host array, ready) -- for the conditional
        norms the (n, R) host array arrives by a background copy (ready()
        returns once it has), the (R,) factors of the global norms at once
        (ready None)."""
        torch = self.torch
        n, R = holder['bal'].shape
        cond = norm.startswith('conditional')
        holder['sf'] = torch.empty((n, R) if cond else R, dtype=torch.float64,
                                   device=self.dev)
        sf = self.ctx.size_factors_dev(
            holder['bal'].data_ptr() if n else None, dist, n, R, norm, n_bins,
            d_sf_out=holder['sf'].data_ptr() if holder['sf'].numel() else None,
            host_out=not (cond and n))
        if sf is None:
            return to_host_async(holder['sf'])
        return sf, None

    def scale_disp(self, holder, design, mean_thresh, dist_min, dist):
        """scaled and disp_idx (analysis.py:109-115) from the resident
        balanced and size factors (h3d_scale_disp_dev); the disp flags stay
        on the device in ``holder['di']``, balanced is released. The rows the
        device leaves to numpy's product (flag 2: non-finite, or a mean
        within 1e-12 of the threshold) are decided here by the reference's
        own expression. Returns (scaled, ready, disp_idx): scaled arrives by
        a background copy (ready() returns once it has)."""
        torch = self.torch
        n, R = holder['bal'].shape
        holder['di'] = torch.empty(n, dtype=torch.uint8, device=self.dev)
        t_scaled = torch.empty((n, R), dtype=torch.float64, device=self.dev)
        sf = holder['sf']
        _, flag = self.ctx.scale_disp_dev(
            holder['bal'].data_ptr() if n else None,
            sf.data_ptr() if sf.numel() else None, sf.dim() == 1,
            holder['row'].data_ptr() if n else None,
            holder['col'].data_ptr() if n else None, n, R, design,
            mean_thresh, dist_min,
            d_flag_out=holder['di'].data_ptr() if n else None,
            d_scaled_out=t_scaled.data_ptr() if n else None)
        del holder['bal']
        disp_idx = flag == 1
        amb = np.flatnonzero(flag == 2)
        if len(amb):
            rows = t_scaled[torch.from_numpy(amb).to(self.dev)].cpu().numpy()
            mean = np.dot(rows, design) / np.sum(design, axis=0)
            disp_idx[amb] = np.all(mean >= mean_thresh, axis=1) & \
                (dist[amb] >= dist_min)
            holder['di'].copy_(torch.from_numpy(disp_idx.view(np.uint8)))
        scaled, ready = to_host_async(t_scaled)
        return scaled, ready, disp_idx

    def keep(self, chrom, holder, disp_idx, bias, bias_stamps=None):
        """Registers a prepared chromosome (its stage files just queued).
        ``bias_stamps``: the bias files' stamps taken where they were read
        (bias_stamps(); prepare_data's reader thread), else taken here."""
        torch = self.torch
        n = int(holder['row'].shape[0])
        t_di = holder.get('di')
        if t_di is None:
            t_di = torch.from_numpy(np.ascontiguousarray(
                disp_idx, dtype=np.uint8)).to(self.dev)
        files = {self.h._npy(s, chrom): ('ours', self.h.write_generation(
            self.h._npy(s, chrom))) for s in self.STAGES}
        files.update(bias_stamps if bias_stamps is not None
                     else self._bias_stamps(chrom))
        self.chroms[chrom] = ChromDev(
            holder['row'], holder['col'], holder['raw'], holder['sf'],
            holder['sf'].dim() == 1, t_di, int(np.count_nonzero(disp_idx)),
            bias, files)
        if self.session is not None and chrom in self.session['chroms']:
            self.session = None
        return n

    # -- the chromosome's union, resident or from the outdir ------------
    def chrom(self, chrom):
        ent = self.chroms.get(chrom)
        if ent is not None and self._current(ent.files):
            return ent
        self.chroms.pop(chrom, None)
        return self._load(chrom)

    def _load(self, chrom):
        """The union of a chromosome another process (or an earlier object)
        prepared: read from the outdir files and uploaded once."""
        torch = self.torch
        h = self.h
        files = {}
        arrs = {}
        for s in self.STAGES:
            fname = h._npy(s, chrom)
            files[fname] = self._token(fname)
            arrs[s] = h.load_data(s, chrom)
        files.update(self._bias_stamps(chrom))
        raw = np.asarray(arrs['raw'])
        if raw.size and (raw.min() < 0 or raw.max() > np.iinfo(np.int32).max):
            raise _native.H3DError('raw counts must be in [0, 2^31)')
        sf = np.ascontiguousarray(arrs['size_factors'], dtype=np.float64)

        def up(a, dt):
            return torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(
                self.dev)
        di = np.asarray(arrs['disp_idx'], dtype=bool)
        ent = ChromDev(up(arrs['row'], np.int32), up(arrs['col'], np.int32),
                       up(raw, np.int32), up(sf, np.float64), sf.ndim == 1,
                       up(di, np.uint8), int(np.count_nonzero(di)),
                       h.load_bias(chrom), files)
        self.chroms[chrom] = ent
        return ent

    # -- estimate_disp / lrt inputs ---------------------------------------
    def disp_pixels(self, chroms, R):
        """raw (n, R) int32, f (n, R), dist (n) of the disp pixels of
        ``chroms`` concatenated in chromosome order (analysis.py:169-183),
        on the device, and the offsets between the chromosomes."""
        torch = self.torch
        ents = [self.chrom(c) for c in chroms]
        offsets = np.concatenate([[0], np.cumsum([e.n_disp for e in ents])])
        n = int(offsets[-1])
        t_raw = torch.empty((n, R), dtype=torch.int32, device=self.dev)
        t_f = torch.empty((n, R), dtype=torch.float64, device=self.dev)
        t_dist = torch.empty(n, dtype=torch.int32, device=self.dev)
        for e, o in zip(ents, offsets[:-1]):
            if not e.n:
                continue
            o = int(o)
            self.ctx.disp_pixels_dev(
                e.row.data_ptr(), e.col.data_ptr(), e.raw.data_ptr(),
                e.sf.data_ptr(), e.sf_per_rep, e.bias, e.disp_idx.data_ptr(),
                e.n, R, e.n_disp,
                t_raw.data_ptr() + o * R * 4 if e.n_disp else None,
                t_f.data_ptr() + o * R * 8 if e.n_disp else None,
                t_dist.data_ptr() + o * 4 if e.n_disp else None)
        return t_raw, t_f, t_dist, offsets

    def lrt_buffers(self, n, C):
        """The LRT's outputs for ``n`` pixels, device and host: (p / llr /
        mu0 as one (3, n) tensor, mu1 (n, C); their host destinations).
        estimate_disp allocates them before its own results start streaming
        to the host (analysis/d2h.py: a large host allocation waits for the
        copy thread's page faults), the session hands them to lrt once."""
        torch = self.torch
        if not n:
            return None
        return (torch.empty((3, n), dtype=torch.float64, device=self.dev),
                torch.empty((n, C), dtype=torch.float64, device=self.dev),
                np.empty((3, n)), np.empty((n, C)))

    def disp_keys(self, chroms, index):
        """parallel.PixelKeys of disp_pixels(chroms)' pixels, in the same
        order: each pixel's row, its chromosome's genome index (``index``:
        name -> index, the same on every rank) and its row of the
        chromosome's size-factor table -- the distinct size-factor rows of
        its disp pixels (torch.unique; a conditional norm has one per
        distance bin, a global one a single row) -- with every chromosome's
        filtered bias and that table: what the distance re-shard ships
        instead of f (h3d_pixel_f_dev rebuilds it bit for bit)."""
        from hic3defdr_amd import parallel
        torch = self.torch
        rows, gs, sfis, tables = [], [], [], {}
        for c in chroms:
            e = self.chrom(c)
            g = int(index[c])
            if e.sf_per_rep:
                tab = e.sf.reshape(1, -1)
            else:
                sel = e.disp_idx.bool()
                tab, inv = torch.unique(e.sf[sel], dim=0, return_inverse=True)
            tables[g] = (np.asarray(e.bias, dtype=np.float64),
                         tab.cpu().numpy())
            if not e.n_disp:
                continue
            sel = e.disp_idx.bool()
            rows.append(e.row[sel].to(torch.int32))
            gs.append(torch.full((e.n_disp,), g, dtype=torch.int32,
                                 device=self.dev))
            sfis.append(torch.zeros(e.n_disp, dtype=torch.int32,
                                    device=self.dev) if e.sf_per_rep
                        else inv.reshape(-1).to(torch.int32))

        def cat(parts):
            return torch.cat(parts) if parts else \
                torch.zeros(0, dtype=torch.int32, device=self.dev)
        return parallel.PixelKeys(cat(rows), cat(gs), cat(sfis), tables,
                                  len(index))

    def start_session(self, chroms, t_raw, t_f, t_dist, offsets, t_tab, D, C,
                      lrt_bufs=None):
        """estimate_disp's resident result for lrt: its pixels and device
        tables, valid while its disp files and its chromosomes' stage files
        are current; ``lrt_bufs`` (lrt_buffers) for the first lrt on it."""
        files = {}
        for c in chroms:
            files[self.h._npy('disp', c)] = self._token(self.h._npy('disp', c))
            files.update(self.chroms[c].files)
        self.session = {'chroms': tuple(chroms), 'raw': t_raw, 'f': t_f,
                        'dist': t_dist, 'offsets': offsets, 'tables': t_tab,
                        'D': D, 'C': C, 'files': files, 'bufs': lrt_bufs}

    def keep_pvalues(self, chroms, t_p, offsets):
        """lrt's device p-values of ``chroms`` (its pvalues files just
        queued), for bh while those files are current."""
        files = {self.h._npy('pvalues', c): self._token(
            self.h._npy('pvalues', c)) for c in chroms}
        self.pvals = {'chroms': tuple(chroms), 'p': t_p, 'offsets': offsets,
                      'files': files}

    def pvalues_session(self, chroms):
        """The kept p-values if they cover exactly ``chroms`` and their files
        are current."""
        s = getattr(self, 'pvals', None)
        if s is None or s['chroms'] != tuple(chroms):
            return None
        if not self._current(s['files']):
            self.pvals = None
            return None
        return s

    def lrt_session(self, chroms):
        """The session if it covers exactly ``chroms`` and is current."""
        s = self.session
        if s is None or s['chroms'] != tuple(chroms):
            return None
        if not self._current(s['files']):
            self.session = None
            return None
        return s
