"""Pipeline mixin (reference hic3defdr/analysis/analysis.py:24-364).

Same methods, signatures and outdir outputs as the reference; the per-pixel
work runs on the GPU through libh3d.so:

  prepare_data  -> h3d_union_count/fill (union + raw/balanced gathers),
                   h3d_size_factors (every norm of util/scaling.py)
  estimate_disp -> h3d_disp_per_dist (qcml per distance x condition),
                   h3d_disp_table (lowess smoother, host C++ in libh3d)
  lrt           -> h3d_lrt (fused per-pixel NB GLM fits + LRT + chi2)
  bh            -> h3d_bh_ctx (radix sort + reverse min-scan on the GPU)
  threshold / classify / collect
                -> h3d_find_clusters + h3d_format_clusters (host C++ in
                   libh3d: the reference's DirectedDisjointSet clustering and
                   the cluster JSON / TSV text)

``n_threads`` is accepted for signature compatibility: the reference's
process pools (util/parallelization.py) are replaced by the GPU. Under
torchrun (a torch.distributed process group is initialised) every stage
shards itself over the ranks (hic3defdr_amd.parallel): each rank owns the
chromosomes LPT assigns it for prepare_data and lrt, estimate_disp pools
the distances genome-wide by re-sharding the disp pixels by distance (one
all_to_all; every rank then runs the single-GPU driver on its distances),
and BH gathers the p-values on rank 0 and scatters the q-values back.
"""
import concurrent.futures
import os

import numpy as np
import scipy.sparse as sparse

from hic3defdr_amd import _native, numa, parallel
from hic3defdr_amd.analysis.core import DispFn
from hic3defdr_amd.analysis.d2h import small_to_host, to_host_async
from hic3defdr_amd.analysis.resident import bias_stamps
from hic3defdr_amd.util.classification import classify_clusters
from hic3defdr_amd.util.cluster_table import ClusterTable
from hic3defdr_amd.util.clusters import (load_cluster_list,
                                         load_cluster_pixels,
                                         pixel_membership, save_clusters)
from hic3defdr_amd.util.thresholding import threshold_clusters
from hic3defdr_amd.util.printing import eprint

NATIVE_NORMS = tuple(_native.H3D_NORM)
NATIVE_ESTIMATORS = ('qcml',)
# H3D_RESIDENT=0: prepare_data does not keep the union in HBM (estimate_disp
# and lrt then upload it from the outdir files, as a new process would)
_KEEP_RESIDENT = os.environ.get('H3D_RESIDENT', '1') != '0'
# chromosomes whose input files are read ahead of prepare_data's device work
# (H3D_PREP_AHEAD; 1 = the next one only). Measured on the cfg3 genome
# through run_to_qvalues (r06m, three interleaved runs each): 1.49-1.53 s at
# 1, 1.55-1.60 s at 2, 1.57-1.82 s at 3 -- more readers in flight contend
# with the outdir writers and the device thread for the host's cores
_PREP_AHEAD = int(os.environ.get('H3D_PREP_AHEAD', '1'))
_NPZ_PINNED = os.environ.get('H3D_NPZ_PINNED', '1') != '0'
_NUMA_DONE = []


def _pinned_bytes(nbytes):
    """A uint8 numpy array over pinned host memory (torch's caching host
    allocator: a freed block serves the next chromosome's archives, so
    the pinning is paid about once per run); pageable without torch or a
    device."""
    try:
        import torch
        return torch.empty(int(nbytes), dtype=torch.uint8,
                           pin_memory=True).numpy()
    except (ImportError, RuntimeError):   # no torch / no device to pin for
        return np.empty(int(nbytes), dtype=np.uint8)


def _canonical_csr(fname):
    """The replicate matrix as sorted, duplicate-free CSR rows (what the
    union kernels expect): libh3d's zlib reader for the CSR archives
    save_npz writes -- inflated into pinned host memory (H3D_NPZ_PINNED=0:
    pageable), so h3d_union_count's uploads are DMA copies instead of
    staged pageable ones -- scipy for any other sparse format load_npz
    takes (analysis.py:94,100)."""
    try:
        return _native.load_npz_csr(fname, alloc=_pinned_bytes
                                    if _NPZ_PINNED else None)
    except _native.H3DError:
        pass   # scipy reads it (or raises as the reference would)
    m = sparse.load_npz(fname).tocsr()
    m.sum_duplicates()
    return m


def _pixel_factors(bias, row, col, size_factors):
    """bias[row] * bias[col] * size_factors (analysis.py:181, :272-275), the
    same products in the same order, through np.take and in-place multiplies
    (half the time of the fancy-indexed expression's temporaries)."""
    f = np.take(bias, row, axis=0)
    f *= np.take(bias, col, axis=0)
    f *= size_factors
    return f


class AnalyzingHiC3DeFDR(object):

    def _ctx(self):
        dev = parallel.device_for_rank()
        if not _NUMA_DONE:
            # H3D_NUMA_BIND=1: this process's threads on its GPU's NUMA node
            # (numa.py), once, before the stages start their threads
            _NUMA_DONE.append(numa.maybe_bind(dev))
        return _native.context(dev)

    def _shards(self):
        """This rank's chromosomes (all of them without a process group);
        chromosome sizes read once per object."""
        sizes = self.__dict__.get('_chrom_sizes')
        if sizes is None:
            sizes = parallel.chrom_sizes(self.bias_patterns, self.chroms)
            self.__dict__['_chrom_sizes'] = sizes
        return parallel.Shards(self.chroms, sizes)

    def _barrier(self, sh):
        """The end of a sharded stage: this rank's queued outdir writes land
        first (core.py's write-behind), then the ranks meet -- so after the
        barrier every rank's files of the stage are on disk for any rank
        (threshold / classify / collect read every chromosome)."""
        if sh.dist is not None:
            self.flush()
            sh.barrier()

    def _cond_of_rep(self):
        d = np.asarray(self.design, dtype=bool)
        if not np.all(d.sum(axis=1) == 1):
            raise ValueError('every replicate must belong to exactly one '
                             'condition')
        return d.argmax(axis=1).astype(np.int32)

    # ------------------------------------------------------------------
    def prepare_data(self, chrom=None, norm='conditional_mor', n_bins=-1,
                     n_threads=-1, verbose=True):
        """Reference ``analysis.py:28-133``."""
        if n_bins == -1:
            n_bins = int(self.dist_thresh_max / 5)
        if norm not in NATIVE_NORMS:
            raise NotImplementedError(
                'norm=%r: the GPU path implements %s' % (norm, NATIVE_NORMS))
        if chrom is None:
            sh = self._shards()
            # the next chromosomes' files (NPZ inflate, bias, clusters) are
            # read on threads while one is prepared: _PREP_AHEAD of them in
            # flight, each inflating its replicates' archives on its own
            # threads
            ahead = max(1, _PREP_AHEAD)
            with concurrent.futures.ThreadPoolExecutor(ahead) as pre:
                futs = [pre.submit(self._prepare_inputs, c)
                        for c in sh.mine[:ahead]]
                for i, c in enumerate(sh.mine):
                    inputs = futs[i].result()
                    futs[i] = None
                    if i + ahead < len(sh.mine):
                        futs.append(pre.submit(self._prepare_inputs,
                                               sh.mine[i + ahead]))
                    self._prepare_chrom(c, norm, n_bins, verbose, inputs)
            self._barrier(sh)
            return
        self._prepare_chrom(chrom, norm, n_bins, verbose,
                            self._prepare_inputs(chrom))

    def _prepare_inputs(self, chrom):
        """One chromosome's input files: bias (load_bias, and the bias
        files' stamps for the resident session), the replicates' canonical
        CSR matrices (their NPZ archives inflated concurrently: zlib inflate
        and crc32 release the GIL) and the loop clusters."""
        with concurrent.futures.ThreadPoolExecutor(
                min(8, len(self.raw_npz_patterns))) as ex:
            fut = [ex.submit(_canonical_csr, p.replace('<chrom>', chrom))
                   for p in self.raw_npz_patterns]
            # stamped before reading: a file replaced while it is read shows
            # as changed to the session's validity checks
            stamps = bias_stamps(self.bias_patterns, chrom) \
                if _KEEP_RESIDENT else None
            bias = self.load_bias(chrom)
            # the clusters' pixels as arrays (loop_idx needs only their
            # union; parsed in C, not as Python sets of tuples)
            cl = [load_cluster_pixels(p.replace('<chrom>', chrom))
                  for p in self.loop_patterns.values()] \
                if self.loop_patterns else None
            mats = [f.result() for f in fut]
        return bias, mats, cl, stamps

    def _prepare_chrom(self, chrom, norm, n_bins, verbose, inputs):
        """prepare_data of one chromosome (analysis.py:28-133) from its
        input files (_prepare_inputs)."""
        eprint('preparing data for chrom %s' % chrom, skip=not verbose)
        bias, mats, cl, stamps = inputs
        ctx = self._ctx()
        res = self._resident() if _KEEP_RESIDENT else None
        holder = {}
        eprint('  computing union pixel set', skip=not verbose)
        try:
            row, col, raw, balanced = ctx.sparse_union(
                mats, bias, self.dist_thresh_max,
                device_alloc=res.union_alloc(holder) if res else None,
                host_balanced=res is None, host_raw=res is None)
        except _native.H3DError as e:
            # only counts beyond int32 (the device copy's width) fall back to
            # the host union; every other failure (HIP errors, out of memory
            # while allocating the device copy) propagates
            if not holder or e.code != _native.H3D_EINPUT:
                raise
            # counts beyond int32: no device copy (the disp / lrt kernels
            # reject such counts anyway, as before)
            res, holder = None, {}
            row, col, raw, balanced = ctx.sparse_union(mats, bias,
                                                       self.dist_thresh_max)
        eprint('  computing size factors', skip=not verbose)
        dist = col - row
        design = np.asarray(self.design, dtype=bool)
        ready = {}
        if raw is None:
            # the union's counts leave the device in the background (int32
            # there, the outdir's int64 here; analysis/d2h.py)
            raw, ready['raw'] = to_host_async(holder['raw'], dtype=np.int64)
        # analysis.py:104-108: conditional norms see the distances
        if res is not None and 'bal' in holder:
            size_factors, ready['size_factors'] = res.size_factors(
                holder, dist, norm, n_bins or 0)
            # analysis.py:109-115 on the device (h3d_scale_disp_dev)
            scaled, ready['scaled'], disp_idx = res.scale_disp(
                holder, design, self.mean_thresh, self.dist_thresh_min, dist)
        else:
            size_factors = ctx.size_factors(balanced, dist, norm, n_bins or 0)
            scaled = balanced / size_factors
            mean = np.dot(scaled, design) / np.sum(design, axis=0)
            disp_idx = np.all(mean >= self.mean_thresh, axis=1) & \
                (dist >= self.dist_thresh_min)
        if self.loop_patterns:
            eprint('  making loop_idx', skip=not verbose)
            loop_idx = pixel_membership(row, col, cl, mask=disp_idx)
            self._save_npy(self._npy('loop_idx', chrom), loop_idx, owned=True)
        eprint('  saving data to disk', skip=not verbose)
        for name, a in (('row', row), ('col', col), ('raw', raw),
                        ('size_factors', size_factors), ('scaled', scaled),
                        ('disp_idx', disp_idx)):
            self._save_npy(self._npy(name, chrom), a, owned=True,
                           ready=ready.get(name))
        if res is not None and 'sf' in holder:
            res.keep(chrom, holder, disp_idx, bias, bias_stamps=stamps)

    # ------------------------------------------------------------------
    def _f_and_dist(self, chroms=None):
        """raw/f/dist of the disp pixels of ``chroms`` (default all),
        concatenated in chromosome order (reference ``analysis.py:169-183``),
        and the offsets between the chromosomes."""
        chroms = self.chroms if chroms is None else chroms
        raws, fs, dists = [], [], []
        for chrom in chroms:
            di = self.load_data('disp_idx', chrom)
            row = self.load_data('row', chrom, idx=di)
            col = self.load_data('col', chrom, idx=di)
            raws.append(self.load_data('raw', chrom, idx=di))
            bias = self.load_bias(chrom)
            sf = self.load_data('size_factors', chrom)
            # per-replicate (1-D) factors of the non-conditional norms
            # broadcast over the pixels, as lrt uses them (analysis.py:272-275).
            # Deviation: the reference indexes them with the pixel mask here
            # (analysis.py:181) and raises IndexError.
            if sf.ndim == 2:
                sf = sf[di]
            fs.append(_pixel_factors(bias, row, col, sf))
            dists.append(col - row)
        R = self.design.shape[0]
        offsets = np.concatenate([[0], np.cumsum([len(r) for r in raws])])
        if not raws:
            return (np.zeros((0, R), dtype=np.int64), np.zeros((0, R)),
                    np.zeros(0, dtype=np.int32), offsets)
        return np.concatenate(raws), np.concatenate(fs), \
            np.concatenate(dists), offsets

    def _resident(self):
        """The device copy of this object's stages (analysis/resident.py)."""
        r = self.__dict__.get('_dev_resident')
        if r is None or r.ctx is not self._ctx():
            try:
                from hic3defdr_amd.analysis.resident import Resident
                r = Resident(self)
            except ImportError as e:
                raise _native.H3DError(
                    'the GPU path needs torch (device memory): %s' % e)
            self.__dict__['_dev_resident'] = r
        return r

    def _disp_per_dist_sharded(self, t_raw, t_f, t_dist, C, D):
        """estimate_disp's per-(distance, condition) qcml over every rank's
        pixels: re-sharded by distance (parallel.disp_per_dist_by_distance:
        one all_to_all, the single-GPU driver per rank, one all-reduce of the
        table), or with H3D_DISP_SHARD=pass kept in place with the NLL sums
        of each data pass all-reduced (parallel.make_allreduce); every rank
        ends with the same disp_per_dist."""
        import torch
        ctx = self._ctx()
        dev = torch.device('cuda', ctx.device)
        torch.cuda.set_device(dev)
        # torch's stream only: a device-wide synchronize would also wait for
        # the background copies of earlier stages' results (analysis/d2h.py,
        # their own stream); libh3d's calls return with its stream drained
        torch.cuda.current_stream(dev).synchronize()
        # a real stream shared by libh3d and the collective: torch's default
        # stream has handle 0, which h3d_set_stream reads as "the ctx's own
        # stream" -- the all-reduce would then race the kernels around it
        stream = torch.cuda.Stream(dev)
        ctx.set_stream(stream.cuda_stream)
        try:
            with torch.cuda.stream(stream):
                if os.environ.get('H3D_DISP_SHARD') != 'pass':
                    # the keys of f travel instead of f (15-byte records at
                    # R = 4; H3D_RESHARD_FULL=1: the full 52-byte record)
                    keys = None if os.environ.get('H3D_RESHARD_FULL') == '1' \
                        else self._resident().disp_keys(
                            self._shards().mine,
                            {c: i for i, c in enumerate(self.chroms)})
                    return parallel.disp_per_dist_by_distance(
                        ctx, t_raw, t_f, t_dist, self._cond_of_rep(), C, D,
                        keys=keys)
                return ctx.disp_per_dist_dev(
                    t_raw.data_ptr(), t_f.data_ptr(), t_dist.data_ptr(),
                    t_raw.shape[0], self.design.shape[0], self._cond_of_rep(),
                    C, D, reduce=parallel.make_allreduce())
        finally:
            stream.synchronize()
            ctx.set_stream(None)

    def estimate_disp(self, estimator='qcml', frac=None, auto_frac_factor=15.,
                      weighted_lowess=True, n_threads=-1):
        """Reference ``analysis.py:135-223``. The native estimator runs on
        the device end to end (resident.py): the disp pixels of this rank's
        chromosomes built in HBM, qcml per (distance, condition), the
        smoothed tables and ``disp = table[dist]``; disp goes to the outdir
        (write-behind) and stays resident for lrt."""
        eprint('estimating dispersion')
        sh = self._shards()
        design = np.asarray(self.design, dtype=bool)
        R, C = design.shape
        D = self.dist_thresh_max + 1
        if callable(estimator) or estimator not in NATIVE_ESTIMATORS:
            if sh.sharded:
                raise NotImplementedError(
                    'sharded estimate_disp implements %s' % (NATIVE_ESTIMATORS,))
            if not callable(estimator):
                raise NotImplementedError(
                    'estimator=%r: the reference divides its int64 raw slice '
                    'in place for cml/mme (dispersion.py:76,129) and raises; '
                    'the GPU path implements %s' % (estimator,
                                                    NATIVE_ESTIMATORS))
            return self._estimate_disp_callable(estimator, frac,
                                                auto_frac_factor,
                                                weighted_lowess)
        import torch
        res = self._resident()
        ctx = self._ctx()
        cond = self._cond_of_rep()
        t_raw, t_f, t_dist, offsets = res.disp_pixels(sh.mine, R)
        n = int(t_raw.shape[0])
        t_tab = torch.empty((D, C), dtype=torch.float64, device=res.dev)
        t_disp = torch.empty((n, C), dtype=torch.float64, device=res.dev)
        # lrt's outputs, allocated before the disp copy below starts paging in
        # its host array (resident.lrt_buffers)
        lrt_bufs = res.lrt_buffers(n, C)
        if sh.sharded:
            disp_per_dist = self._disp_per_dist_sharded(t_raw, t_f, t_dist, C,
                                                        D)
            t_dpd = torch.from_numpy(np.ascontiguousarray(disp_per_dist)).to(
                res.dev)
            torch.cuda.current_stream(res.dev).synchronize()
            ctx.disp_tables_dev(t_dpd.data_ptr(), D, C, t_tab.data_ptr(),
                                weighted=weighted_lowess, frac=frac,
                                auto_frac_factor=auto_frac_factor)
        else:
            # torch's stream only (the allocations above): a device-wide
            # synchronize also waited for prepare_data's background result
            # copies (d2h.py, their own stream) -- up to ~30 ms of cfg2's
            # estimate_disp through the class
            torch.cuda.current_stream(res.dev).synchronize()
            disp_per_dist = ctx.estimate_disp_dev(
                t_raw.data_ptr() if n else None, t_f.data_ptr() if n else None,
                t_dist.data_ptr() if n else None, n, R, cond, C, D,
                t_tab.data_ptr(), weighted=weighted_lowess, frac=frac,
                auto_frac_factor=auto_frac_factor)
        eprint('  fitting distance vs dispersion relationship')
        # settles the device smoother (a degenerate fit is redone on the host)
        ctx.table_gather_dev(t_tab.data_ptr(), D, C,
                             t_dist.data_ptr() if n else None, n,
                             t_disp.data_ptr() if n else None)
        # (table_gather_dev returns with the ctx stream drained); the per-pixel
        # disp goes to the outdir by a copy into pageable host memory on a
        # background thread (analysis/d2h.py; pinning measured slower there)
        tables = small_to_host(t_tab)
        disp, disp_ready = to_host_async(t_disp)
        del t_disp
        if sh.rank == 0:
            for c, cond_name in enumerate(self.design.columns):
                self.save_disp_fn(cond_name, DispFn(tables[:, c],
                                                    disp_per_dist[:, c],
                                                    weighted=weighted_lowess))
        eprint('  saving estimated dispersions to disk')
        for i, chrom in enumerate(sh.mine):
            self._save_npy(self._npy('disp', chrom),
                           disp[offsets[i]:offsets[i + 1]], owned=True,
                           ready=disp_ready)
        if sh.rank == 0:
            self.save_data(disp_per_dist, 'disp_per_dist')
        res.start_session(sh.mine, t_raw, t_f, t_dist, offsets, t_tab, D, C,
                          lrt_bufs)
        self._barrier(sh)

    def _estimate_disp_callable(self, estimator, frac, auto_frac_factor,
                                weighted_lowess):
        """A user-supplied Python estimator runs where the user wrote it, on
        the host (analysis.py:164-165, :196-206)."""
        design = np.asarray(self.design, dtype=bool)
        C = design.shape[1]
        D = self.dist_thresh_max + 1
        raw, f, dist, offsets = self._f_and_dist()
        disp_per_dist = np.zeros((D, C))
        for c in range(C):
            for d in range(D):
                sel = dist == d
                rs = raw[sel][:, design[:, c]]
                fs = f[sel][:, design[:, c]]
                disp_per_dist[d, c] = np.nan if not rs.size else \
                    estimator(rs, f=fs)
        eprint('  fitting distance vs dispersion relationship')
        tables = _native.disp_tables(disp_per_dist, weighted=weighted_lowess,
                                     frac=frac,
                                     auto_frac_factor=auto_frac_factor)
        disp = np.zeros((len(raw), C))
        for c, cond in enumerate(self.design.columns):
            disp[:, c] = tables[:, c][dist]
            self.save_disp_fn(cond, DispFn(tables[:, c], disp_per_dist[:, c],
                                           weighted=weighted_lowess))
        eprint('  saving estimated dispersions to disk')
        for i, chrom in enumerate(self.chroms):
            self._save_npy(self._npy('disp', chrom),
                           disp[offsets[i]:offsets[i + 1]], owned=True)
        self.save_data(disp_per_dist, 'disp_per_dist')

    # ------------------------------------------------------------------
    def lrt(self, chrom=None, refit_mu=True, n_threads=-1, verbose=True):
        """Reference ``analysis.py:225-284``, on the device: over
        estimate_disp's resident pixels and tables in one launch while its
        disp files are current (resident.py), otherwise per chromosome from
        the outdir (the per-pixel disp as the reference loads it)."""
        sh = self._shards() if chrom is None else None
        chroms = sh.mine if chrom is None else [chrom]
        res = self._resident()
        sess = res.lrt_session(chroms) if chrom is None else None
        if sess is not None:
            for c in chroms:
                eprint('running LRT for chrom %s' % c, skip=not verbose)
            # the session's preallocated outputs serve its first lrt only
            # (the host arrays then belong to the outdir queue)
            bufs, sess['bufs'] = sess.get('bufs'), None
            self._lrt_run(res, chroms, sess['raw'], sess['f'], sess['dist'],
                          sess['offsets'], refit_mu, table=sess['tables'],
                          bufs=bufs)
        else:
            for c in chroms:
                eprint('running LRT for chrom %s' % c, skip=not verbose)
                t_raw, t_f, t_dist, offsets = res.disp_pixels([c],
                                                              len(self.design))
                disp = self.load_data('disp', c)
                self._lrt_run(res, [c], t_raw, t_f, None, offsets, refit_mu,
                              disp=disp)
        if sh is not None:
            self._barrier(sh)

    def _lrt_run(self, res, chroms, t_raw, t_f, t_dist, offsets, refit_mu,
                 table=None, disp=None, bufs=None):
        """One LRT launch over the concatenated disp pixels of ``chroms``:
        with the device ``table`` (D, C) and t_dist, or the per-pixel
        ``disp`` (n, C) from the outdir; the four outputs saved per
        chromosome (write-behind). ``bufs``: preallocated outputs
        (Resident.lrt_buffers)."""
        import torch
        ctx = self._ctx()
        n = int(t_raw.shape[0])
        C = self.design.shape[1]
        if n and (bufs is None or bufs[0].shape[1] != n
                  or bufs[1].shape[1] != C):
            bufs = res.lrt_buffers(n, C)
        if n:
            tp, t1, h3_dst, h1_dst = bufs
            ptrs = (tp[0].data_ptr(), tp[1].data_ptr(), tp[2].data_ptr(),
                    t1.data_ptr())
            if table is not None:
                ctx.lrt_dev_tab(t_raw.data_ptr(), t_f.data_ptr(),
                                t_dist.data_ptr(), table.data_ptr(),
                                table.shape[0], n, len(self.design),
                                self._cond_of_rep(), *ptrs, refit_mu=refit_mu)
            else:
                ctx.lrt_dev(t_raw.data_ptr(), t_f.data_ptr(), None, disp, n,
                            len(self.design), self._cond_of_rep(), *ptrs,
                            refit_mu=refit_mu)
            # (the lrt calls return with the ctx stream drained); the outputs
            # reach the outdir by background copies (analysis/d2h.py), waited
            # for by their writer / first reader
            h3, r3 = to_host_async(tp, dst=h3_dst)
            mu1, r1 = to_host_async(t1, dst=h1_dst)
        else:
            tp = None
            h3, mu1 = np.empty((3, 0)), np.empty((0, C))
            r3 = r1 = None
        p, llr, mu0 = h3
        for i, c in enumerate(chroms):
            a, b = offsets[i], offsets[i + 1]
            self._save_npy(self._npy('pvalues', c), p[a:b], owned=True,
                           ready=r3)
            self._save_npy(self._npy('llr', c), llr[a:b], owned=True,
                           ready=r3)
            self._save_npy(self._npy('mu_hat_null', c), mu0[a:b], owned=True,
                           ready=r3)
            self._save_npy(self._npy('mu_hat_alt', c), mu1[a:b], owned=True,
                           ready=r1)
        if table is not None and tp is not None:
            res.keep_pvalues(chroms, tp[0], offsets)

    # ------------------------------------------------------------------
    def bh(self):
        """Reference ``analysis.py:286-303``."""
        eprint('applying BH-FDR correction')
        sh = self._shards()
        if sh.sharded:
            mine = {}
            for chrom in sh.mine:
                li = self.load_data('loop_idx', chrom) \
                    if self.loop_patterns else None
                mine[chrom] = self.load_data('pvalues', chrom, idx=li)
            for chrom, q in parallel.distributed_bh(
                    sh, mine, ctx=self._ctx()).items():
                self.save_data(q, 'qvalues', chrom)
            self._barrier(sh)
            return
        loop_idx = self.load_data('loop_idx', 'all')[0] \
            if self.loop_patterns else None
        # lrt's device p-values, when this object ran lrt and they are current
        res = self.__dict__.get('_dev_resident') if _KEEP_RESIDENT else None
        pv = res.pvalues_session(self.chroms) \
            if res is not None and res.ctx is self._ctx() else None
        if pv is not None:
            self._bh_resident(pv, loop_idx)
            return
        pvalues, offsets = self.load_data('pvalues', 'all', idx=loop_idx)
        q = self._ctx().bh(pvalues)
        for i, chrom in enumerate(self.chroms):
            self.save_data(q[offsets[i]:offsets[i + 1]], 'qvalues', chrom)

    def _bh_resident(self, pv, loop_idx):
        """bh on lrt's device p-values (the pvalues files hold the same
        values): the loop pixels gathered on the device, h3d_bh_dev, q-values
        to the outdir by the background copy."""
        import torch
        ctx = self._ctx()
        t_p, offsets = pv['p'], np.asarray(pv['offsets'])
        if loop_idx is not None:
            loop_idx = np.asarray(loop_idx, dtype=bool)
            sel = np.flatnonzero(loop_idx)
            t_p = t_p.index_select(0, torch.from_numpy(sel).to(t_p.device))
            offsets = np.concatenate([[0], np.cumsum(
                [np.count_nonzero(loop_idx[a:b])
                 for a, b in zip(offsets[:-1], offsets[1:])])])
        n = int(t_p.shape[0])
        t_q = torch.empty(n, dtype=torch.float64, device=t_p.device)
        # on a torch stream shared with libh3d, so the copy's event covers it
        stream = torch.cuda.Stream(t_p.device)
        stream.wait_stream(torch.cuda.current_stream(t_p.device))
        ctx.set_stream(stream.cuda_stream)
        try:
            with torch.cuda.stream(stream):
                if n:
                    ctx.bh_dev(t_p.data_ptr(), n, t_q.data_ptr())
                q, ready = to_host_async(t_q)
        finally:
            ctx.set_stream(None)
        for i, chrom in enumerate(self.chroms):
            self._save_npy(self._npy('qvalues', chrom),
                           q[offsets[i]:offsets[i + 1]], owned=True,
                           ready=ready)

    def run_to_qvalues(self, norm='conditional_mor', n_bins_norm=-1,
                       estimator='qcml', frac=None, auto_frac_factor=15.,
                       weighted_lowess=True, refit_mu=True, n_threads=-1,
                       verbose=True):
        """Reference ``analysis.py:305-364``."""
        self.prepare_data(norm=norm, n_bins=n_bins_norm, n_threads=n_threads,
                          verbose=verbose)
        self.estimate_disp(estimator=estimator, frac=frac,
                           auto_frac_factor=auto_frac_factor,
                           weighted_lowess=weighted_lowess,
                           n_threads=n_threads)
        self.lrt(refit_mu=refit_mu, n_threads=n_threads, verbose=verbose)
        self.bh()
        # every stage's outdir file (every rank's, under torchrun: bh ends
        # with _barrier) has landed when the pipeline returns
        self.flush()

    # ------------------------------------------------------------------
    def _chroms_for(self, chrom):
        return self.chroms if chrom is None else [chrom]

    def threshold(self, chrom=None, fdr=0.05, cluster_size=3, n_threads=-1):
        """Reference ``analysis.py:366-431``: sig / insig clusters per FDR
        and cluster size -> ``sig_<fdr>_<size>_<chrom>.json`` (+ ``.tsv``
        when ``res`` is set), same for ``insig``."""
        fdrs = list(fdr) if hasattr(fdr, '__len__') else [fdr]
        sizes = list(cluster_size) if hasattr(cluster_size, '__len__') \
            else [cluster_size]
        for ch in self._chroms_for(chrom):
            eprint('thresholding and clustering chrom %s' % ch)
            row, col, q = self.load_data('qvalues', ch, coo=True)
            for f in fdrs:
                sig, insig = threshold_clusters(q, row, col, f)
                for s in sizes:
                    for kind, cl in (('sig', sig), ('insig', insig)):
                        kept = cl.size_filter(s)
                        out = '%s/%s_%g_%i_%s.json' % (self.outdir, kind, f, s,
                                                       ch)
                        save_clusters(kept, out)
                        if self.res is not None:
                            ClusterTable.from_clusters(kept, ch, self.res)\
                                .to_tsv(out.replace('.json', '.tsv'))

    def classify(self, chrom=None, fdr=0.05, cluster_size=3, n_threads=-1):
        """Reference ``analysis.py:433-486``: significant pixels take the
        condition of their largest alt-model mean and are re-clustered per
        condition -> ``<cond>_<fdr>_<size>_<chrom>.json`` (+ ``.tsv``)."""
        fdrs = list(fdr) if hasattr(fdr, '__len__') else [fdr]
        sizes = list(cluster_size) if hasattr(cluster_size, '__len__') \
            else [cluster_size]
        for ch in self._chroms_for(chrom):
            eprint('classifying differential interactions on chrom %s' % ch)
            disp_idx = self.load_data('disp_idx', ch)
            loop_idx = self.load_data('loop_idx', ch)
            row = self.load_data('row', ch, idx=(disp_idx, loop_idx))
            col = self.load_data('col', ch, idx=(disp_idx, loop_idx))
            mu_hat_alt = self.load_data('mu_hat_alt', ch, idx=loop_idx)
            for f in fdrs:
                for s in sizes:
                    infile = '%s/sig_%g_%i_%s.json' % (self.outdir, f, s, ch)
                    if not os.path.isfile(infile):
                        self.threshold(chrom=ch, fdr=f, cluster_size=s)
                    sig = load_cluster_list(infile)
                    per_class = classify_clusters(row, col, mu_hat_alt, sig)
                    for i, cl in enumerate(per_class):
                        out = '%s/%s_%g_%i_%s.json' % (
                            self.outdir, self.design.columns[i], f, s, ch)
                        save_clusters(cl, out)
                        if self.res is not None:
                            ClusterTable.from_clusters(cl, ch, self.res)\
                                .to_tsv(out.replace('.json', '.tsv'))

    def collect(self, fdr=0.05, cluster_size=3, n_threads=-1):
        """Reference ``analysis.py:488-572``: every chromosome's insig
        ("constitutive") and per-condition tables -> one sorted
        ``results_<fdr>_<size>.tsv`` with a ``classification`` column."""
        if self.res is None:
            raise ValueError(
                'the collect() step can only be run if the res kwarg was '
                'passed during construction of the HiC3DeFDR object; please '
                'run the classify() step instead or re-create the HiC3DeFDR '
                'object (you do not need to re-run any other steps)')
        eprint('collecting differential interactions')
        fdrs = list(fdr) if hasattr(fdr, '__len__') else [fdr]
        sizes = list(cluster_size) if hasattr(cluster_size, '__len__') \
            else [cluster_size]
        conds = list(self.design.columns)
        for f in fdrs:
            for s in sizes:
                pattern = '%s/<class>_%g_%i_<chrom>.tsv' % (self.outdir, f, s)

                def path(k, ch):
                    return pattern.replace('<class>', k).replace('<chrom>', ch)
                if not all(os.path.isfile(path('insig', ch))
                           for ch in self.chroms):
                    self.threshold(fdr=f, cluster_size=s)
                if not all(os.path.isfile(path(c, ch)) for c in conds
                           for ch in self.chroms):
                    self.classify(fdr=f, cluster_size=s)
                tables = []
                for ch in self.chroms:
                    tables.append(ClusterTable.read_tsv(path('insig', ch))
                                  .with_classification('constitutive'))
                    for c in conds:
                        tables.append(ClusterTable.read_tsv(path(c, ch))
                                      .with_classification(c))
                ClusterTable.concat(tables).sorted().to_tsv(
                    '%s/results_%g_%i.tsv' % (self.outdir, f, s))
