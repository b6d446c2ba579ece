"""Persistence mixin (reference hic3defdr/analysis/core.py): the outdir is the
contract between stages — ``<outdir>/<name>_<chrom>.npy`` per chromosome,
``disp_per_dist.npy``, ``disp_fn_<cond>.pickle`` and ``pickle``."""
import atexit
import collections
import concurrent.futures
import ctypes
import os
import pickle
import sys
import threading
import zlib

import numpy as np


def _write_npy(fname, data, ready=None):
    if ready is not None:
        ready()      # an async device -> host copy still landing in `data`
    np.save(fname, data)
    st = os.stat(fname)
    return (st.st_ino, st.st_size, st.st_mtime_ns, st.st_ctime_ns)


def _load_column(fname):
    """np.loadtxt of a one-column text file, parsed by libh3d when it takes
    the file (_native.read_text_column: the same values, no GIL held)."""
    from hic3defdr_amd import _native
    col = _native.read_text_column(fname)
    return np.loadtxt(fname) if col is None else col


def _write_bytes(fname, blob):
    with open(fname, 'wb') as fh:
        fh.write(blob)


class _NpyWriter(object):
    """The outdir's write-behind threads: queued .npy writes land on
    background threads (the product's stages hand their results over and go
    on; reference core.py:198-218 writes them inline). A file's writes go to
    one lane (a single thread chosen by the file name), so they land in
    order; different files land in parallel on H3D_NPY_WRITERS lanes
    (default 4: prepare_data's ~0.5 GB of cfg2 arrays is page-cache copying
    that scales with threads). Worker threads of concurrent.futures are
    joined at interpreter exit, so every queued write lands; an error of one
    is reported on stderr there if nobody read it."""

    def __init__(self):
        self._lock = threading.Lock()
        self._ex = None
        self._futs = []

    def submit(self, fname, data, ready=None, fn=None):
        """Queues np.save of ``data`` (or ``fn(fname, data)``) on the lane
        of ``fname``."""
        with self._lock:
            if self._ex is None:
                n = max(1, int(os.environ.get('H3D_NPY_WRITERS', '4')))
                self._ex = [concurrent.futures.ThreadPoolExecutor(
                    1, thread_name_prefix='h3d-npy%d' % i) for i in range(n)]
                atexit.register(self._report)
            self._futs = [f for f in self._futs if not f.done()]
            lane = zlib.crc32(os.fsencode(os.path.abspath(fname))) % \
                len(self._ex)
            fut = self._ex[lane].submit(_write_npy, fname, data, ready) \
                if fn is None else self._ex[lane].submit(fn, fname, data)
            self._futs.append(fut)
            return fut

    def _report(self):
        for f in list(self._futs):
            try:
                f.result()
            except Exception as e:   # noqa: BLE001 -- exit-time report
                sys.stderr.write('hic3defdr_amd: outdir write failed: %r\n'
                                 % (e,))


_WRITER = _NpyWriter()


class _Reaper(object):
    """Drops the outdir's large host arrays on a background thread. Freeing
    a large numpy buffer unmaps its pages: ~36 ms per GB on the GPU box's
    host (7 ms for a 200 MB array, measured r05), paid by whichever thread
    drops the last reference -- the cache's evictions put ~0.35 s of it on
    the main thread of a whole-genome prepare_data. Handed here, the frees
    run while the main thread waits in libh3d / HIP calls (which release the
    GIL). The arrays are immutable once queued (core._save_npy), so dropping
    them elsewhere changes nothing but where the unmapping runs."""

    _MIN_BYTES = 8 << 20

    def __init__(self):
        self._lock = threading.Lock()
        self._q = None

    @staticmethod
    def _release_pages(a):
        """Returns the pages of numpy array ``a`` to the kernel with
        madvise(MADV_DONTNEED) through ctypes -- which drops the GIL -- when
        this thread holds the only reference to it and it owns its buffer:
        the free() that follows then unmaps mostly released pages. numpy
        frees a buffer while holding the GIL, so a large free on this thread
        used to stall every Python thread (~36 ms per GB on the GPU box; the
        main thread's GIL waits showed up in every call of prepare_data).
        H3D_REAP_MADVISE=0 turns it off."""
        if not _MADVISE or not isinstance(a, np.ndarray) or \
                not a.flags.owndata or a.nbytes < _Reaper._MIN_BYTES:
            return
        # nobody else holds it: the references are _run's local, this
        # frame's ``a`` and getrefcount's argument (a view's base or any
        # other holder makes it more, and the pages stay)
        if sys.getrefcount(a) > 3:
            return
        libc = _libc()
        if libc is None:
            return
        page = 4096
        addr = a.ctypes.data
        lo = (addr + page - 1) // page * page
        hi = (addr + a.nbytes) // page * page
        if hi > lo:
            libc.madvise(ctypes.c_void_p(lo), ctypes.c_size_t(hi - lo), 4)

    def _run(self):
        q = self._q
        while True:
            obj = q.get()
            arrs = list(obj) if isinstance(obj, tuple) else [obj]
            obj = None
            while arrs:
                a = arrs.pop()
                self._release_pages(a)
                a = None

    def drop(self, obj, nbytes):
        if nbytes < self._MIN_BYTES:
            return
        with self._lock:
            if self._q is None:
                import queue
                self._q = queue.SimpleQueue()
                threading.Thread(target=self._run, name='h3d-reap',
                                 daemon=True).start()
        self._q.put(obj)


_MADVISE = os.environ.get('H3D_REAP_MADVISE', '1') != '0' and \
    sys.platform.startswith('linux')
_LIBC = []


def _libc():
    if not _LIBC:
        try:
            lib = ctypes.CDLL(None, use_errno=True)
            lib.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_int]
            lib.madvise.restype = ctypes.c_int
            _LIBC.append(lib)
        except (OSError, AttributeError):
            _LIBC.append(None)
    return _LIBC[0]


_REAPER = _Reaper()


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
    it. On top of that, in the reference's order:

    - ``lowess_fit``'s left boundary (``lowess.py:84-85``): every
      ``x <= left_boundary`` (= the first finite dispersion value,
      ``analysis.py:212``) returns the fit at its leftmost knot;
    - the weighted fit then replaces everything below ``x[inc_idx]`` by
      linear interpolation of the raw (distance, dispersion) points, and below
      the first fitted distance by ``y[0]`` (``lowess.py:229-242``).
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
        self.left_boundary = float(self.y[0])
        # leftmost lowess knot: the first expanded (weighted) or fitted x
        self.left_value = float(self.table[int(self.x[self.inc_idx])])

    def __call__(self, x_star):
        x = np.asarray(x_star, dtype=float)
        t = self.table
        xi = np.rint(x)
        on_knot = (xi == x) & (xi >= 0) & (xi < len(t))
        out = np.empty(x.shape, dtype=float)
        out[on_knot] = t[xi[on_knot].astype(np.int64)]
        off = ~on_knot
        if off.any():
            out[off] = _interp_extrap(np.arange(len(t), dtype=float), t,
                                      x[off])
        out[x <= self.left_boundary] = self.left_value
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
        bias = np.column_stack([_load_column(p.replace('<chrom>', chrom))
                                for p in self.bias_patterns])
        lo, hi = self.bias_thresh, 1. / self.bias_thresh
        bias[((bias < lo) | (bias > hi)).any(axis=1)] = 0
        return bias

    # -- outdir arrays --------------------------------------------------
    # Which pixel set a per-chromosome stage array is parallel to, as the mask
    # chain that selects its (row, col) from the union pixel set
    # (reference core.py:117-134). Stages not listed cannot be loaded as COO.
    _PIXEL_SET = dict(
        [(n, ()) for n in ('raw', 'size_factors', 'scaled', 'disp_idx')] +
        [(n, ('disp_idx',)) for n in ('loop_idx', 'disp', 'mu_hat_null',
                                      'mu_hat_alt', 'llr', 'pvalues')] +
        [('qvalues', ('disp_idx', 'loop_idx'))])
    _NOT_COO = frozenset(['row', 'col', 'bias', 'cov_per_bin',
                          'disp_per_bin'])

    def _npy(self, name, chrom=None):
        return '%s/%s.npy' % (self.outdir, name) if chrom is None \
            else '%s/%s_%s.npy' % (self.outdir, name, chrom)

    def _column(self, rep, cond):
        """Column of a (pixels, reps) / (pixels, conds) array, or None."""
        if rep is not None:
            return list(self.design.index).index(rep)
        if cond is not None:
            return list(self.design.columns).index(cond)
        return None

    @staticmethod
    def _narrow(mask, sub):
        """The entries of boolean ``mask`` that ``sub`` (parallel to the True
        entries of ``mask``) keeps: index chaining (reference core.py:141-145)."""
        out = np.zeros_like(mask)
        out[np.flatnonzero(mask)[sub]] = True
        return out

    # Write-through cache of the outdir arrays this object saved: a later
    # stage reading its own output back skips the disk read -- but only while
    # the file on disk is still the one written (same inode, size, mtime and
    # ctime; a rewrite that restores the mtime still moves the ctime), so
    # edits or replacements of the outdir files are always seen. Bounded: an
    # LRU over the arrays' bytes, at most H3D_NPY_CACHE_BYTES (default
    # 1 GiB; 0 turns the cache off), so a whole-genome run does not keep a
    # second copy of every stage of every chromosome on the host.
    #
    # Writes are behind (_WRITER, one background thread, FIFO): save_data
    # returns once the array is queued; until its write has landed the
    # queued array IS the file's content for every reader in this process
    # (load_data serves it, a reader of the file on disk waits for it), and
    # flush() / interpreter exit wait for every queued write (an error of a
    # write is raised there, or by the next read of that file).
    _CACHE_BYTES = int(os.environ.get('H3D_NPY_CACHE_BYTES', 1 << 30))
    # Bytes the queued (not yet landed) writes may hold: a save beyond it
    # waits for the oldest queued writes first, so a whole-genome run's
    # stages do not pile up on the host faster than the disk takes them.
    _PENDING_BYTES = int(os.environ.get('H3D_NPY_PENDING_BYTES', 4 << 30))

    def _cache(self):
        c = self.__dict__.get('_npy_cache')
        if c is None:
            c = self.__dict__['_npy_cache'] = collections.OrderedDict()
            self.__dict__['_npy_cache_bytes'] = 0
        return c

    def _cache_drop(self, fname):
        hit = self._cache().pop(fname, None)
        if hit is not None:
            self.__dict__['_npy_cache_bytes'] -= hit[1].nbytes
            _REAPER.drop(hit, hit[1].nbytes)

    def _cache_put(self, fname, data, stamp):
        self._cache_drop(fname)
        cap = self._CACHE_BYTES
        if data.nbytes > cap:
            _REAPER.drop(data, data.nbytes)
            return
        c = self._cache()
        while c and self.__dict__['_npy_cache_bytes'] + data.nbytes > cap:
            self._cache_drop(next(iter(c)))          # least recently used
        c[fname] = (stamp, data)
        self.__dict__['_npy_cache_bytes'] += data.nbytes

    def cache_nbytes(self):
        """Bytes held by the outdir cache."""
        self._cache()
        return self.__dict__['_npy_cache_bytes']

    @staticmethod
    def _stamp(fname):
        st = os.stat(fname)
        return (st.st_ino, st.st_size, st.st_mtime_ns, st.st_ctime_ns)

    def _pending(self):
        p = self.__dict__.get('_npy_pending')
        if p is None:
            p = self.__dict__['_npy_pending'] = {}
        return p

    def _settle(self, fname):
        """The queued write of ``fname`` if it has landed: its stamp goes to
        the cache entry (the array stays cached as long as the file is the one
        written). Returns the still-queued (future, array), or None."""
        hit = self._pending().get(fname)
        if hit is None:
            return None
        fut, data = hit[0], hit[1]
        if not fut.done():
            return hit
        del self._pending()[fname]
        stamp = fut.result()   # raises the write's error
        self.__dict__.setdefault('_npy_written', {})[fname] = stamp
        self._cache_put(fname, data, stamp)
        return None

    def _settle_landed(self):
        """Moves every landed write from the queue into the size-limited
        cache (and its stamp into the written files)."""
        for fname in [f for f, v in self._pending().items()
                      if v[0].done()]:
            self._settle(fname)

    def pending_nbytes(self):
        """Bytes held by this object's queued (not yet landed) writes."""
        return sum(v[1].nbytes for v in self._pending().values())

    def _bound_pending(self, incoming):
        """Waits for the oldest queued writes (the writer is FIFO) until the
        queue plus ``incoming`` bytes fit _PENDING_BYTES (a single larger
        array is still queued, alone)."""
        self._settle_landed()
        held = self.pending_nbytes()
        for fname in list(self._pending()):
            if held + incoming <= self._PENDING_BYTES:
                break
            fut, data = self._pending()[fname][:2]
            fut.result()
            self._settle(fname)
            held -= data.nbytes

    def flush(self):
        """Waits for every queued outdir write of this object (raises the
        first write error)."""
        pk = self.__dict__.get('_pickle_pending', {})
        for fname in list(pk):
            pk.pop(fname).result()
        for fname in list(self._pending()):
            self._pending()[fname][0].result()
            self._settle(fname)

    def is_current(self, fname):
        """True when ``fname`` holds what this object last wrote there (its
        write queued, or landed and not modified since)."""
        if self._settle(fname) is not None:
            return True
        stamp = self.__dict__.get('_npy_written', {}).get(fname)
        if stamp is None:
            return False
        try:
            return self._stamp(fname) == stamp
        except OSError:
            return False

    def _cached(self, fname):
        q = self._settle(fname)
        if q is not None:
            if q[2] is not None:
                q[2]()       # the queued array's async copy has landed
            return q[1]
        hit = self._cache().get(fname)
        if hit is None:
            return None
        try:
            if self._stamp(fname) == hit[0]:
                self._cache().move_to_end(fname)
                return hit[1]
        except OSError:
            pass
        self._cache_drop(fname)
        return None

    def _read(self, fname, idx, col):
        """One .npy, optionally subset by a row mask and/or one column."""
        a = self._cached(fname)
        if a is not None:
            # copies, as np.load hands out fresh arrays
            if idx is None:
                return a.copy() if col is None else a[:, col].copy()
            return a[idx] if col is None else a[idx, col]
        if idx is None:
            a = np.load(fname)
            return a if col is None else a[:, col]
        a = np.load(fname, mmap_mode='r')
        return np.asarray(a[idx] if col is None else a[idx, col])

    def _save_npy(self, fname, data, owned=False, ready=None):
        """Queues ``data`` for ``fname``. ``owned``: the caller hands the
        array over (a fresh result nobody else holds), so it is queued and
        cached without a copy. ``ready``: a callable that returns once
        ``data`` holds its values (an async device -> host copy into it is
        in flight, analysis/d2h.py); the writer and every reader of the
        queued array call it first."""
        data = np.asanyarray(data)
        gen = self.__dict__.setdefault('_npy_gen', {})
        gen[fname] = gen.get(fname, 0) + 1
        self._cache_drop(fname)
        prev = self._pending().pop(fname, None)
        if type(data) is not np.ndarray:
            if prev is not None:
                prev[0].result()
            np.save(fname, data)
            self.__dict__.setdefault('_npy_written', {})[fname] = \
                self._stamp(fname)
            return
        self._bound_pending(data.nbytes)
        if not owned:
            if ready is not None:
                ready()
                ready = None
            data = data.copy()
        data.setflags(write=False)   # the queued content must not change
        self._pending()[fname] = (_WRITER.submit(fname, data, ready), data,
                                  ready)

    def write_generation(self, fname):
        """How many times this object has written ``fname`` (0: never)."""
        return self.__dict__.get('_npy_gen', {}).get(fname, 0)

    def load_npy_file(self, fname, mmap_mode=None):
        """np.load of an outdir file, after this object's queued write of it
        has landed."""
        hit = self._pending().get(fname)
        if hit is not None:
            hit[0].result()
            self._settle(fname)
        return np.load(fname, mmap_mode=mmap_mode)

    def load_data(self, name, chrom=None, idx=None, rep=None, cond=None,
                  coo=False):
        """Reference ``core.py:62-196``: one chromosome's array (``chrom``),
        an unchromosomed one (``chrom=None``), or every chromosome
        concatenated plus offsets (``chrom='all'``; ``idx`` then spans the
        genome). ``idx`` may be a (big, small) mask pair, chained. ``coo``
        returns (row, col, data) with row/col taken through the stage's mask
        chain.

        Deviation: without loop_patterns the reference's ``loop_idx``
        short-circuit calls the non-existent ``np.load_data``
        (``core.py:105``); here it returns the all-True vector it intends."""
        if name == 'loop_idx' and self.loop_patterns is None and \
                idx is None and chrom != 'all':
            return np.ones(int(self.load_data('disp_idx', chrom).sum()),
                           dtype=bool)
        col = self._column(rep, cond)
        if coo:
            if chrom == 'all' or idx is not None:
                raise ValueError("cannot pass coo=True with chrom='all' or idx")
            if name in self._NOT_COO:
                raise ValueError('data with name %s cannot be loaded as COO'
                                 % name)
            if name not in self._PIXEL_SET:
                raise ValueError('data name %s not recognized' % name)
            chain = [self.load_data(m, chrom) for m in self._PIXEL_SET[name]]
            sel = None
            if chain:
                sel = chain[0]
                for sub in chain[1:]:
                    sel = self._narrow(sel, sub)
            data = self.load_data(name, chrom)
            return (self.load_data('row', chrom, idx=sel),
                    self.load_data('col', chrom, idx=sel),
                    data if col is None else data[:, col])
        if isinstance(idx, tuple):
            idx = self._narrow(*idx)
        if chrom != 'all':
            return self._read(self._npy(name, chrom), idx, col)
        pieces, start = [], 0
        for c in self.chroms:
            fname = self._npy(name, c)
            sub = None
            if idx is not None:
                a = self._cached(fname)
                n = (a if a is not None else np.load(fname, mmap_mode='r')).shape[0]
                sub, start = idx[start:start + n], start + n
            pieces.append(self._read(fname, sub, col))
        offsets = np.concatenate([[0], np.cumsum([len(a) for a in pieces])])
        return np.concatenate(pieces), offsets

    def save_data(self, data, name, chrom=None):
        """Reference ``core.py:198-218``: ``chrom`` is a chromosome name,
        None (unchromosomed), or an offsets array splitting ``data`` over
        ``self.chroms``."""
        if isinstance(chrom, np.ndarray):
            for c, lo, hi in zip(self.chroms, chrom[:-1], chrom[1:]):
                self._save_npy(self._npy(name, c), data[lo:hi])
            return
        self._save_npy(self._npy(name, chrom), data)

    def load_disp_fn(self, cond):
        """Reference ``core.py:220-236`` (after this object's queued write of
        the file has landed)."""
        fname = '%s/disp_fn_%s.pickle' % (self.outdir, cond)
        fut = self.__dict__.get('_pickle_pending', {}).pop(fname, None)
        if fut is not None:
            fut.result()
        with open(fname, 'rb') as h:
            return pickle.load(h)

    def save_disp_fn(self, cond, disp_fn):
        """Reference ``core.py:238-253``: the object is pickled here (its
        state as of this call), the bytes land on the outdir's write-behind
        queue (flush() / load_disp_fn wait for them; ~0.3 ms per file on the
        GPU box's host otherwise paid inline)."""
        fname = '%s/disp_fn_%s.pickle' % (self.outdir, cond)
        blob = pickle.dumps(disp_fn, -1)
        pk = self.__dict__.setdefault('_pickle_pending', {})
        # one lane per file name: a newer write lands after the older one
        pk[fname] = _WRITER.submit(fname, blob, fn=_write_bytes)
