"""ctypes binding of libh3d.so (include/h3d.h).

The product path has no CPU fallback: if the library or a gfx950 device is
missing, every entry point raises ``H3DError``.
"""
import ctypes
import os
import threading

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('H3D_LIB', os.path.join(PKG, 'lib', 'libh3d.so'))

H3D_EST = {'qcml': 0, 'cml': 1, 'mme': 2}
# size-factor methods (util/scaling.py), h3d.h H3D_NORM_*
H3D_NORM = {'conditional_mor': 0, 'conditional_scaling': 1,
            'median_of_ratios': 2, 'simple_scaling': 3, 'no_scaling': 4}

ERRORS = {-1: 'bad argument', -2: 'HIP runtime error',
          -3: 'numerical failure', -4: 'out of device memory',
          -5: 'invalid numeric input', -6: 'no gfx950 device'}

EXPORTS = [
    'h3d_version', 'h3d_device_count', 'h3d_open', 'h3d_close',
    'h3d_last_error', 'h3d_set_stream', 'h3d_union_count', 'h3d_union_fill',
    'h3d_size_factors_cmor', 'h3d_size_factors', 'h3d_disp_per_dist', 'h3d_disp_per_dist_dev',
    'h3d_disp_table', 'h3d_disp_tables', 'h3d_lrt', 'h3d_lrt_dev', 'h3d_bh',
    'h3d_profile_enable', 'h3d_profile_read', 'h3d_profile_reset',
    'h3d_find_clusters', 'h3d_find_clusters_ordered', 'h3d_format_clusters', 'h3d_lrt_poisson',
    'h3d_lrt_poisson_dev', 'h3d_mme_per_pixel', 'h3d_lrt_wide', 'h3d_cml',
    'h3d_bh_ctx', 'h3d_bh_dev', 'h3d_npz_csr_info', 'h3d_npz_csr_read',
    'h3d_disp_tables_dev', 'h3d_disp_tables_wait', 'h3d_lrt_dev_tab',
    'h3d_estimate_disp_dev', 'h3d_bh_sort_dev', 'h3d_bh_scan_dev',
    'h3d_bh_finish_dev', 'h3d_union_fill_dev', 'h3d_size_factors_dev',
    'h3d_disp_pixels_dev', 'h3d_table_gather_dev', 'h3d_disp_seg_stats',
    'h3d_scale_disp_dev', 'h3d_npz_backend', 'h3d_npz_csr_read_slack',
    'h3d_pixel_f_dev', 'h3d_read_text_column', 'h3d_set_qcml_tol',
]


# entry points a library built from an older tree may lack; callers check
OPTIONAL = ('h3d_find_clusters_ordered', 'h3d_npz_backend',
            'h3d_npz_csr_read_slack', 'h3d_read_text_column',
            'h3d_disp_tables', 'h3d_npz_csr_info', 'h3d_npz_csr_read',
            'h3d_disp_tables_dev', 'h3d_disp_tables_wait', 'h3d_lrt_dev_tab',
            'h3d_estimate_disp_dev')


class H3DError(RuntimeError):
    """A libh3d call failed (the reference would have raised too, or the
    native library / GPU is unavailable). ``code``: the library's return
    code (``ERRORS``), None when the failure was not a libh3d return."""

    def __init__(self, msg, code=None):
        RuntimeError.__init__(self, msg)
        self.code = code


H3D_EINPUT = -5


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_D = ctypes.c_double
ALLREDUCE_FN = ctypes.CFUNCTYPE(_I, ctypes.POINTER(_D), _I64, _P)

_lib = None
_lock = threading.RLock()  # context() -> Context() -> load_library()


def load_library(path=None):
    """Loads libh3d.so (once) and declares every prototype of h3d.h."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise H3DError('libh3d.so not found at %s: run '
                           '`python -c "import __graft_entry__ as g; g.build()"`'
                           % p)
        # One HIP runtime per process: torch (when installed) ships its own
        # libamdhip64.so.7 under the same SONAME as the /opt/rocm one libh3d
        # links, and whichever loads first serves both. Loading torch's first
        # keeps torch.cuda working next to libh3d (the other order leaves
        # torch without devices) and lets torch tensors / streams be handed
        # to the *_dev entry points.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(p)
        sig = {
            'h3d_version': (_I, []),
            'h3d_device_count': (_I, []),
            'h3d_open': (_P, [_I]),
            'h3d_close': (None, [_P]),
            'h3d_last_error': (ctypes.c_char_p, []),
            'h3d_set_stream': (_I, [_P, _P]),
            'h3d_set_qcml_tol': (_I, [_P, _D]),
            'h3d_union_count': (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _I, _P]),
            'h3d_union_fill': (_I, [_P, _P, _P, _P, _P, _I64]),
            'h3d_union_fill_dev': (_I, [_P, _P, _P, _P, _P, _I64, _P, _P, _P,
                                        _P]),
            'h3d_size_factors_dev': (_I, [_P, _P, _P, _I64, _I, _I, _I, _P,
                                          _P]),
            'h3d_disp_pixels_dev': (_I, [_P, _P, _P, _P, _P, _I, _P, _I, _P,
                                         _I64, _I, _I64, _P, _P, _P]),
            'h3d_table_gather_dev': (_I, [_P, _P, _I, _I, _P, _I64, _P]),
            'h3d_pixel_f_dev': (_I, [_P, _P, _P, _P, _P, _I64, _I, _P, _P, _P,
                                     _P, _I, _P]),
            'h3d_scale_disp_dev': (_I, [_P, _P, _P, _I, _P, _P, _I64, _I, _I,
                                        _P, ctypes.c_double, _I, _P, _P, _P,
                                        _P]),
            'h3d_disp_seg_stats': (_I, [_P, _I, _P, _P]),
            'h3d_size_factors_cmor': (_I, [_P, _P, _P, _I64, _I, _I, _P]),
            'h3d_size_factors': (_I, [_P, _P, _P, _I64, _I, _I, _I, _P]),
            'h3d_disp_per_dist': (_I, [_P, _P, _P, _P, _I64, _I, _I, _P, _I,
                                       _I, _P, _P]),
            'h3d_disp_per_dist_dev': (_I, [_P, _P, _P, _P, _I64, _I, _I, _P,
                                           _I, _I, _P, _P, ALLREDUCE_FN, _P]),
            'h3d_disp_table': (_I, [_P, _I, _I, _D, _D, _P]),
            'h3d_disp_tables': (_I, [_P, _I, _I, _I, _D, _D, _P]),
            'h3d_lrt': (_I, [_P, _P, _P, _P, _P, _I64, _I, _I, _P, _I, _I, _P,
                             _P, _P, _P, _P]),
            'h3d_lrt_dev': (_I, [_P, _P, _P, _P, _P, _I64, _I, _I, _P, _I, _I,
                                 _P, _P, _P, _P, _P]),
            'h3d_bh': (_I, [_P, _I64, _P]),
            'h3d_bh_ctx': (_I, [_P, _P, _I64, _P]),
            'h3d_bh_dev': (_I, [_P, _P, _I64, _P]),
            'h3d_bh_sort_dev': (_I, [_P, _P, _P, _I64, _P, _P, _P]),
            'h3d_bh_scan_dev': (_I, [_P, _P, _I64, _I64, _I64, _P, _P]),
            'h3d_bh_finish_dev': (_I, [_P, _P, _I64, _D, _P]),
            'h3d_profile_enable': (_I, [_P, _I]),
            'h3d_profile_read': (_I, [_P, ctypes.c_char_p, _P, _P, _P]),
            'h3d_profile_reset': (_I, [_P]),
            'h3d_find_clusters': (_I, [_P, _P, _I64, _I, _P, _P]),
            'h3d_find_clusters_ordered': (_I, [_P, _P, _I64, _I, _P, _P, _P]),
            'h3d_format_clusters': (_I, [_P, _P, _P, _P, _I64, _P, _I64, _P,
                                         _P]),
            'h3d_lrt_poisson': (_I, [_P, _P, _P, _I64, _I, _I, _P, _P, _P,
                                     _P, _P]),
            'h3d_lrt_poisson_dev': (_I, [_P, _P, _P, _I64, _I, _I, _P, _P,
                                         _P, _P, _P]),
            'h3d_mme_per_pixel': (_I, [_P, _P, _P, _I64, _I, _I, _P, _D,
                                       _P]),
            'h3d_lrt_wide': (_I, [_P, _P, _P, _P, _I64, _I, _I, _P, _I, _P,
                                  _P, _P, _P]),
            'h3d_cml': (_I, [_P, _P, _I64, _I, _P]),
            'h3d_disp_tables_dev': (_I, [_P, _P, _I, _I, _I, _D, _D, _P]),
            'h3d_disp_tables_wait': (_I, [_P]),
            'h3d_estimate_disp_dev': (_I, [_P, _P, _P, _P, _I64, _I, _I, _P, _I,
                                           _I, _D, _D, _P, _P, _P]),
            'h3d_lrt_dev_tab': (_I, [_P, _P, _P, _P, _P, _I64, _I, _I, _P, _I,
                                     _I, _P, _P, _P, _P, _P]),
            'h3d_npz_csr_info': (_I, [ctypes.c_char_p, _P, _P, _P]),
            'h3d_npz_backend': (_I, []),
            'h3d_read_text_column': (_I, [ctypes.c_char_p, _P, _I64, _P]),
            'h3d_npz_csr_read_slack': (_I, [ctypes.c_char_p, _I64, _I64, _P,
                                            _P, _P, _I64, _P]),
            'h3d_npz_csr_read': (_I, [ctypes.c_char_p, _I64, _I64, _P, _P, _P,
                                      _P]),
        }
        for name, (res, args) in sig.items():
            if name in OPTIONAL and not hasattr(lib, name):
                continue   # an older libh3d (A/B runs against past builds)
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib


def _check(rc, what):
    if rc != 0:
        msg = load_library().h3d_last_error().decode(errors='replace')
        raise H3DError('%s: %s (%d: %s)' % (what, msg, rc,
                                            ERRORS.get(rc, '?')), code=rc)


def _wmode(weighted):
    """The smoother's ``weighted`` argument at the ABI: 0 plain lowess, 1
    weighted lowess with the smallest scaled weight pinned to 1 (the
    product's default), 2 (``weighted='reference'``) weighted
    lowess with the reference's own ``w * (1 / w)`` scaling, which floors a
    minimum weight that rounds to 1 - 2^-53 to zero copies
    (lowess.py:183-201)."""
    if isinstance(weighted, str):
        if weighted != 'reference':
            raise ValueError('weighted must be a bool or "reference"')
        return 2
    return int(bool(weighted))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


class CSR(object):
    """The three arrays of a CSR matrix as the union kernels take them
    (indptr int64, indices int32, data float64; the attribute names of
    scipy.sparse.csr_matrix)."""

    def __init__(self, indptr, indices, data, shape):
        self.indptr, self.indices, self.data = indptr, indices, data
        self.shape = shape


def read_text_column(path):
    """A one-column text file (a replicate's bias vector) as np.loadtxt
    reads it, parsed by libh3d (h3d_read_text_column) without holding the
    GIL -- prepare_data's reader thread parses the next chromosome's bias
    files while the main thread drives the device, and np.loadtxt held the
    GIL for all of it. None when libh3d does not take the file (anything but
    one decimal number per line, or an older library): the caller reads it
    with np.loadtxt."""
    try:
        lib = load_library()
        size = os.path.getsize(path)
    except (H3DError, OSError):
        return None
    if not hasattr(lib, 'h3d_read_text_column'):
        return None
    cap = size // 2 + 1          # a value takes at least a digit and a newline
    out = np.empty(cap)
    n = ctypes.c_int64(0)
    if lib.h3d_read_text_column(os.fsencode(path), _ptr(out), cap,
                                ctypes.byref(n)) != 0:
        return None
    return out[:n.value]


_NPZ_SLACK = 4096


def load_npz_csr(path, alloc=None):
    """A scipy.sparse.save_npz CSR archive read by libh3d's reader
    (h3d_npz_csr_info / _read; the reference loads it with
    scipy.sparse.load_npz, analysis.py:94,100). Rows whose columns are not
    strictly increasing are canonicalised as scipy's sum_duplicates does.
    Raises H3DError for archives the reader does not take (other sparse
    formats, unsupported dtypes); the caller decides whether to use scipy.
    ``alloc(nbytes)``: the uint8 buffers indices and data are inflated into
    (default numpy; prepare_data passes pinned host memory, so the union's
    uploads of them run at DMA speed)."""
    lib = load_library()
    if not hasattr(lib, 'h3d_npz_csr_read'):
        raise H3DError('libh3d.so predates h3d_npz_csr_read')
    bp = os.fsencode(path)
    n_rows, n_cols, nnz = _I64(0), _I64(0), _I64(0)
    _check(lib.h3d_npz_csr_info(bp, ctypes.byref(n_rows), ctypes.byref(n_cols),
                                ctypes.byref(nnz)), 'h3d_npz_csr_info')
    indptr = np.empty(n_rows.value + 1, dtype=np.int64)
    canon = _I(0)
    # (not for nnz 0: numpy places an empty slice at its base's start)
    if hasattr(lib, 'h3d_npz_csr_read_slack') and nnz.value > 0:
        # _NPZ_SLACK bytes ahead of indices / data: the members are inflated
        # in place, their .npy headers landing in the slack
        mk = alloc or (lambda k: np.empty(k, dtype=np.uint8))
        ib = mk(_NPZ_SLACK + 4 * nnz.value)
        db = mk(_NPZ_SLACK + 8 * nnz.value)
        indices = ib[_NPZ_SLACK:].view(np.int32)
        data = db[_NPZ_SLACK:].view(np.float64)
        _check(lib.h3d_npz_csr_read_slack(
            bp, n_rows.value, nnz.value, _ptr(indptr), _ptr(indices),
            _ptr(data), _NPZ_SLACK, ctypes.byref(canon)),
            'h3d_npz_csr_read_slack')
    else:
        indices = np.empty(nnz.value, dtype=np.int32)
        data = np.empty(nnz.value, dtype=np.float64)
        _check(lib.h3d_npz_csr_read(bp, n_rows.value, nnz.value,
                                    _ptr(indptr), _ptr(indices), _ptr(data),
                                    ctypes.byref(canon)), 'h3d_npz_csr_read')
    shape = (n_rows.value, n_cols.value)
    if canon.value:
        return CSR(indptr, indices, data, shape)
    import scipy.sparse as sparse
    m = sparse.csr_matrix((data, indices, indptr), shape=shape)
    m.sum_duplicates()
    return CSR(_c(m.indptr, np.int64), _c(m.indices, np.int32),
               _c(m.data, np.float64), shape)


class Context(object):
    """One libh3d context bound to one GPU (``h3d_open``)."""

    def __init__(self, device=0):
        self.lib = load_library()
        self.device = device
        h = self.lib.h3d_open(device)
        if not h:
            raise H3DError('h3d_open(%d): %s' % (
                device, self.lib.h3d_last_error().decode(errors='replace')))
        self.handle = h

    def close(self):
        if self.handle:
            self.lib.h3d_close(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle):
        _check(self.lib.h3d_set_stream(self.handle, stream_handle),
               'h3d_set_stream')

    def set_qcml_tol(self, tol):
        """qcml's convergence tolerance for this ctx's later estimate_disp
        calls (h3d_set_qcml_tol; dispersion.py:10's tol, default 1e-4)."""
        _check(self.lib.h3d_set_qcml_tol(self.handle, float(tol)),
               'h3d_set_qcml_tol')

    # -- prepare_data -------------------------------------------------------
    def sparse_union(self, csrs, bias, dist_max, device_alloc=None,
                     host_balanced=True, host_raw=True):
        """csrs: list of canonical CSR matrices (scipy or `CSR`, n_bins x
        n_bins); bias
        (n_bins, R) filtered. Returns row, col (int32), raw (int64 (n, R)),
        balanced (float64 (n, R)). ``device_alloc(n, R)``, when given,
        returns device pointers (row, col, raw int32, balanced; any may be
        None) that also receive the union (h3d_union_fill_dev); with a device
        balanced, ``host_balanced=False`` skips its host copy (balanced is
        then None)."""
        R = len(csrs)
        n_bins = bias.shape[0]
        keep = []
        ip = (ctypes.c_void_p * R)()
        ix = (ctypes.c_void_p * R)()
        dt = (ctypes.c_void_p * R)()
        nnz = np.zeros(R, dtype=np.int64)
        for r, m in enumerate(csrs):
            a = _c(m.indptr, np.int64)
            b = _c(m.indices, np.int32)
            c = _c(m.data, np.float64)
            keep += [a, b, c]
            ip[r], ix[r], dt[r] = a.ctypes.data, b.ctypes.data, c.ctypes.data
            nnz[r] = len(c)
        bias = _c(bias, np.float64)
        n_px = ctypes.c_int64(0)
        _check(self.lib.h3d_union_count(
            self.handle, R, n_bins, ip, ix, dt, _ptr(nnz), _ptr(bias),
            int(dist_max), ctypes.byref(n_px)), 'h3d_union_count')
        n = n_px.value
        row = np.empty(n, dtype=np.int32)
        col = np.empty(n, dtype=np.int32)
        # host_raw=False with a device raw copy: raw is None (fetched from
        # the device copy in the background by the caller)
        raw = np.empty((n, R), dtype=np.int64) \
            if host_raw or device_alloc is None else None
        bal = np.empty((n, R), dtype=np.float64) \
            if host_balanced or device_alloc is None else None
        if device_alloc is None:
            _check(self.lib.h3d_union_fill(self.handle, _ptr(row), _ptr(col),
                                           _ptr(raw), _ptr(bal), n),
                   'h3d_union_fill')
        else:
            d = device_alloc(n, R)
            if bal is None and n and not d[3]:
                raise ValueError('host_balanced=False needs a device balanced')
            if raw is None and n and not d[2]:
                raise ValueError('host_raw=False needs a device raw')
            _check(self.lib.h3d_union_fill_dev(
                self.handle, _ptr(row), _ptr(col), _ptr(raw),
                _ptr(bal) if bal is not None else None, n,
                *[_P(v) if v else None for v in d]), 'h3d_union_fill_dev')
        return row, col, raw, bal

    def size_factors_dev(self, d_balanced, dist, n, R, norm='conditional_mor',
                         n_bins=0, d_sf_out=None, host_out=True):
        """size_factors on a device balanced (n, R); the result on the host
        and, with ``d_sf_out``, in that device buffer ((n, R) or (R,))."""
        if norm not in H3D_NORM:
            raise ValueError('unknown norm %r' % (norm,))
        cond = norm.startswith('conditional')
        dist = _c(dist, np.int32) if cond else None
        # host_out=False (conditional norms with a device copy): no host
        # copy, None is returned (the caller fetches the device one)
        out = np.empty((n, R) if cond else R, dtype=np.float64) \
            if (host_out or not cond or not d_sf_out) else None
        _check(self.lib.h3d_size_factors_dev(
            self.handle, _P(d_balanced), _ptr(dist), n, R, H3D_NORM[norm],
            int(n_bins or 0), _ptr(out), _P(d_sf_out) if d_sf_out else None),
            'h3d_size_factors_dev')
        return out

    def scale_disp_dev(self, d_balanced, d_sf, sf_per_rep, d_row, d_col, n,
                       R, design, mean_thresh, dist_thresh_min,
                       d_flag_out=None, d_scaled_out=None):
        """prepare_data's scaled (n, R) and disp_idx flags (n; 0 / 1, or 2
        where numpy's product decides) on the device (h3d_scale_disp_dev);
        returns the host copies (scaled, flag) -- scaled None when it goes to
        the device buffer ``d_scaled_out`` instead."""
        design = np.ascontiguousarray(design, dtype=np.uint8)
        if design.ndim != 2 or design.shape[0] != R:
            raise ValueError('design must be (R, C)')
        scaled = np.empty((n, R), dtype=np.float64) if not d_scaled_out \
            else None
        flag = np.empty(n, dtype=np.uint8)
        _check(self.lib.h3d_scale_disp_dev(
            self.handle, _P(d_balanced), _P(d_sf), int(bool(sf_per_rep)),
            _P(d_row), _P(d_col), n, R, design.shape[1], _ptr(design),
            float(mean_thresh), int(dist_thresh_min), _ptr(scaled),
            _ptr(flag), _P(d_flag_out) if d_flag_out else None,
            _P(d_scaled_out) if d_scaled_out else None),
            'h3d_scale_disp_dev')
        return scaled, flag

    def disp_pixels_dev(self, d_row, d_col, d_raw, d_sf, sf_per_rep, bias,
                        d_disp_idx, n, R, n_disp, d_raw_out, d_f_out,
                        d_dist_out):
        """A chromosome's disp pixels on the device (h3d_disp_pixels_dev):
        raw (n_disp, R) int32, f = bias[row] * bias[col] * sf, dist."""
        bias = _c(bias, np.float64)
        _check(self.lib.h3d_disp_pixels_dev(
            self.handle, _P(d_row), _P(d_col), _P(d_raw), _P(d_sf),
            int(bool(sf_per_rep)), _ptr(bias), bias.shape[0], _P(d_disp_idx),
            n, R, n_disp, _P(d_raw_out) if d_raw_out else None,
            _P(d_f_out) if d_f_out else None,
            _P(d_dist_out) if d_dist_out else None), 'h3d_disp_pixels_dev')

    def pixel_f_dev(self, d_row, d_dist, d_chrom, d_sfi, n, R, d_bias, d_boff,
                    d_sf, d_soff, nchrom, d_f_out):
        """f of re-sharded pixels from their keys (h3d_pixel_f_dev): device
        pointers in and out, synchronous."""
        _check(self.lib.h3d_pixel_f_dev(
            self.handle, _P(d_row), _P(d_dist), _P(d_chrom), _P(d_sfi), n, R,
            _P(d_bias), _P(d_boff), _P(d_sf), _P(d_soff), nchrom,
            _P(d_f_out)), 'h3d_pixel_f_dev')

    def disp_seg_stats(self, D, C):
        """(qcml iterations, Brent NLL evaluations) per segment (D, C) of
        the last estimate_disp call on this ctx."""
        qi = np.zeros((D, C), dtype=np.int32)
        ev = np.zeros((D, C), dtype=np.int32)
        _check(self.lib.h3d_disp_seg_stats(self.handle, D * C, _ptr(qi),
                                           _ptr(ev)), 'h3d_disp_seg_stats')
        return qi, ev

    def table_gather_dev(self, d_tables, D, C, d_dist, n, d_out):
        """disp = tables[dist] on the device (h3d_table_gather_dev)."""
        _check(self.lib.h3d_table_gather_dev(self.handle, _P(d_tables), D, C,
                                             _P(d_dist), n, _P(d_out)),
               'h3d_table_gather_dev')

    def size_factors_cmor(self, balanced, dist, n_bins):
        balanced = _c(balanced, np.float64)
        dist = _c(dist, np.int32)
        n, R = balanced.shape
        out = np.empty((n, R), dtype=np.float64)
        _check(self.lib.h3d_size_factors_cmor(
            self.handle, _ptr(balanced), _ptr(dist), n, R,
            int(n_bins or 0), _ptr(out)), 'h3d_size_factors_cmor')
        return out

    def size_factors(self, balanced, dist, norm='conditional_mor', n_bins=0):
        """Any norm of util/scaling.py: the conditional ones give (n, R)
        (``n_bins`` equal-number distance bins, 0/None = exact distances),
        the others (R,)."""
        if norm not in H3D_NORM:
            raise ValueError('unknown norm %r' % (norm,))
        balanced = _c(balanced, np.float64)
        n, R = balanced.shape
        cond = norm.startswith('conditional')
        dist = _c(dist, np.int32) if cond else None
        out = np.empty((n, R) if cond else R, dtype=np.float64)
        _check(self.lib.h3d_size_factors(
            self.handle, _ptr(balanced), _ptr(dist), n, R, H3D_NORM[norm],
            int(n_bins or 0), _ptr(out)), 'h3d_size_factors')
        return out

    # -- estimate_disp ------------------------------------------------------
    def disp_per_dist(self, raw, f, dist, cond_of_rep, C, D,
                      estimator='qcml'):
        raw = _c(raw, np.int64)
        f = _c(f, np.float64)
        dist = _c(dist, np.int32)
        cond = _c(cond_of_rep, np.int32)
        n, R = raw.shape
        out = np.empty((D, C), dtype=np.float64)
        flags = np.zeros((D, C), dtype=np.int32)
        _check(self.lib.h3d_disp_per_dist(
            self.handle, _ptr(raw), _ptr(f), _ptr(dist), n, R, C, _ptr(cond),
            D, H3D_EST[estimator], _ptr(out), _ptr(flags)),
            'h3d_disp_per_dist')
        return out

    def disp_per_dist_dev(self, d_raw, d_f, d_dist, n, R, cond_of_rep, C, D,
                          reduce=None):
        """Device-pointer variant; ``reduce(ptr, count)`` all-reduces a device
        buffer of doubles in place (multi-GPU)."""
        cond = _c(cond_of_rep, np.int32)
        out = np.empty((D, C), dtype=np.float64)
        flags = np.zeros((D, C), dtype=np.int32)
        if reduce is not None:
            def _cb(ptr, count, user):
                try:
                    reduce(ctypes.cast(ptr, ctypes.c_void_p).value, count)
                    return 0
                except Exception:  # surfaced as H3D_EHIP by the library
                    return 1
            cb = ALLREDUCE_FN(_cb)
        else:
            cb = ALLREDUCE_FN()
        _check(self.lib.h3d_disp_per_dist_dev(
            self.handle, d_raw, d_f, d_dist, n, R, C, _ptr(cond), D, 0,
            _ptr(out), _ptr(flags), cb, None), 'h3d_disp_per_dist_dev')
        return out

    # -- lrt -----------------------------------------------------------------
    def lrt(self, raw, f, dist, disp_table, cond_of_rep, refit_mu=True,
            want_disp=True):
        """``dist=None``: ``disp_table`` is the per-pixel dispersion (n, C)."""
        raw = _c(raw, np.int64)
        f = _c(f, np.float64)
        dist = _c(dist, np.int32) if dist is not None else None
        tab = _c(disp_table, np.float64)
        cond = _c(cond_of_rep, np.int32)
        n, R = raw.shape
        D, C = tab.shape
        if dist is None:
            if D != n:
                raise ValueError('per-pixel disp must be (n, C)')
            D = 0
        p = np.empty(n)
        llr = np.empty(n)
        mu0 = np.empty(n)
        mu1 = np.empty((n, C))
        disp = np.empty((n, C)) if want_disp else None
        _check(self.lib.h3d_lrt(
            self.handle, _ptr(raw), _ptr(f), _ptr(dist), _ptr(tab), n, R, C,
            _ptr(cond), D, int(bool(refit_mu)), _ptr(p), _ptr(llr), _ptr(mu0),
            _ptr(mu1), _ptr(disp)), 'h3d_lrt')
        return p, llr, mu0, mu1, disp

    def lrt_wide(self, raw, f, disp_wide, cond_of_rep, C, refit_mu=True):
        """lrt.py's own call: per pixel and replicate dispersions (n, R)."""
        raw = _c(raw, np.int64)
        f = _c(f, np.float64)
        dw = _c(disp_wide, np.float64)
        cond = _c(cond_of_rep, np.int32)
        n, R = raw.shape
        if f.shape != (n, R) or dw.shape != (n, R):
            raise ValueError('raw, f and disp must all be (n, R)')
        p, llr, mu0 = np.empty(n), np.empty(n), np.empty(n)
        mu1 = np.empty((n, C))
        _check(self.lib.h3d_lrt_wide(
            self.handle, _ptr(raw), _ptr(f), _ptr(dw), n, R, C, _ptr(cond),
            int(bool(refit_mu)), _ptr(p), _ptr(llr), _ptr(mu0), _ptr(mu1)),
            'h3d_lrt_wide')
        return p, llr, mu0, mu1

    def cml(self, data):
        """cml on (n, r) data already divided by f."""
        data = _c(data, np.float64)
        n, r = data.shape
        out = ctypes.c_double(0)
        _check(self.lib.h3d_cml(self.handle, _ptr(data), n, r,
                                ctypes.byref(out)), 'h3d_cml')
        return out.value

    def bh(self, pvalues):
        """BH q-values on this ctx's GPU (h3d_bh_ctx; same bits as bh())."""
        p = _c(pvalues, np.float64)
        q = np.empty_like(p)
        _check(self.lib.h3d_bh_ctx(self.handle, _ptr(p), len(p), _ptr(q)),
               'h3d_bh_ctx')
        return q

    def bh_dev(self, d_p, n, d_q):
        _check(self.lib.h3d_bh_dev(self.handle, _P(d_p), n, _P(d_q)),
               'h3d_bh_dev')

    # pieces of the rank-sharded BH (parallel.bh_sharded, h3d.h)
    def bh_sort_dev(self, d_p, d_val, n, d_key_out, d_val_out):
        m = ctypes.c_int64(0)
        _check(self.lib.h3d_bh_sort_dev(self.handle, _P(d_p), _P(d_val), n,
                                        _P(d_key_out), _P(d_val_out),
                                        ctypes.byref(m)), 'h3d_bh_sort_dev')
        return m.value

    def bh_scan_dev(self, d_ps, mb, offset, m, d_scanned):
        lo = ctypes.c_double(0)
        _check(self.lib.h3d_bh_scan_dev(self.handle, _P(d_ps), mb, offset, m,
                                        _P(d_scanned), ctypes.byref(lo)),
               'h3d_bh_scan_dev')
        return lo.value

    def bh_finish_dev(self, d_scanned, mb, higher_min, d_q):
        _check(self.lib.h3d_bh_finish_dev(self.handle, _P(d_scanned), mb,
                                          float(higher_min), _P(d_q)),
               'h3d_bh_finish_dev')

    def lrt_dev(self, d_raw, d_f, d_dist, disp_table, n, R, cond_of_rep,
                d_p, d_llr, d_mu0, d_mu1, d_disp=None, refit_mu=True):
        tab = _c(disp_table, np.float64)
        cond = _c(cond_of_rep, np.int32)
        D, C = tab.shape
        _check(self.lib.h3d_lrt_dev(
            self.handle, d_raw, d_f, d_dist, _ptr(tab), n, R, C, _ptr(cond),
            D, int(bool(refit_mu)), d_p, d_llr, d_mu0, d_mu1, d_disp),
            'h3d_lrt_dev')

    def disp_tables_dev(self, d_dpd, D, C, d_tables, weighted=True,
                        frac=None, auto_frac_factor=15.):
        """disp_tables on the GPU: device (D, C) float64 in and out, enqueued
        without waiting (settled by lrt_dev_tab or disp_tables_wait)."""
        _check(self.lib.h3d_disp_tables_dev(
            self.handle, d_dpd, D, C, _wmode(weighted),
            -1.0 if frac is None else float(frac), float(auto_frac_factor),
            d_tables), 'h3d_disp_tables_dev')

    def estimate_disp_dev(self, d_raw, d_f, d_dist, n, R, cond_of_rep, C, D,
                          d_tables, weighted=True, frac=None,
                          auto_frac_factor=15.):
        """disp_per_dist_dev whose smoothed (D, C) tables are computed on
        the device into ``d_tables`` (settled by lrt_dev_tab /
        disp_tables_wait); returns disp_per_dist on the host."""
        cond = _c(cond_of_rep, np.int32)
        out = np.empty((D, C), dtype=np.float64)
        flags = np.zeros((D, C), dtype=np.int32)
        _check(self.lib.h3d_estimate_disp_dev(
            self.handle, d_raw, d_f, d_dist, n, R, C, _ptr(cond), D,
            _wmode(weighted), -1.0 if frac is None else float(frac),
            float(auto_frac_factor), _ptr(out), _ptr(flags), d_tables),
            'h3d_estimate_disp_dev')
        return out

    def disp_tables_wait(self):
        _check(self.lib.h3d_disp_tables_wait(self.handle),
               'h3d_disp_tables_wait')

    def lrt_dev_tab(self, d_raw, d_f, d_dist, d_table, D, n, R, cond_of_rep,
                    d_p, d_llr, d_mu0, d_mu1, d_disp=None, refit_mu=True):
        """lrt_dev with the (D, C) table in device memory."""
        cond = _c(cond_of_rep, np.int32)
        C = int(cond.max()) + 1
        _check(self.lib.h3d_lrt_dev_tab(
            self.handle, d_raw, d_f, d_dist, d_table, n, R, C, _ptr(cond),
            D, int(bool(refit_mu)), d_p, d_llr, d_mu0, d_mu1, d_disp),
            'h3d_lrt_dev_tab')

    # -- alternative models (analysis/alternatives.py) -----------------------
    def lrt_poisson(self, raw, f, cond_of_rep, C):
        """Poisson LRT (alternatives.py:25-42, refit_mu=True): p, llr,
        mu_hat_null (n,), mu_hat_alt (n, C)."""
        raw = _c(raw, np.int64)
        f = _c(f, np.float64)
        cond = _c(cond_of_rep, np.int32)
        n, R = raw.shape
        p = np.empty(n)
        llr = np.empty(n)
        mu0 = np.empty(n)
        mu1 = np.empty((n, C))
        _check(self.lib.h3d_lrt_poisson(
            self.handle, _ptr(raw), _ptr(f), n, R, C, _ptr(cond), _ptr(p),
            _ptr(llr), _ptr(mu0), _ptr(mu1)), 'h3d_lrt_poisson')
        return p, llr, mu0, mu1

    def lrt_poisson_dev(self, d_raw, d_f, n, R, cond_of_rep, C, d_p, d_llr,
                        d_mu0, d_mu1):
        cond = _c(cond_of_rep, np.int32)
        _check(self.lib.h3d_lrt_poisson_dev(
            self.handle, d_raw, d_f, n, R, C, _ptr(cond), d_p, d_llr, d_mu0,
            d_mu1), 'h3d_lrt_poisson_dev')

    def mme_per_pixel(self, data, f, cond_of_rep, C, min_disp=-np.inf):
        """Per-pixel MME dispersion of each condition (dispersion.py:83-104)
        floored at ``min_disp`` (NaN stays NaN): (n, C)."""
        data = _c(data, np.float64)
        f = _c(f, np.float64) if f is not None else None
        cond = _c(cond_of_rep, np.int32)
        n, R = data.shape
        out = np.empty((n, C))
        _check(self.lib.h3d_mme_per_pixel(
            self.handle, _ptr(data), _ptr(f), n, R, C, _ptr(cond),
            float(min_disp), _ptr(out)), 'h3d_mme_per_pixel')
        return out

    # -- measurement ---------------------------------------------------------
    def profile(self, on=True, level=2):
        """HIP-event timing on the ctx stream: level 1 = the roofline
        kernels only (disp_work, lrt), 2 = every kernel scope."""
        _check(self.lib.h3d_profile_enable(self.handle,
                                           int(level) if on else 0),
               'h3d_profile_enable')

    def profile_reset(self):
        _check(self.lib.h3d_profile_reset(self.handle), 'h3d_profile_reset')

    def profile_read(self, name):
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        u = ctypes.c_int64(0)
        _check(self.lib.h3d_profile_read(self.handle, name.encode(),
                                         ctypes.byref(ms), ctypes.byref(n),
                                         ctypes.byref(u)), 'h3d_profile_read')
        return ms.value, n.value, u.value


def disp_table(disp_per_dist_col, weighted=True, frac=None,
               auto_frac_factor=15.):
    """Host-side smoother (libh3d, C++): the fitted dispersion function
    tabulated at every integer distance."""
    lib = load_library()
    col = _c(disp_per_dist_col, np.float64)
    out = np.empty(len(col))
    _check(lib.h3d_disp_table(_ptr(col), len(col), _wmode(weighted),
                              -1.0 if frac is None else float(frac),
                              float(auto_frac_factor), _ptr(out)),
           'h3d_disp_table')
    return out


def disp_tables(disp_per_dist, weighted=True, frac=None, auto_frac_factor=15.):
    """disp_table for every column of ``disp_per_dist`` (D, C), the
    conditions smoothed on concurrent threads inside libh3d (one call)."""
    lib = load_library()
    d = _c(disp_per_dist, np.float64)
    D, C = d.shape
    if not hasattr(lib, 'h3d_disp_tables'):
        return np.stack([disp_table(d[:, c], weighted, frac, auto_frac_factor)
                         for c in range(C)], axis=1)
    out = np.empty((D, C))
    _check(lib.h3d_disp_tables(_ptr(d), D, C, _wmode(weighted),
                               -1.0 if frac is None else float(frac),
                               float(auto_frac_factor), _ptr(out)),
           'h3d_disp_tables')
    return out


def bh(pvalues):
    lib = load_library()
    p = _c(pvalues, np.float64)
    q = np.empty_like(p)
    _check(lib.h3d_bh(_ptr(p), len(p), _ptr(q)), 'h3d_bh')
    return q


def cluster_labels(row, col, connectivity=1):
    """Cluster index of every pixel, clusters numbered in the reference's
    get_groups() order (libh3d host code, clusters.py:73-97)."""
    lib = load_library()
    r = _c(row, np.int64)
    c = _c(col, np.int64)
    lab = np.empty(len(r), dtype=np.int64)
    nc = ctypes.c_int64(0)
    _check(lib.h3d_find_clusters(_ptr(r), _ptr(c), len(r), int(connectivity),
                                 _ptr(lab), ctypes.byref(nc)),
           'h3d_find_clusters')
    return lab, nc.value


def cluster_order(row, col, connectivity=1):
    """(labels, n_clusters, order): cluster_labels plus the pixel indices
    cluster by cluster, each cluster in the iteration order of the
    reference's Python set (h3d_find_clusters_ordered). Pixels distinct."""
    lib = load_library()
    r = _c(row, np.int64)
    c = _c(col, np.int64)
    lab = np.empty(len(r), dtype=np.int64)
    order = np.empty(len(r), dtype=np.int64)
    nc = ctypes.c_int64(0)
    _check(lib.h3d_find_clusters_ordered(
        _ptr(r), _ptr(c), len(r), int(connectivity), _ptr(lab),
        ctypes.byref(nc), _ptr(order)), 'h3d_find_clusters_ordered')
    return lab, nc.value, order


def format_clusters(row, col, members, starts):
    """Text "[[i, j], ...]" of each cluster -> (bytes, end offsets)."""
    lib = load_library()
    r = _c(row, np.int64)
    c = _c(col, np.int64)
    m = _c(members, np.int64)
    s = _c(starts, np.int64)
    k = len(s) - 1
    ln = ctypes.c_int64(0)
    _check(lib.h3d_format_clusters(_ptr(r), _ptr(c), _ptr(m), _ptr(s), k,
                                   None, 0, None, ctypes.byref(ln)),
           'h3d_format_clusters')
    buf = ctypes.create_string_buffer(max(ln.value, 1))
    ends = np.empty(k, dtype=np.int64)
    _check(lib.h3d_format_clusters(_ptr(r), _ptr(c), _ptr(m), _ptr(s), k,
                                   buf, ln.value, _ptr(ends),
                                   ctypes.byref(ln)), 'h3d_format_clusters')
    return buf.raw[:ln.value], ends


_ctx = {}


def context(device=None):
    """Process-wide context for ``device`` (default: LOCAL_RANK or 0)."""
    if device is None:
        device = int(os.environ.get('LOCAL_RANK', '0'))
    with _lock:
        if device not in _ctx:
            _ctx[device] = Context(device)
        return _ctx[device]
