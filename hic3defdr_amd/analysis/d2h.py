"""Device -> host copies of the stage results the outdir contract needs
(reference analysis.py:222-223, :281-284 write them from host arrays), off
the pipeline's critical path.

``to_host_async(t)`` returns ``(array, ready)`` at once: a fresh host array of
``t``'s shape and dtype, and a callable that returns once ``t``'s values have
landed in it. The copy runs on one background thread ("h3d-d2h", copies in
submission order) on a dedicated non-default stream, so the pipeline's next
stage launches its kernels while the previous stage's results stream out;
the stage hands (array, ready) to the write-behind queue
(``core._save_npy(..., ready=ready)``), whose writer -- and any reader of the
queued array -- calls ``ready()`` first. The copy goes into ordinary pageable
memory: pinning the ~210 MB a cfg2 run moves (disp, p, llr, mu) cost as much
as the copy itself (~18 ms per run, measured r05g), and the thread takes the
copy off the critical path either way. The device tensor is held by the
pending copy, so its memory is not reused before the copy has read it.
"""
import concurrent.futures
import threading

import numpy as np

_lock = threading.Lock()
_state = {}


def _pool():
    with _lock:
        ex = _state.get('ex')
        if ex is None:
            ex = _state['ex'] = concurrent.futures.ThreadPoolExecutor(
                1, thread_name_prefix='h3d-d2h')
        return ex


def _nonblocking_stream(dev):
    """A stream created hipStreamNonBlocking, wrapped for torch: work on
    it is not ordered against the legacy default stream, so a
    synchronise of torch's default stream (the class's stages) does not
    wait for these copies (measured: 25-29 ms of estimate_disp's
    synchronise through the class with a plain torch.cuda.Stream, r06ao).
    None when the runtime does not take the call."""
    import ctypes
    import torch
    try:
        hip = ctypes.CDLL('libamdhip64.so.7')
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            if hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1)):
                return None
        return torch.cuda.ExternalStream(h.value, device=dev)
    except (OSError, AttributeError, RuntimeError):
        return None


def _copy(t, dst, after_event):
    import torch
    dev = t.device
    s = _state.get(('stream', dev.index))
    if s is None:
        s = _nonblocking_stream(dev) or torch.cuda.Stream(dev)
        _state[('stream', dev.index)] = s
    same = torch.empty(0, dtype=t.dtype).numpy().dtype == dst.dtype
    with torch.cuda.stream(s):
        s.wait_event(after_event)
        if same:
            torch.from_numpy(dst).copy_(t)
        else:
            host = t.cpu()
    s.synchronize()
    if not same:   # e.g. the int32 device counts -> the outdir's int64 raw
        np.copyto(dst, host.numpy(), casting='safe')


def small_to_host(t):
    """A small device tensor's values on the host now, through pinned
    memory: a copy into pageable memory is staged by the HIP runtime behind
    every other pageable copy in flight -- this module's background copies
    among them -- and a 4 KB table waited ~47 ms behind them (r06an)."""
    import torch
    h = torch.empty(tuple(t.shape), dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h.numpy()


def to_host_async(t, dtype=None, dst=None):
    """(host array, ready callable) for device tensor ``t`` (contiguous);
    the copy starts after the work enqueued so far on torch's current stream
    of t's device. ``dtype``: the host array's dtype when it differs from
    t's (a safe widening, done on the copy thread). ``dst``: a host array of
    t's shape allocated earlier (host_empty) to land in -- a large host
    allocation made while this module's thread is paging in an earlier
    copy's destination waits for the address-space lock (~1 ms per 100 MB
    on the GPU box's host, measured r06)."""
    import torch
    t = t.contiguous()
    np_dtype = dtype if dtype is not None else \
        torch.empty(0, dtype=t.dtype).numpy().dtype
    if dst is None:
        dst = np.empty(tuple(t.shape), dtype=np_dtype)
    elif dst.shape != tuple(t.shape) or dst.dtype != np_dtype:
        raise ValueError('to_host_async: dst %s %s for a %s %s tensor'
                         % (dst.shape, dst.dtype, tuple(t.shape), np_dtype))
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    # the copy writes through its own view: the write-behind queue marks the
    # array it is handed read-only (core._save_npy, owned=True) while the
    # copy may still be landing
    fut = _pool().submit(_copy, t, dst.view(), ev)

    def ready():
        fut.result()
    return dst, ready
