"""Multi-GPU sharding of the hot path.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).

* prepare_data and lrt are independent per chromosome: chromosomes are
  assigned to ranks by greedy longest-processing-time on pixel counts
  (``lpt_assign``); no data-path collective.
* estimate_disp pools every distance genome-wide (reference
  analysis.py:169-206), so per-shard dispersions would NOT equal the
  reference. Instead every rank keeps its own pixels and the per-(distance,
  condition) NLL sums of each Brent step are summed across ranks with one
  small all-reduce (D x C doubles, ~3 KB) per data pass
  (``make_allreduce``). Every rank then advances identical qcml/Brent state
  machines, so all ranks finish with the same disp_per_dist, bit for bit,
  and smooth it identically. The only change from one GPU is the order in
  which the per-rank partial sums are added (ULP-level).
"""
import ctypes


def lpt_assign(sizes, world_size):
    """Greedy LPT: items (name -> size) onto ``world_size`` bins. Returns a
    list of name lists, one per rank (deterministic)."""
    order = sorted(sizes.items(), key=lambda kv: (-kv[1], str(kv[0])))
    loads = [0] * world_size
    out = [[] for _ in range(world_size)]
    for name, s in order:
        r = min(range(world_size), key=lambda i: (loads[i], i))
        out[r].append(name)
        loads[r] += s
    return out


class _CudaArray(object):
    """Zero-copy view of a device buffer for torch.as_tensor."""

    def __init__(self, ptr, count):
        self.__cuda_array_interface__ = {
            'shape': (int(count),), 'typestr': '<f8',
            'data': (int(ptr), False), 'version': 3, 'strides': None}


def make_allreduce(group=None):
    """``reduce(ptr, count)`` for ``Context.disp_per_dist_dev``: sums a
    device buffer of doubles in place across ranks on the current stream.
    The caller must run libh3d on torch's current stream
    (``ctx.set_stream(torch.cuda.current_stream().cuda_stream)``)."""
    import torch
    import torch.distributed as dist

    def reduce(ptr, count):
        t = torch.as_tensor(_CudaArray(ptr, count), device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)

    return reduce


def make_cpu_allreduce(group=None):
    """Same contract for the host emulation (gloo, CPU tests): ``ptr`` is a
    host address."""
    import numpy as np
    import torch
    import torch.distributed as dist

    def reduce(ptr, count):
        buf = (ctypes.c_double * int(count)).from_address(int(ptr))
        arr = np.frombuffer(buf, dtype=np.float64)
        t = torch.from_numpy(arr)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)

    return reduce
