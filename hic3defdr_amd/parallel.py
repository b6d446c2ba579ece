"""Multi-GPU sharding of the hot path.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI;
"gloo" works too). ``HiC3DeFDR.run_to_qvalues()`` under torchrun shards
itself (``Shards``): every rank prepares and tests its own chromosomes and
writes their outdir files (one shared outdir, as the reference's per-
chromosome processes do); estimate_disp keeps the genome-wide pooling with
the per-pass all-reduce below; BH gathers the loop pixels' p-values on rank 0
and scatters the q-values back (``distributed_bh``).

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
import os

import numpy as np


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
    device buffer of doubles in place across ranks on torch's current
    stream. libh3d must launch on that same stream, and it must be a real
    (non-default) stream: ``s = torch.cuda.Stream(); ctx.set_stream(
    s.cuda_stream)`` under ``torch.cuda.stream(s)`` -- the default stream's
    handle is 0, which h3d_set_stream takes as "the ctx's own stream"."""
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


class Shards(object):
    """This process's place in the job: rank, world size and the chromosomes
    it owns (LPT over ``sizes``). World size 1 (no torch.distributed process
    group) owns everything."""

    def __init__(self, chroms, sizes=None):
        self.world, self.rank, self.dist = 1, 0, None
        try:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                self.world = dist.get_world_size()
                self.rank = dist.get_rank()
                self.dist = dist
        except ImportError:
            pass
        sizes = sizes or {c: 1 for c in chroms}
        self.assign = lpt_assign({c: sizes[c] for c in chroms}, self.world)
        mine = set(self.assign[self.rank])
        self.mine = [c for c in chroms if c in mine]   # in chromosome order
        self.order = {c: i for i, c in enumerate(chroms)}

    @property
    def sharded(self):
        return self.world > 1

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()


def chrom_sizes(bias_patterns, chroms):
    """Bins per chromosome (line count of the first replicate's bias file),
    the LPT weight: the pixel band has ~bins x (dmax + 1) pixels."""
    out = {}
    for c in chroms:
        with open(bias_patterns[0].replace('<chrom>', c), 'rb') as fh:
            out[c] = sum(1 for _ in fh)
    return out


def distributed_bh(shards, pvalues, bh):
    """Genome-wide BH over every rank's p-values (analysis.py:286-303 over
    all chromosomes): ``pvalues`` maps this rank's chromosomes to arrays;
    rank 0 gathers them (chromosome order of ``shards.assign``), applies
    ``bh`` once and scatters each rank its chromosomes' q-values."""
    dist = shards.dist
    gathered = [None] * shards.world if shards.rank == 0 else None
    dist.gather_object(pvalues, gathered, dst=0)
    scatter_in = None
    if shards.rank == 0:
        allp = {}
        for part in gathered:
            allp.update(part)
        order = [c for r in range(shards.world) for c in shards.assign[r]]
        order = sorted(order, key=lambda c: shards.order[c])
        lens = [len(allp[c]) for c in order]
        q = bh(np.concatenate([allp[c] for c in order])) if lens else []
        off = np.concatenate([[0], np.cumsum(lens)]).astype(int)
        qs = {c: q[off[i]:off[i + 1]] for i, c in enumerate(order)}
        scatter_in = [{c: qs[c] for c in shards.assign[r]}
                      for r in range(shards.world)]
    out = [None]
    dist.scatter_object_list(out, scatter_in, src=0)
    return out[0]


def device_for_rank():
    """GPU of this process: ``H3D_DEVICE`` if set (several ranks on one GPU,
    tests), else LOCAL_RANK."""
    return int(os.environ.get('H3D_DEVICE', os.environ.get('LOCAL_RANK', '0')))
