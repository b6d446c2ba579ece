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
  reference. The segments (distance, condition) are independent of each
  other, so the pixels are re-sharded by DISTANCE for this stage
  (``disp_per_dist_by_distance``): one all_to_all moves every disp pixel
  (raw, f, dist: 12 R + 4 bytes) to the rank owning its distance (d mod
  world), each rank runs the single-GPU driver -- every Brent search
  in-kernel -- on the distances it owns, and one all-reduce of the D x C
  table (owners' rows, zeros elsewhere) gives every rank the same
  disp_per_dist. Two collectives per estimate_disp instead of one per data
  pass; the only change from one GPU is the order of each segment's pixels
  (ULP-level).
* The per-pass alternative (``make_allreduce``, H3D_DISP_SHARD=pass) keeps
  the pixels in place and all-reduces the per-(distance, condition) NLL sums
  of every Brent step (D x C doubles, ~3 KB, ~54 passes per cfg2
  estimate_disp); every rank advances identical state machines.
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


def disp_per_dist_by_distance(ctx, t_raw, t_f, t_dist, cond_of_rep, C, D,
                              group=None):
    """estimate_disp's (D, C) disp_per_dist over every rank's pixels: the
    pixels move to the rank owning their distance (d mod world) with ONE
    all_to_all, each rank runs the single-GPU driver on what it received,
    and ONE all-reduce of the owners' rows gives every rank the whole table.

    t_raw (n, R) int32, t_f (n, R) float64, t_dist (n,) int32: this rank's
    disp pixels on its GPU. libh3d must run on torch's current stream (a real
    one: see make_allreduce). Returns the table as a (D, C) numpy array."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = t_raw.device
    n, R = t_raw.shape
    owner = t_dist.long() % world
    order = torch.argsort(owner, stable=True)
    width = 12 * R + 4

    def as_bytes(t, w):
        if n == 0:  # an empty tensor's stride cannot be re-viewed
            return torch.empty((0, w), dtype=torch.uint8, device=dev)
        return t.contiguous().view(torch.uint8).reshape(n, w)

    # one byte record per pixel: raw (4 R) | f (8 R) | dist (4)
    rec = torch.cat([as_bytes(t_raw, 4 * R), as_bytes(t_f, 8 * R),
                     as_bytes(t_dist, 4)], dim=1)[order].contiguous()
    send = torch.bincount(owner, minlength=world)
    # gloo exchanges host tensors
    xdev = dev if dist.get_backend(group) != 'gloo' else torch.device('cpu')
    recv = torch.empty_like(send, device=xdev)
    dist.all_to_all_single(recv, send.to(xdev), group=group)
    s_list, r_list = send.tolist(), recv.tolist()
    m = int(sum(r_list))
    out = torch.empty((m, width), dtype=torch.uint8, device=xdev)
    dist.all_to_all_single(out, rec.to(xdev), output_split_sizes=r_list,
                           input_split_sizes=s_list, group=group)
    out = out.to(dev)
    if m:
        raw_m = out[:, :4 * R].contiguous().view(torch.int32).reshape(m, R)
        f_m = out[:, 4 * R:12 * R].contiguous().view(torch.float64).reshape(m, R)
        dist_m = out[:, 12 * R:].contiguous().view(torch.int32).reshape(m)
    else:
        raw_m = torch.empty((0, R), dtype=torch.int32, device=dev)
        f_m = torch.empty((0, R), dtype=torch.float64, device=dev)
        dist_m = torch.empty(0, dtype=torch.int32, device=dev)
    tab = ctx.disp_per_dist_dev(raw_m.data_ptr(), f_m.data_ptr(),
                                dist_m.data_ptr(), m, R, cond_of_rep, C, D)
    own = (np.arange(D) % world) == rank
    tab[~own] = 0.0
    t_tab = torch.from_numpy(tab).to(xdev)
    dist.all_reduce(t_tab, op=dist.ReduceOp.SUM, group=group)
    return t_tab.cpu().numpy()


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
