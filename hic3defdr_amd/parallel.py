"""Multi-GPU sharding of the hot path.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI;
"gloo" works too). ``HiC3DeFDR.run_to_qvalues()`` under torchrun shards
itself (``Shards``): every rank prepares and tests its own chromosomes and
writes their outdir files (one shared outdir, as the reference's per-
chromosome processes do); estimate_disp keeps the genome-wide pooling by a
re-shard by distance; BH runs genome-wide as a sample sort of the p-values
over the ranks (``bh_sharded``).

* prepare_data and lrt are independent per chromosome: chromosomes are
  assigned to ranks by greedy longest-processing-time on pixel counts
  (``lpt_assign``); no data-path collective.
* estimate_disp pools every distance genome-wide (reference
  analysis.py:169-206), so per-shard dispersions would NOT equal the
  reference. The segments (distance, condition) are independent of each
  other, so the pixels are re-sharded by DISTANCE for this stage
  (``disp_per_dist_by_distance``): the distances go to ranks by LPT on
  their genome-wide pixel counts (one all-reduce of a D-long count vector,
  ``distance_owners``), one all_to_all moves every disp pixel (raw, row,
  dist, chromosome, size-factor row: 15 bytes at R = 4; f is rebuilt from
  them bit for bit on arrival, ``exchange_compact``) to the rank owning its
  distance, each rank runs the
  single-GPU driver -- every Brent search in-kernel -- on the distances it
  owns, and one all-reduce of the D x C table (owners' rows, zeros
  elsewhere) gives every rank the same disp_per_dist. The only change from
  one GPU is the order of each segment's pixels (ULP-level).
* BH (``bh_sharded``, used by ``distributed_bh`` and bench): each rank
  sorts its p-values, ships each to the rank owning its value range, ranks
  its bucket globally from the bucket sizes and completes the reverse
  minimum with the higher buckets' minima -- O(n / world) sort work per rank
  and two all_to_alls of one double per p-value, instead of every rank
  sorting the whole genome's p-values; bit-identical to one process' BH
  (tied p-values share one q, so neither the rank order nor the order
  inside a tie changes a bit). ``bh_all_ranks`` (all_gather + one BH of
  everything on every rank) remains for host BH functions.
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


def distance_owners(counts, world):
    """Rank owning each distance: LPT over the distances by their genome-wide
    weight (`counts`, (D,)): pixel counts, or the modelled / measured work of
    each distance (``distance_cost``), so every rank gets about the same
    work. Deterministic: every rank computes the same table from the same
    weights."""
    counts = np.asarray(counts)
    counts = counts.astype(np.float64 if counts.dtype.kind == 'f'
                           else np.int64)
    order = np.lexsort((np.arange(len(counts)), -counts))
    loads = np.zeros(world, dtype=counts.dtype)
    owner = np.zeros(len(counts), dtype=np.int32)
    for d in order:
        r = int(np.argmin(loads))        # first of the least loaded
        owner[d] = r
        loads[r] += counts[d]
    return owner


def distance_cost(counts, count_sums, n_reps):
    """A-priori work of each distance for ``distance_owners``: its pixels x
    a per-pixel cost that grows with the distance's mean count per
    pixel-replicate (``count_sums`` / (``counts`` x ``n_reps``)): the
    q2qnbinom incomplete-gamma series / continued fractions run longer for
    larger means (their trip counts grow like the square root of the gamma
    shape mu / (1 + disp mu)), the Brent NLL passes do not. Calibrated on
    the measured per-segment work of the cfg3 genome (tools/emulate_ranks.py,
    profiles/r04/)."""
    counts = np.asarray(counts, dtype=np.float64)
    mu = np.asarray(count_sums, dtype=np.float64) / np.maximum(
        counts * n_reps, 1.0)
    shape = mu / (1.0 + 0.05 * mu)
    return counts * (1.0 + 0.35 * np.sqrt(shape))


def _xdev(dev, group=None):
    import torch
    import torch.distributed as dist
    # gloo exchanges host tensors
    return dev if dist.get_backend(group) != 'gloo' else torch.device('cpu')


def _split(m, k, j):
    """Size of part j of a block of m records cut into k parts (the same on
    the sending and the receiving rank)."""
    return m * (j + 1) // k - m * j // k


def exchange_columns(cols, owner, group=None, chunks=1):
    """Moves pixel i of every column in ``cols`` (tensors of n rows: (n,) or
    (n, k), any dtype, one device) to the rank ``owner[i]`` names, packed as
    one byte record per pixel (the columns' bytes side by side). Returns this
    rank's received columns (same dtypes and trailing shapes): the pixels of
    source rank 0 first, each source's in its own order.

    ``chunks`` > 1: every destination's block is cut into that many parts
    and part j of all blocks goes in its own all_to_all_single, issued
    asynchronously -- the packing of part j + 1 (a gather on the device)
    runs while part j is on the wire, and the receiving rank places each
    part at its offset, so the result is the one-shot exchange's bit for
    bit (tests/test_dist_gloo.py). Every rank issues the same number of
    collectives, pixels or not."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = cols[0].device
    xdev = _xdev(dev, group)
    n = int(cols[0].shape[0])
    tails = [tuple(c.shape[1:]) for c in cols]
    widths = [int(np.prod(t, dtype=np.int64)) * c.element_size()
              for t, c in zip(tails, cols)]
    width = int(sum(widths))
    order = torch.argsort(owner, stable=True)

    def as_bytes(t, w):
        if n == 0:  # an empty tensor's stride cannot be re-viewed
            return torch.empty((0, w), dtype=torch.uint8, device=dev)
        return t.contiguous().view(torch.uint8).reshape(n, w)

    send = torch.bincount(owner, minlength=world)
    recv = torch.empty_like(send, device=xdev)
    dist.all_to_all_single(recv, send.to(xdev), group=group)
    s_list, r_list = send.tolist(), recv.tolist()
    m = int(sum(r_list))
    k = max(1, int(chunks))
    bcols = [as_bytes(c, w) for c, w in zip(cols, widths)]
    s_off = np.concatenate([[0], np.cumsum(s_list)])
    r_off = np.concatenate([[0], np.cumsum(r_list)])
    works, parts = [], []
    for j in range(k):
        ss = [_split(s_list[d], k, j) for d in range(world)]
        rs = [_split(r_list[d], k, j) for d in range(world)]
        # rows of part j of every destination block, in block order
        idx = torch.cat([order[int(s_off[d]) + s_list[d] * j // k:
                               int(s_off[d]) + s_list[d] * j // k + ss[d]]
                         for d in range(world)]) if n else order[:0]
        rec = torch.cat([c[idx] for c in bcols], dim=1).to(xdev)
        got = torch.empty((int(sum(rs)), width), dtype=torch.uint8,
                          device=xdev)
        works.append(dist.all_to_all_single(
            got, rec, output_split_sizes=rs, input_split_sizes=ss,
            group=group, async_op=True))
        parts.append((got, rs, rec))
    out = torch.empty((m, width), dtype=torch.uint8, device=xdev)
    for j, (w, (got, rs, _)) in enumerate(zip(works, parts)):
        w.wait()
        pos = 0
        for d in range(world):
            a = int(r_off[d]) + r_list[d] * j // k
            out[a:a + rs[d]] = got[pos:pos + rs[d]]
            pos += rs[d]
    out = out.to(dev)
    res, pos = [], 0
    for c, t, w in zip(cols, tails, widths):
        if m:
            res.append(out[:, pos:pos + w].contiguous().view(c.dtype)
                       .reshape((m,) + t))
        else:
            res.append(torch.empty((0,) + t, dtype=c.dtype, device=dev))
        pos += w
    return res


def exchange_by_owner(t_raw, t_f, t_dist, owner, group=None, chunks=1):
    """exchange_columns of (raw (n, R) int32, f (n, R) float64, dist (n,)
    int32): one 12 R + 4 byte record per pixel (the full record; the
    distance re-shard ships the keys of f instead when it has them,
    exchange_compact)."""
    return tuple(exchange_columns([t_raw, t_f, t_dist], owner, group,
                                  chunks))


class PixelKeys(object):
    """What the distance re-shard ships instead of a disp pixel's f
    (8 R bytes): the keys f is rebuilt from on the receiving rank, bit for
    bit -- f = (bias[row] * bias[row + dist]) * sf (h3d_disp_pixels_dev's
    product, analysis.py:181) -- plus this rank's tables.

    row, chrom, sfi: (n,) int32 tensors on the pixels' device: the pixel's
    bin row, its chromosome's index in the genome (0 .. nchrom - 1, the same
    on every rank), the row of its chromosome's size-factor table.
    tables: {chromosome index: (bias (n_bins, R), size-factor rows (S, R))}
    for this rank's chromosomes (host float64; the bias filtered as
    core.load_bias). ``device_tables`` stacks every rank's (one all-reduce of
    the sizes, one of the rows; cached)."""

    def __init__(self, row, chrom, sfi, tables, nchrom):
        self.row, self.chrom, self.sfi = row, chrom, sfi
        self.tables = tables
        self.nchrom = int(nchrom)
        self._dev = None

    def device_tables(self, dev, R, group=None):
        """(bias (B, R), boff (nchrom + 1), sf (S, R), soff (nchrom + 1)) on
        ``dev``, every rank's chromosomes stacked in genome order: each
        chromosome is held by one rank, the others contribute zeros to the
        two sums (x + 0 = x: the rows arrive bit for bit)."""
        import torch
        import torch.distributed as dist
        if self._dev is not None:
            return self._dev
        xdev = _xdev(dev, group)
        G = self.nchrom
        sizes = np.zeros(2 * G, dtype=np.int64)
        for g, (b, s) in self.tables.items():
            sizes[g], sizes[G + g] = len(b), len(s)
        t_sizes = torch.from_numpy(sizes).to(xdev)
        dist.all_reduce(t_sizes, op=dist.ReduceOp.SUM, group=group)
        sizes = t_sizes.cpu().numpy()
        boff = np.concatenate([[0], np.cumsum(sizes[:G])]).astype(np.int64)
        soff = np.concatenate([[0], np.cumsum(sizes[G:])]).astype(np.int64)
        rows = np.zeros((int(boff[-1] + soff[-1]), R))
        for g, (b, s) in self.tables.items():
            rows[boff[g]:boff[g + 1]] = b
            rows[boff[-1] + soff[g]:boff[-1] + soff[g + 1]] = s
        t_rows = torch.from_numpy(rows).to(xdev)
        dist.all_reduce(t_rows, op=dist.ReduceOp.SUM, group=group)
        t_rows = t_rows.to(dev)
        nb = int(boff[-1])
        self._dev = (t_rows[:nb].contiguous(),
                     torch.from_numpy(boff).to(dev),
                     t_rows[nb:].contiguous(),
                     torch.from_numpy(soff).to(dev))
        return self._dev


def _narrowest(vmax):
    """The narrowest integer dtype holding 0 .. vmax."""
    import torch
    for dt, top in ((torch.uint8, 255), (torch.int16, 32767)):
        if vmax <= top:
            return dt
    return torch.int32


def exchange_compact(ctx, t_raw, t_dist, keys, owner, group=None, chunks=1):
    """The distance re-shard's pixel exchange with f rebuilt on arrival: one
    record per pixel of raw (R counts), row, dist, chromosome and
    size-factor row, each column in the narrowest integer width that holds
    every rank's values (one all-reduce of the four maxima; the escape to a
    wider column is automatic) -- R = 4, counts < 2^15, D <= 256, <= 256
    chromosomes and size-factor rows: 15 bytes against the full record's 52
    -- then f by h3d_pixel_f_dev from the
    stacked bias / size-factor tables (PixelKeys.device_tables). Returns the
    received (raw (m, R) int32, f (m, R) float64, dist (m,) int32), bit for
    bit what exchange_by_owner delivers."""
    import torch
    import torch.distributed as dist
    dev = t_raw.device
    xdev = _xdev(dev, group)
    n, R = t_raw.shape
    tabs = keys.device_tables(dev, R, group)
    mx = torch.zeros(4, dtype=torch.int64, device=dev)
    if n:
        mx = torch.stack([t_raw.max().long(), t_dist.max().long(),
                          keys.chrom.max().long(), keys.sfi.max().long()])
    lo = min(int(t_raw.min()), int(t_dist.min()), int(keys.chrom.min()),
             int(keys.sfi.min())) if n else 0
    if lo < 0:
        raise ValueError('exchange_compact: negative count, distance or key')
    mx = mx.to(xdev)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    w = [_narrowest(int(v)) for v in mx.tolist()]
    cols = [t_raw.to(w[0]), keys.row.to(torch.int32), t_dist.to(w[1]),
            keys.chrom.to(w[2]), keys.sfi.to(w[3])]
    raw_m, row_m, dist_m, chrom_m, sfi_m = exchange_columns(cols, owner,
                                                            group, chunks)
    m = int(raw_m.shape[0])
    raw_m = raw_m.to(torch.int32)
    dist_m = dist_m.to(torch.int32).contiguous()
    f_m = torch.empty((m, R), dtype=torch.float64, device=dev)
    if m:
        row_m = row_m.contiguous()
        chrom_m = chrom_m.to(torch.int32).contiguous()
        sfi_m = sfi_m.to(torch.int32).contiguous()
        ctx.pixel_f_dev(row_m.data_ptr(), dist_m.data_ptr(),
                        chrom_m.data_ptr(), sfi_m.data_ptr(), m, R,
                        tabs[0].data_ptr(), tabs[1].data_ptr(),
                        tabs[2].data_ptr(), tabs[3].data_ptr(), keys.nchrom,
                        f_m.data_ptr())
    return raw_m.contiguous(), f_m, dist_m


def compact_record_bytes(R, raw_max, dist_max, nchrom, sf_rows):
    """Bytes of one exchange_compact record (the model of
    tools/emulate_ranks.py)."""
    import torch
    sz = [torch.empty(0, dtype=_narrowest(v)).element_size()
          for v in (raw_max, dist_max, nchrom - 1, sf_rows - 1)]
    return R * sz[0] + 4 + sz[1] + sz[2] + sz[3]


# parts of the distance re-shard's all_to_all (H3D_RESHARD_CHUNKS): the
# packing of one part overlaps the transfer of the previous
RESHARD_CHUNKS = int(os.environ.get('H3D_RESHARD_CHUNKS', '4'))


def disp_per_dist_by_distance(ctx, t_raw, t_f, t_dist, cond_of_rep, C, D,
                              group=None, chunks=None, keys=None):
    """estimate_disp's (D, C) disp_per_dist over every rank's pixels: the
    distances go to ranks by LPT on their genome-wide pixel counts (one
    all-reduce of D counts), the pixels move to the rank owning their
    distance (the all_to_all in ``chunks`` asynchronous parts), each rank
    runs the single-GPU driver on what it received, and ONE all-reduce of
    the owners' rows gives every rank the whole table.

    t_raw (n, R) int32, t_f (n, R) float64, t_dist (n,) int32: this rank's
    disp pixels on its GPU. ``keys`` (PixelKeys): ship the keys of f instead
    of f (exchange_compact: 15-byte records at R = 4 instead of 52, f rebuilt
    bit for bit on arrival); without them the full record
    (exchange_by_owner). libh3d must run on torch's current stream (a real
    one: see make_allreduce). Returns the table as a (D, C) numpy array."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = t_raw.device
    xdev = _xdev(dev, group)
    n, R = t_raw.shape
    dl = t_dist.long()
    inb = (dl >= 0) & (dl < D)
    cnt = torch.bincount(dl[inb], minlength=D)[:D].to(xdev)
    dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=group)
    owner_of = distance_owners(cnt.cpu().numpy(), world)
    # distances outside [0, D) go to rank 0, whose driver rejects them
    owner = torch.zeros(n, dtype=torch.int64, device=dev)
    owner[inb] = torch.from_numpy(owner_of.astype(np.int64)).to(dev)[dl[inb]]
    k = RESHARD_CHUNKS if chunks is None else chunks
    if keys is not None:
        raw_m, f_m, dist_m = exchange_compact(ctx, t_raw, t_dist, keys, owner,
                                              group, k)
    else:
        raw_m, f_m, dist_m = exchange_by_owner(t_raw, t_f, t_dist, owner,
                                               group, k)
    m = int(raw_m.shape[0])
    tab = ctx.disp_per_dist_dev(raw_m.data_ptr(), f_m.data_ptr(),
                                dist_m.data_ptr(), m, R, cond_of_rep, C, D)
    tab[owner_of != rank] = 0.0
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
                if dist.get_backend() == 'nccl':
                    # collectives (barrier, the BH all_gather) run on the
                    # current device: this rank's GPU, not cuda:0
                    import torch
                    torch.cuda.set_device(device_for_rank())
        except ImportError:
            pass
        sizes = sizes or {c: 1 for c in chroms}
        self.assign = lpt_assign({c: sizes[c] for c in chroms}, self.world)
        mine = set(self.assign[self.rank])
        self.mine = [c for c in chroms if c in mine]   # in chromosome order
        self.order = {c: i for i, c in enumerate(chroms)}

    @property
    def sharded(self):
        # H3D_FORCE_SHARDED=1: the sharded paths (distance re-shard, sharded
        # BH) even at world size 1 -- a test hook, so that the collectives run
        # under RCCL on a one-GPU box (tests/test_gpu_multirank.py)
        return self.world > 1 or (self.dist is not None and
                                  os.environ.get('H3D_FORCE_SHARDED') == '1')

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()


def chrom_sizes(bias_patterns, chroms):
    """Bins per chromosome (line count of the first replicate's bias file),
    the LPT weight: the pixel band has ~bins x (dmax + 1) pixels."""
    out = {}
    for c in chroms:
        with open(bias_patterns[0].replace('<chrom>', c), 'rb') as fh:
            data = fh.read()
        # the file's lines (a last one without its newline counts)
        out[c] = data.count(b'\n') + (1 if data and not
                                       data.endswith(b'\n') else 0)
    return out


def gather_all(t, group=None):
    """Every rank's 1-D tensor `t` (any length) concatenated in rank order,
    on every rank (one all_gather of the lengths, one of the values padded
    to the longest), and this rank's offset in it."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    xdev = _xdev(t.device, group)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=xdev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    top = max(ns + [1])
    buf = torch.zeros(top, dtype=t.dtype, device=xdev)
    buf[:t.numel()] = t.to(xdev)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    allv = torch.cat([parts[r][:ns[r]] for r in range(world)])
    return allv.to(t.device), int(sum(ns[:rank]))


def bh_all_ranks(t_p, bh_fn, group=None):
    """Genome-wide BH over every rank's p-values `t_p` (1-D float64 tensor):
    each rank gathers all of them, runs `bh_fn` (tensor -> tensor, e.g. the
    GPU BH) on the whole vector and returns its own slice of q."""
    allp, off = gather_all(t_p, group)
    return bh_fn(allp)[off:off + t_p.numel()]


class DeviceBhOps(object):
    """bh_sharded's per-rank compute on the rank's GPU (libh3d's
    h3d_bh_sort_dev / _scan_dev / _finish_dev, tensors on the ctx's
    device). The ctx may run on its own stream: torch's current stream is
    drained before each call (its tensors are the inputs), and each call
    returns with the ctx stream drained."""

    def __init__(self, ctx):
        self.ctx = ctx

    def _ready(self, t):
        import torch
        torch.cuda.current_stream(t.device).synchronize()

    def sort(self, keys, vals=None):
        """(keys ascending with non-finite last, their values -- the given
        ones or the positions --, number of finite keys)."""
        import torch
        keys = keys.contiguous()
        self._ready(keys)
        n = keys.numel()
        ko = torch.empty_like(keys)
        vo = torch.empty(n, dtype=torch.int64, device=keys.device)
        m = self.ctx.bh_sort_dev(keys.data_ptr(),
                                 None if vals is None else vals.data_ptr(),
                                 n, ko.data_ptr(), vo.data_ptr())
        return ko, vo, m

    def scan(self, ps, offset, m):
        """(suffix minimum of the BH ratios of a sorted bucket at global
        ranks offset.., its first entry)."""
        import torch
        sc = torch.empty_like(ps)
        self._ready(ps)
        lo = self.ctx.bh_scan_dev(ps.data_ptr(), ps.numel(), offset, m,
                                  sc.data_ptr())
        return sc, lo

    def finish(self, scanned, higher_min):
        import torch
        q = torch.empty_like(scanned)
        self._ready(scanned)
        self.ctx.bh_finish_dev(scanned.data_ptr(), scanned.numel(),
                               higher_min, q.data_ptr())
        return q


def bh_sharded(t_p, ops, group=None, samples=64):
    """Genome-wide BH over every rank's p-values `t_p` (1-D float64 tensor),
    each rank computing the q-values of one VALUE range (a sample sort)
    instead of every rank sorting all of them: returns this rank's q (same
    order as `t_p`), bit-identical to the single-process BH of all ranks'
    p-values concatenated (reference analysis.py:286-303; q of NaN p is
    NaN and NaN p are not counted).

    1. each rank sorts its p-values (ops.sort) and contributes `samples`
       evenly spaced order statistics + its finite count to one all_gather;
       every rank derives the same world - 1 splitters (count-weighted
       quantiles), so equal values always land in one bucket;
    2. one all_gather of every rank's per-bucket counts (global offsets),
       one all_to_all of the values to their bucket's rank;
    3. the bucket is sorted, its ratios p_(j) / ((offset + j + 1) / m)
       min-scanned from the top (ops.scan), one all_gather of the bucket
       minima completes the reverse minimum across buckets (ops.finish);
    4. one all_to_all returns each q to the rank (and position) it came
       from.
    `ops`: DeviceBhOps (the GPU) or a host stand-in with the same methods."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = t_p.device
    xdev = _xdev(dev, group)
    n = t_p.numel()
    ks, idx, m_loc = ops.sort(t_p.to(torch.float64))
    fin = ks[:m_loc]
    # 1. splitters
    if m_loc:
        pos = torch.div(torch.arange(samples, device=dev) * m_loc, samples,
                        rounding_mode='floor')
        smp = fin[pos]
    else:
        smp = torch.full((samples,), float('inf'), dtype=torch.float64,
                         device=dev)
    meta = torch.cat([smp, torch.tensor([float(m_loc)], dtype=torch.float64,
                                        device=dev)]).to(xdev)
    got = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(got, meta, group=group)
    g = torch.stack(got).cpu().numpy()
    cnt = g[:, -1]
    sv = g[:, :-1].ravel()
    sw = np.repeat(cnt / samples, samples)
    keep = sw > 0
    sv, sw = sv[keep], sw[keep]
    o = np.argsort(sv, kind='stable')
    sv, cw = sv[o], np.cumsum(sw[o])
    if len(sv):
        at = np.searchsorted(cw, cw[-1] * np.arange(1, world) / world)
        split = sv[np.minimum(at, len(sv) - 1)]
    else:
        split = np.full(world - 1, np.inf)
    # 2. bucket b = (split[b - 1], split[b]]
    cut = torch.searchsorted(fin, torch.from_numpy(split).to(dev),
                             right=True).tolist() if world > 1 else []
    bounds = [0] + [int(c) for c in cut] + [m_loc]
    send = [bounds[b + 1] - bounds[b] for b in range(world)]
    st = torch.tensor(send, dtype=torch.int64, device=xdev)
    sends = [torch.empty_like(st) for _ in range(world)]
    dist.all_gather(sends, st, group=group)
    table = np.stack([s.cpu().numpy() for s in sends])   # [src, bucket]
    recv = [int(v) for v in table[:, rank]]
    sizes = table.sum(axis=0)
    offset, m = int(sizes[:rank].sum()), int(sizes.sum())
    mb = int(sizes[rank])
    got_p = torch.empty(mb, dtype=torch.float64, device=xdev)
    dist.all_to_all_single(got_p, fin.to(xdev), output_split_sizes=recv,
                           input_split_sizes=send, group=group)
    # 3. the bucket's q
    bs, perm, _ = ops.sort(got_p.to(dev))
    sc, lo = ops.scan(bs, offset, m)
    lt = torch.tensor([lo], dtype=torch.float64, device=xdev)
    los = [torch.empty_like(lt) for _ in range(world)]
    dist.all_gather(los, lt, group=group)
    higher = min([float(v.item()) for v in los[rank + 1:]] or [float('inf')])
    q_sorted = ops.finish(sc, higher)
    # 4. back in received order, then to the senders
    q_recv = torch.empty_like(q_sorted)
    q_recv[perm] = q_sorted
    back = torch.empty(m_loc, dtype=torch.float64, device=xdev)
    dist.all_to_all_single(back, q_recv.to(xdev), output_split_sizes=send,
                           input_split_sizes=recv, group=group)
    q = torch.full((n,), float('nan'), dtype=torch.float64, device=dev)
    q[idx[:m_loc]] = back.to(dev)
    return q


def distributed_bh(shards, pvalues, bh=None, ctx=None):
    """Genome-wide BH over every rank's p-values (analysis.py:286-303 over
    all chromosomes): ``pvalues`` maps this rank's chromosomes to arrays.
    With ``ctx`` (the product): ``bh_sharded`` on the rank's GPU; else
    ``bh`` maps a numpy vector to its q-values and runs on all-gathered
    p-values. Returns this rank's chromosomes' q-values (dict)."""
    import torch
    dist = shards.dist
    mine = [c for c in shards.mine if c in pvalues]
    local = np.concatenate([np.asarray(pvalues[c], dtype=np.float64)
                            for c in mine]) if mine else np.zeros(0)
    if ctx is not None:
        gdev = torch.device('cuda', ctx.device)
        q = bh_sharded(torch.from_numpy(local).to(gdev), DeviceBhOps(ctx))
    else:
        dev = torch.device('cuda', torch.cuda.current_device()) \
            if dist.get_backend() == 'nccl' else torch.device('cpu')
        q = bh_all_ranks(torch.from_numpy(local).to(dev),
                         lambda t: torch.from_numpy(bh(t.cpu().numpy())))
    q = q.cpu().numpy()
    off = np.concatenate([[0], np.cumsum([len(pvalues[c]) for c in mine])])
    return {c: q[off[i]:off[i + 1]] for i, c in enumerate(mine)}


def device_for_rank():
    """GPU of this process: ``H3D_DEVICE`` if set (several ranks on one GPU,
    tests), else LOCAL_RANK."""
    return int(os.environ.get('H3D_DEVICE', os.environ.get('LOCAL_RANK', '0')))
