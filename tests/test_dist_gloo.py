"""world_size-2 gloo tests of the multi-GPU decomposition (CPU only).

estimate_disp is sharded by chromosome; the per-(distance, condition) NLL
sums of every data pass are all-reduced so each rank advances the same
qcml/Brent state machines (hic3defdr_amd/parallel.py). The rank-local pass
runs in the host emulation of the device driver (libh3d_hosttest.so,
h3dt_disp_rounds), the all-reduce is torch.distributed over gloo."""
import ctypes
import os
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
from hic3defdr_amd import build as h3dbuild
from hic3defdr_amd import parallel

D = 41
CHROMS = {'chrA': 260, 'chrB': 180}
CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                      ctypes.c_int64, ctypes.c_void_p)


def _prep(tmp):
    from hic3defdr_amd import synthetic
    kw = synthetic.write_dataset(tmp, CHROMS, dist_thresh_max=D - 1, seed=5)
    out = {}
    for c in CHROMS:
        npz = [p.replace('<chrom>', c) for p in kw['raw_npz_patterns']]
        bfs = [p.replace('<chrom>', c) for p in kw['bias_patterns']]
        prep = oracle.prepare_chrom(npz, bfs, kw['design'],
                                    dist_thresh_max=D - 1)
        bias = oracle.load_bias(bfs)
        di = prep['disp_idx']
        row, col = prep['row'][di], prep['col'][di]
        out[c] = (prep, bias, prep['raw'][di].astype(np.int32),
                  bias[row] * bias[col] * prep['size_factors'][di],
                  (col - row).astype(np.int32))
    return kw, out


def _rounds(raw, f, dist, cond, reduce=None):
    lib = ctypes.CDLL(h3dbuild.build_hosttest())
    C = int(cond.max()) + 1
    out = np.empty((D, C))
    fl = np.zeros((D, C), dtype=np.int32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    raw = np.ascontiguousarray(raw, dtype=np.int32)
    f = np.ascontiguousarray(f)
    dist = np.ascontiguousarray(dist, dtype=np.int32)
    cond = np.ascontiguousarray(cond, dtype=np.int32)
    if reduce is not None:
        def _cb(ptr, count, user):
            reduce(ctypes.cast(ptr, ctypes.c_void_p).value, count)
            return 0
        cb = CB(_cb)
    else:
        cb = CB()
    rc = lib.h3dt_disp_rounds(ctypes.c_int64(len(raw)), raw.shape[1], C,
                              p(raw), p(f), p(dist), p(cond), D, cb, None,
                              p(out), p(fl))
    assert rc == 0
    return out


def _worker(rank, world, tmp, port, result_file):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    kw, data = _prep(os.path.join(tmp, 'r%d' % rank))
    shards = parallel.lpt_assign({c: len(data[c][2]) for c in CHROMS}, world)
    mine = shards[rank]
    raw = np.concatenate([data[c][2] for c in mine])
    f = np.concatenate([data[c][3] for c in mine])
    dist_ = np.concatenate([data[c][4] for c in mine])
    cond = kw['design'].argmax(axis=1)
    out = _rounds(raw, f, dist_, cond, parallel.make_cpu_allreduce())
    if rank == 0:
        np.save(result_file, out)
    dist.barrier()
    dist.destroy_process_group()


def test_lpt_assign():
    assert parallel.lpt_assign({'a': 10, 'b': 7, 'c': 5, 'd': 4}, 2) == \
        [['a', 'd'], ['b', 'c']]
    assert parallel.lpt_assign({'x': 1}, 3) == [['x'], [], []]


def test_sharded_disp_equals_single_rank_and_oracle():
    h3dbuild.build_hosttest()
    with tempfile.TemporaryDirectory() as tmp:
        res = os.path.join(tmp, 'out.npy')
        port = 29500 + (os.getpid() % 1000)
        mp.spawn(_worker, args=(2, tmp, port, res), nprocs=2, join=True)
        sharded = np.load(res)
        kw, data = _prep(os.path.join(tmp, 'single'))
        raw = np.concatenate([data[c][2] for c in CHROMS])
        f = np.concatenate([data[c][3] for c in CHROMS])
        dist_ = np.concatenate([data[c][4] for c in CHROMS])
        cond = kw['design'].argmax(axis=1)
        single = _rounds(raw, f, dist_, cond)
        np.testing.assert_array_equal(np.isnan(sharded), np.isnan(single))
        # only the order of the cross-rank partial sums differs: ULP-level NLL
        # changes, which Brent's parabolic steps carry to ~1e-8 in disp
        np.testing.assert_allclose(sharded, single, rtol=1e-6, atol=1e-12)
        preps = [data[c][0] for c in CHROMS]
        biases = [data[c][1] for c in CHROMS]
        _, dpd, _ = oracle.estimate_disp(preps, biases, kw['design'],
                                         dist_thresh_max=D - 1)
        np.testing.assert_allclose(sharded, dpd, rtol=1e-6, atol=1e-12)


class _HostCtx(object):
    """Stands in for the GPU context in disp_per_dist_by_distance on CPU:
    disp_per_dist_dev reads the received host tensors through their
    addresses and runs the host emulation of the single-rank driver."""

    def disp_per_dist_dev(self, d_raw, d_f, d_dist, n, R, cond_of_rep, C, Dd,
                          reduce=None):
        assert reduce is None and Dd == D

        def arr(ptr, ctype, count):
            if count == 0:
                return np.zeros(0, dtype=np.dtype(ctype))
            buf = (ctype * count).from_address(ptr)
            return np.frombuffer(buf, dtype=np.dtype(ctype)).copy()
        raw = arr(d_raw, ctypes.c_int32, n * R).reshape(n, R)
        f = arr(d_f, ctypes.c_double, n * R).reshape(n, R)
        dist_ = arr(d_dist, ctypes.c_int32, n)
        return _rounds(raw, f, dist_, np.asarray(cond_of_rep))

    def pixel_f_dev(self, d_row, d_dist, d_chrom, d_sfi, n, R, d_bias, d_boff,
                    d_sf, d_soff, nchrom, d_f_out):
        """h3d_pixel_f_dev's product, (bias[row] * bias[col]) * sf, in
        numpy on the host tensors behind the addresses."""
        def view(ptr, ctype, count):
            buf = (ctype * count).from_address(ptr)
            return np.frombuffer(buf, dtype=np.dtype(ctype))
        row = view(d_row, ctypes.c_int32, n)
        dist_ = view(d_dist, ctypes.c_int32, n)
        g = view(d_chrom, ctypes.c_int32, n)
        sfi = view(d_sfi, ctypes.c_int32, n)
        boff = view(d_boff, ctypes.c_int64, nchrom + 1)
        soff = view(d_soff, ctypes.c_int64, nchrom + 1)
        bias = view(d_bias, ctypes.c_double, int(boff[-1]) * R).reshape(-1, R)
        sf = view(d_sf, ctypes.c_double, int(soff[-1]) * R).reshape(-1, R)
        out = view(d_f_out, ctypes.c_double, n * R).reshape(n, R)
        r0 = boff[g] + row
        out[...] = bias[r0] * bias[r0 + dist_] * sf[soff[g] + sfi]


def _reshard_worker(rank, world, tmp, port, result_file):
    import torch
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    kw, data = _prep(os.path.join(tmp, 'r%d' % rank))
    mine = parallel.lpt_assign({c: len(data[c][2]) for c in CHROMS},
                               world)[rank]
    R = kw['design'].shape[0]
    raw = np.concatenate([data[c][2] for c in mine] or
                         [np.zeros((0, R), np.int32)])
    f = np.concatenate([data[c][3] for c in mine] or [np.zeros((0, R))])
    dist_ = np.concatenate([data[c][4] for c in mine] or
                           [np.zeros(0, np.int32)])
    cond = kw['design'].argmax(axis=1).astype(np.int32)
    out = parallel.disp_per_dist_by_distance(
        _HostCtx(), torch.from_numpy(np.ascontiguousarray(raw, np.int32)),
        torch.from_numpy(np.ascontiguousarray(f)),
        torch.from_numpy(np.ascontiguousarray(dist_, np.int32)), cond,
        kw['design'].shape[1], D)
    np.save(result_file % rank, out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_distance_reshard_equals_single_rank(world):
    """parallel.disp_per_dist_by_distance: the all_to_all routing by distance
    (byte records of raw / f / dist), the per-rank single-rank driver and
    the owners' table all-reduce give every rank the single-process table.
    world 3 > 2 chromosomes: one rank starts without pixels."""
    h3dbuild.build_hosttest()
    with tempfile.TemporaryDirectory() as tmp:
        res = os.path.join(tmp, 'out_%d.npy')
        port = 29700 + (os.getpid() % 1000) + world
        mp.spawn(_reshard_worker, args=(world, tmp, port, res), nprocs=world,
                 join=True)
        kw, data = _prep(os.path.join(tmp, 'single'))
        raw = np.concatenate([data[c][2] for c in CHROMS])
        f = np.concatenate([data[c][3] for c in CHROMS])
        dist_ = np.concatenate([data[c][4] for c in CHROMS])
        single = _rounds(raw, f, dist_, kw['design'].argmax(axis=1))
        outs = [np.load(res % r) for r in range(world)]
        for o in outs[1:]:
            np.testing.assert_array_equal(o, outs[0])
        np.testing.assert_array_equal(np.isnan(outs[0]), np.isnan(single))
        # a segment's pixels arrive in rank order, not chromosome order: only
        # the order of its NLL partial sums differs
        np.testing.assert_allclose(outs[0], single, rtol=1e-6, atol=1e-12)


def _bh_worker(rank, world, port, chroms, pv, result_file):
    """Product orchestration on gloo: Shards (LPT over the chromosomes) and
    the genome-wide BH gather (rank 0) / scatter (parallel.distributed_bh)."""
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    sh = parallel.Shards(chroms, {c: len(pv[c]) for c in chroms})
    assert sh.sharded and sh.world == world
    q = parallel.distributed_bh(sh, {c: pv[c] for c in sh.mine},
                                oracle.adjust_pvalues)
    assert sorted(q) == sorted(sh.mine)
    np.save(result_file % rank, np.array([sh.mine, [q[c] for c in sh.mine]],
                                         dtype=object), allow_pickle=True)
    dist.barrier()
    dist.destroy_process_group()


def test_distributed_bh_equals_single_process():
    rng = np.random.default_rng(3)
    chroms = ['chr1', 'chr2', 'chr10', 'chrX', 'chrY']
    pv = {c: rng.uniform(0, 1, int(rng.integers(5, 300))) ** 3 for c in chroms}
    pv['chr2'][::7] = np.nan   # NaN p-values stay NaN, are not counted
    world = 3
    with tempfile.TemporaryDirectory() as tmp:
        res = os.path.join(tmp, 'q%d.npy')
        port = 29700 + (os.getpid() % 1000)
        mp.spawn(_bh_worker, args=(world, port, chroms, pv, res), nprocs=world,
                 join=True)
        got = {}
        for r in range(world):
            mine, qs = np.load(res % r, allow_pickle=True)
            got.update(dict(zip(mine, qs)))
    assert sorted(got) == sorted(chroms)
    allq = oracle.adjust_pvalues(np.concatenate([pv[c] for c in chroms]))
    off = np.concatenate([[0], np.cumsum([len(pv[c]) for c in chroms])])
    for i, c in enumerate(chroms):
        np.testing.assert_array_equal(got[c], allq[off[i]:off[i + 1]])


def test_shards_single_process_owns_everything():
    sh = parallel.Shards(['a', 'b', 'c'])
    assert not sh.sharded and sh.mine == ['a', 'b', 'c'] and sh.rank == 0


def test_distance_owners_lpt():
    counts = np.array([0, 0, 50, 40, 30, 30, 20, 10])
    own = parallel.distance_owners(counts, 3)
    loads = np.bincount(own, weights=counts, minlength=3)
    assert loads.max() - loads.min() <= counts.max()
    assert sorted(set(own[2:])) == [0, 1, 2]
    np.testing.assert_array_equal(own, parallel.distance_owners(counts, 3))
    assert (parallel.distance_owners(counts, 1) == 0).all()


GENOME = [150, 90, 130, 60, 110, 75, 140]     # a cfg3-shaped genome, small


def _genome_worker(rank, world, port, result_file):
    """cfg3's multi-GPU partition on gloo: chromosomes LPT-sharded, each rank
    draws only its own (synthetic.draw_band seeds per chromosome), the
    distance re-shard (LPT distance owners) for estimate_disp, and the
    genome-wide BH over all ranks' p-values (bh_all_ranks)."""
    import torch
    import torch.distributed as dist
    from hic3defdr_amd import synthetic
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    mine = parallel.lpt_assign({i: b for i, b in enumerate(GENOME)},
                               world)[rank]
    mine = sorted(mine)
    parts = synthetic.draw_genome(GENOME, (2, 2), D - 1, seed=4,
                                  indices=mine, keys=True)
    raw = np.concatenate([p[0] for p in parts])
    f = np.concatenate([p[1] for p in parts])
    d = np.concatenate([p[2] for p in parts])
    cond = np.array([0, 0, 1, 1], dtype=np.int32)
    tab = parallel.disp_per_dist_by_distance(
        _HostCtx(), torch.from_numpy(raw), torch.from_numpy(f),
        torch.from_numpy(d), cond, 2, D)
    # the bench's compact re-shard: the keys of f (unit size factors)
    keys = parallel.PixelKeys(
        torch.from_numpy(np.concatenate([p[3] for p in parts])),
        torch.from_numpy(np.concatenate([np.full(len(p[0]), i, np.int32)
                                         for i, p in zip(mine, parts)])),
        torch.zeros(len(raw), dtype=torch.int32),
        {i: (p[4], np.ones((1, 4))) for i, p in zip(mine, parts)},
        len(GENOME))
    tab_keys = parallel.disp_per_dist_by_distance(
        _HostCtx(), torch.from_numpy(raw), torch.from_numpy(f),
        torch.from_numpy(d), cond, 2, D, keys=keys)
    np.testing.assert_array_equal(tab_keys, tab)
    # p-values stand-in: a deterministic function of each pixel's counts
    p = torch.from_numpy((raw[:, 0] % 97 + 0.5) / 97.0 * 0.3)
    q = parallel.bh_all_ranks(
        p, lambda t: torch.from_numpy(oracle.adjust_pvalues(t.numpy())))
    np.save(result_file % rank, {'tab': tab, 'mine': sorted(mine),
                                 'q': q.numpy(), 'p': p.numpy()},
            allow_pickle=True)
    dist.barrier()
    dist.destroy_process_group()


def test_genome_partition_world3_equals_single_process():
    h3dbuild.build_hosttest()
    from hic3defdr_amd import synthetic
    world = 3
    with tempfile.TemporaryDirectory() as tmp:
        res = os.path.join(tmp, 'g%d.npy')
        port = 29900 + (os.getpid() % 1000)
        mp.spawn(_genome_worker, args=(world, port, res), nprocs=world,
                 join=True)
        outs = [np.load(res % r, allow_pickle=True).item()
                for r in range(world)]
    parts = synthetic.draw_genome(GENOME, (2, 2), D - 1, seed=4)
    raw = np.concatenate([p[0] for p in parts])
    f = np.concatenate([p[1] for p in parts])
    d = np.concatenate([p[2] for p in parts])
    single = _rounds(raw, f, d, np.array([0, 0, 1, 1]))
    assert sorted(sum((o['mine'] for o in outs), [])) == list(range(len(GENOME)))
    for o in outs[1:]:
        np.testing.assert_array_equal(o['tab'], outs[0]['tab'])
    np.testing.assert_array_equal(np.isnan(outs[0]['tab']), np.isnan(single))
    np.testing.assert_allclose(outs[0]['tab'], single, rtol=1e-6, atol=1e-12)
    # genome-wide BH: every rank's slice = the single-process BH of its p
    allp = np.concatenate([o['p'] for o in outs])
    allq = oracle.adjust_pvalues(allp)
    off = 0
    for o in outs:
        np.testing.assert_array_equal(o['q'], allq[off:off + len(o['p'])])
        off += len(o['p'])


class _HostBhOps(object):
    """bh_sharded's per-rank pieces in numpy (the CPU stand-in for
    parallel.DeviceBhOps): the same sort / ratio / reverse-minimum
    arithmetic as h3d_bh_sort_dev / _scan_dev / _finish_dev."""

    def sort(self, keys, vals=None):
        import torch
        k = keys.numpy()
        key = np.where(np.isfinite(k), k, np.inf)
        o = np.argsort(key, kind='stable')
        v = np.arange(len(k)) if vals is None else vals.numpy()
        return (torch.from_numpy(key[o]), torch.from_numpy(v[o].astype(np.int64)),
                int(np.isfinite(k).sum()))

    def scan(self, ps, offset, m):
        import torch
        p = ps.numpy()
        j = np.arange(len(p), dtype=np.float64)
        ratio = p / ((offset + j + 1) / float(m))
        sc = np.minimum.accumulate(ratio[::-1])[::-1].copy()
        return torch.from_numpy(sc), (float(sc[0]) if len(sc) else np.inf)

    def finish(self, scanned, higher_min):
        import torch
        return torch.from_numpy(np.minimum(np.minimum(scanned.numpy(),
                                                      higher_min), 1.0))


def _bh_sharded_worker(rank, world, port, parts, result_file):
    import torch
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    q = parallel.bh_sharded(torch.from_numpy(parts[rank]), _HostBhOps(),
                            samples=8)
    np.save(result_file % rank, q.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_bh_sharded_equals_single_process(world):
    """parallel.bh_sharded (splitters from count-weighted samples, the
    all_to_all by value range, the bucket's global offset, the reverse
    minimum completed across buckets, the return all_to_all) gives every
    p-value the single-process BH's q bit for bit: ties (many across the
    splitters), NaN and +inf p-values, an all-NaN rank and a rank with a
    single p-value."""
    rng = np.random.default_rng(11)
    p = rng.uniform(0, 1, 4000) ** 4
    p[rng.integers(0, 4000, 900)] = 1.0          # a heavy tie at the top
    p[rng.integers(0, 4000, 300)] = 0.25          # and one in the middle
    p[rng.integers(0, 4000, 50)] = np.nan
    p[rng.integers(0, 4000, 5)] = np.inf
    sizes = [2500, 1, 1499] if world == 3 else [3999, 1]
    parts = np.split(p, np.cumsum(sizes)[:-1])
    if world == 3:
        parts[1] = np.array([np.nan])
    want = oracle.adjust_pvalues(np.concatenate(parts))
    with tempfile.TemporaryDirectory() as tmp:
        res = os.path.join(tmp, 'q%d.npy')
        port = 29300 + (os.getpid() % 1000) + world
        mp.spawn(_bh_sharded_worker, args=(world, port, parts, res),
                 nprocs=world, join=True)
        got = np.concatenate([np.load(res % r) for r in range(world)])
    np.testing.assert_array_equal(got, want)


def _exchange_worker(rank, world, port, result_file, idle=False):
    import torch
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    rng = np.random.default_rng(100 + rank)
    R = 4
    n = 0 if rank == world - 1 else int(rng.integers(1000, 5000))
    raw = torch.from_numpy(rng.integers(0, 1000, (n, R)).astype(np.int32))
    f = torch.from_numpy(rng.random((n, R)))
    d = torch.from_numpy(rng.integers(0, 60, n).astype(np.int32))
    owner = torch.from_numpy(
        rng.integers(0, world - int(idle), n).astype(np.int64))
    outs = []
    for chunks in (1, 3, 7):
        outs.append([t.numpy().copy() for t in parallel.exchange_by_owner(
            raw, f, d, owner, chunks=chunks)])
    np.savez(result_file % rank, *[a for o in outs for a in o])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world,idle', [(2, False), (3, False), (2, True),
                                        (3, True)])
def test_chunked_reshard_equals_one_shot(world, idle):
    """parallel.exchange_by_owner (the distance re-shard's all_to_all): cut
    into 3 or 7 asynchronous parts, every rank receives exactly what the
    one-shot exchange gives it, bit for bit -- and that is every source
    rank's pixels owned by this rank, source by source in their order (the
    last rank sends nothing; with ``idle`` it also owns nothing, so it has
    no pixel either way and must still take part in every part's
    collective)."""
    with tempfile.TemporaryDirectory() as tmp:
        res = os.path.join(tmp, 'x_%d.npz')
        port = 29900 + (os.getpid() % 1000) + world + 10 * int(idle)
        mp.spawn(_exchange_worker, args=(world, port, res, idle),
                 nprocs=world, join=True)
        srcs = []
        for r in range(world):
            rng = np.random.default_rng(100 + r)
            n = 0 if r == world - 1 else int(rng.integers(1000, 5000))
            raw = rng.integers(0, 1000, (n, 4)).astype(np.int32)
            f = rng.random((n, 4))
            d = rng.integers(0, 60, n).astype(np.int32)
            owner = rng.integers(0, world - int(idle), n)
            srcs.append((raw, f, d, owner))
        for r in range(world):
            z = np.load(res % r)
            got = [z['arr_%d' % i] for i in range(9)]
            want = [np.concatenate([s[j][s[3] == r] for s in srcs])
                    for j in range(3)]
            for c in range(3):
                for j in range(3):
                    np.testing.assert_array_equal(got[3 * c + j], want[j])


def _keys_for(kw, data, mine, R):
    """PixelKeys of this rank's chromosomes (genome index = position in
    CHROMS): row, chromosome, size-factor row (np.unique of the disp
    pixels' size-factor rows) and the (bias, size-factor rows) tables."""
    import torch
    names = list(CHROMS)
    rows, chroms, sfis, tables = [], [], [], {}
    for c in mine:
        prep, bias = data[c][0], data[c][1]
        di = prep['disp_idx']
        sf = prep['size_factors'][di]
        uniq, inv = np.unique(sf, axis=0, return_inverse=True)
        g = names.index(c)
        rows.append(prep['row'][di].astype(np.int32))
        chroms.append(np.full(int(di.sum()), g, dtype=np.int32))
        sfis.append(inv.reshape(-1).astype(np.int32))
        tables[g] = (bias, uniq)
    cat = (lambda a: torch.from_numpy(np.concatenate(a) if a else
                                      np.zeros(0, np.int32)))
    return parallel.PixelKeys(cat(rows), cat(chroms), cat(sfis), tables,
                              len(names))


def _compact_worker(rank, world, tmp, port, result_file):
    import torch
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    kw, data = _prep(os.path.join(tmp, 'r%d' % rank))
    mine = parallel.lpt_assign({c: len(data[c][2]) for c in CHROMS},
                               world)[rank]
    R = kw['design'].shape[0]
    raw = np.concatenate([data[c][2] for c in mine] or
                         [np.zeros((0, R), np.int32)])
    f = np.concatenate([data[c][3] for c in mine] or [np.zeros((0, R))])
    dist_ = np.concatenate([data[c][4] for c in mine] or
                           [np.zeros(0, np.int32)])
    t_raw = torch.from_numpy(np.ascontiguousarray(raw, np.int32))
    t_f = torch.from_numpy(np.ascontiguousarray(f))
    t_dist = torch.from_numpy(np.ascontiguousarray(dist_, np.int32))
    keys = _keys_for(kw, data, mine, R)
    owner = torch.from_numpy((dist_ * 7 % world).astype(np.int64))
    full = parallel.exchange_by_owner(t_raw, t_f, t_dist, owner, chunks=3)
    comp = parallel.exchange_compact(_HostCtx(), t_raw, t_dist, keys, owner,
                                     chunks=3)
    cond = kw['design'].argmax(axis=1).astype(np.int32)
    C = kw['design'].shape[1]
    tab_full = parallel.disp_per_dist_by_distance(
        _HostCtx(), t_raw, t_f, t_dist, cond, C, D)
    tab_comp = parallel.disp_per_dist_by_distance(
        _HostCtx(), t_raw, t_f, t_dist, cond, C, D, keys=keys)
    np.savez(result_file % rank, *[t.numpy() for t in full + comp],
             tab_full=tab_full, tab_comp=tab_comp)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_compact_reshard_equals_full_record(world):
    """The distance re-shard's compact exchange (parallel.exchange_compact:
    raw / row / dist / chromosome / size-factor row in their narrowest
    widths, f rebuilt on arrival from the stacked bias and size-factor
    tables) delivers raw, f and dist bit for bit as the full 52-byte record
    does, and disp_per_dist_by_distance gives the same table either way
    (world 3 > 2 chromosomes: one rank holds no chromosome)."""
    h3dbuild.build_hosttest()
    with tempfile.TemporaryDirectory() as tmp:
        res = os.path.join(tmp, 'c_%d.npz')
        port = 29300 + (os.getpid() % 1000) + world
        mp.spawn(_compact_worker, args=(world, tmp, port, res), nprocs=world,
                 join=True)
        for r in range(world):
            z = np.load(res % r)
            for j in range(3):
                a, b = z['arr_%d' % j], z['arr_%d' % (3 + j)]
                assert a.dtype == b.dtype and a.shape == b.shape
                np.testing.assert_array_equal(a, b)
            np.testing.assert_array_equal(z['tab_full'], z['tab_comp'])
    assert parallel.compact_record_bytes(4, 30000, 250, 20, 40) == 15
    assert parallel.compact_record_bytes(4, 1 << 20, 250, 20, 40) == 23
    assert parallel.compact_record_bytes(4, 30000, 400, 300, 40) == 17
