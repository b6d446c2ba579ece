"""torchrun worker for tests/test_gpu_multirank.py::test_bh_sharded_gpu:
parallel.bh_sharded with DeviceBhOps (h3d_bh_sort_dev / _scan_dev /
_finish_dev) on every rank's slice of one seeded p-value vector, every rank
on the GPU H3D_DEVICE names, backend gloo (several ranks on one GPU). Rank
0 gathers the q-values and checks them against h3d_bh_dev on the whole
vector, bit for bit.

    torchrun --nproc-per-node 3 tests/dist_bh_main.py <n>
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    from hic3defdr_amd import _native, parallel
    n = int(sys.argv[1])
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device('cuda', int(os.environ.get('H3D_DEVICE', '0')))
    torch.cuda.set_device(dev)
    rng = np.random.default_rng(7)
    p = rng.uniform(0, 1, n) ** 3
    p[rng.integers(0, n, n // 5)] = 1.0
    p[rng.integers(0, n, n // 50)] = np.nan
    p[rng.integers(0, n, n // 20)] = p[rng.integers(0, n, n // 20)]  # ties
    cuts = np.sort(rng.integers(0, n, world - 1))
    parts = np.split(p, cuts)
    ctx = _native.context(dev.index)
    t = torch.from_numpy(parts[rank]).to(dev)
    q = parallel.bh_sharded(t, parallel.DeviceBhOps(ctx))
    qs, _ = parallel.gather_all(q.cpu())
    if rank == 0:
        tp = torch.from_numpy(p).to(dev)
        want = torch.empty_like(tp)
        ctx.bh_dev(tp.data_ptr(), n, want.data_ptr())
        torch.cuda.synchronize()
        w, g = want.cpu().numpy(), qs.numpy()
        same = np.array_equal(w, g, equal_nan=True)
        print('bh_sharded n=%d world=%d bit-identical=%s' % (n, world, same),
              flush=True)
        if not same:
            bad = np.flatnonzero(~((w == g) | (np.isnan(w) & np.isnan(g))))
            print('first differences', bad[:10], w[bad[:10]], g[bad[:10]],
                  flush=True)
            sys.exit(1)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
