"""Every rank's share of an N-GPU cfg3 run (BASELINE configs[2]: the mm10
genome at 10 kb, R = 4, dmax 200), timed one after another on ONE GPU: the
step time of an N-GPU run is the max over its ranks (bench.py takes the max
over ranks), so all ranks are emulated, not rank 0 alone.

A rank's share (parallel.disp_per_dist_by_distance + lrt of its chromosomes
+ its part of the sharded BH): estimate_disp over the distances the owner
table gives it (what it holds after the all_to_all), the smoothed tables,
lrt over the chromosomes LPT gives it, BH over its own p-values. The
collectives themselves are not run (no second GPU): their time is modelled
from the actual routing's bytes per (source, destination) pair at a stated
xGMI link bandwidth and efficiency plus a per-collective latency, and the
N-GPU step projected with them (serially, no overlap credited). Owner tables compared: LPT on pixel counts (round 3) and LPT on the
per-distance work measured in a first whole-genome pass (qcml iterations x
pixels equalized + Brent evaluations x pixels, weighted by the measured cost
of one pixel-replicate of each, h3d_disp_seg_stats) and on the a-priori
model parallel.distance_cost.

    python tools/emulate_ranks.py [--worlds 2,4,8] [--steps 3]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def collectives(parts, assign, counts, N, D, C, rec_bytes, max_ms, ms1,
                args):
    """The collectives of one N-GPU cfg3 step (not run: one GPU), from the
    actual pixel routing: rank r holds the disp pixels of its LPT
    chromosomes and sends each to the owner of its distance (``rec_bytes``
    per pixel: parallel.compact_record_bytes, or 12 R + 4 for the full
    record); BH sends each p-value to its value-range bucket's rank and the q
    back (8 B each way, ~1/N of a rank's values per peer); the D x C table
    all-reduce and the small all_gathers / count all-reduces are latency
    only. On the full xGMI mesh every (source, destination) pair has its own
    link, so an all_to_all takes about the largest pair's bytes / the link
    bandwidth. Added serially (no overlap credited) to ``max_ms``, the
    slowest rank's measured kernel share."""
    from hic3defdr_amd import parallel
    owner = parallel.distance_owners(counts, N)
    pair = np.zeros((N, N))
    for r in range(N):
        dr = np.concatenate([parts[i][2] for i in assign[r]]) \
            if assign[r] else np.zeros(0, dtype=np.int64)
        pair[r] = np.bincount(owner[dr], minlength=N)[:N] * rec_bytes
    np.fill_diagonal(pair, 0)
    n_r = [sum(len(parts[i][2]) for i in assign[r]) for r in range(N)]
    bh_pair = max(n_r) * 8.0 / N       # ~1/N of a rank's values per peer
    bw = args.link_gbs * 1e9 * args.link_eff
    t_pix = pair.max() / bw * 1e3
    t_bh = 2 * bh_pair / bw * 1e3
    # counts all-reduce, the record-width max all-reduce, 2 exchange
    # all_to_alls (sizes + records), table all-reduce, BH: 3 all_gathers +
    # 2 all_to_alls
    n_coll = 10
    t_lat = n_coll * args.latency_us * 1e-3
    proj = max_ms + t_pix + t_bh + t_lat
    print('N=%d, %d-byte records: projected %.2f ms (kernels %.2f, pixel '
          'all_to_all %.2f, BH %.2f, latency %.2f) -> %.2fx (%.1f%%)' % (
              N, rec_bytes, proj, max_ms, t_pix, t_bh, t_lat, ms1 / proj,
              100 * ms1 / proj / N), flush=True)
    return {'record_bytes': rec_bytes,
            'pixel_all_to_all_max_pair_bytes': float(pair.max()),
            'pixel_all_to_all_bytes_out_per_rank_max': float(pair.sum(1).max()),
            'bh_all_to_all_pair_bytes': float(bh_pair),
            'table_allreduce_bytes': 8 * D * C,
            'assumed': {'link_GBps_per_direction': args.link_gbs,
                        'efficiency': args.link_eff,
                        'latency_us_per_collective': args.latency_us,
                        'collectives_per_step': n_coll},
            'ms': {'kernels_slowest_rank': max_ms, 'pixel_all_to_all': t_pix,
                   'bh_all_to_alls': t_bh, 'latency': t_lat},
            'projected_step_ms_pixels_owners': proj,
            'projected_speedup_vs_n1': ms1 / proj,
            'projected_efficiency': ms1 / proj / N}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--worlds', default='2,4,8')
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--dmax', type=int, default=200)
    ap.add_argument('--out', default=os.path.join(REPO, 'gpurun_out',
                                                  'emulate_ranks.json'))
    # xGMI: 7 links per MI355X, ~153 GB/s each (both directions), i.e.
    # ~76 GB/s per direction; RCCL's all_to_all reaches a fraction of it
    ap.add_argument('--link-gbs', type=float, default=76.5)
    ap.add_argument('--link-eff', type=float, default=0.6)
    ap.add_argument('--latency-us', type=float, default=30.0)
    ap.add_argument('--from', dest='from_json', default=None,
                    help='no GPU: take the measured kernel shares (N = 1 and '
                         'each world\'s slowest rank, pixel-count owners) '
                         'from an earlier run\'s JSON and project the '
                         'collectives for both re-shard records')
    args = ap.parse_args()
    from hic3defdr_amd import parallel, synthetic
    bins = synthetic.MM10_BINS
    D = args.dmax + 1
    R, C = 4, 2
    cond = np.array([0, 0, 1, 1], dtype=np.int32)
    t0 = time.perf_counter()
    parts = synthetic.draw_genome(bins, (2, 2), args.dmax, seed=0, workers=16)
    print('drew the genome in %.1f s' % (time.perf_counter() - t0), flush=True)
    d_all = np.concatenate([p[2] for p in parts])
    counts = np.bincount(d_all, minlength=D)[:D]
    # the re-shard's record: the compact one (parallel.exchange_compact:
    # raw / row / dist / chromosome / size-factor row at their narrowest
    # widths; the genome's unit size factors are one row) and the full one
    rec = {'compact': parallel.compact_record_bytes(
               R, int(max(p[0].max() for p in parts)), args.dmax, len(bins),
               1),
           'full': 12 * R + 4}
    if args.from_json:
        prev = json.load(open(args.from_json))
        ms1 = prev['n1']['ms']
        out = {'from': args.from_json, 'n1_ms': ms1, 'record_bytes': rec,
               'worlds': {}}
        for N in [int(v) for v in args.worlds.split(',')]:
            assign = parallel.lpt_assign({i: b for i, b in enumerate(bins)},
                                         N)
            mx = prev['worlds'][str(N)]['pixels']['max_ms']
            out['worlds'][str(N)] = {
                kind: collectives(parts, assign, counts, N, D, C, rb, mx, ms1,
                                  args)
                for kind, rb in rec.items()}
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, 'w') as fh:
            json.dump(out, fh, indent=1)
        return
    import torch
    from hic3defdr_amd import _native
    ctx = _native.context(0)
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    def up(raw, f, dist):
        return (torch.from_numpy(np.ascontiguousarray(raw, dtype=np.int32)).to(dev),
                torch.from_numpy(np.ascontiguousarray(f)).to(dev),
                torch.from_numpy(np.ascontiguousarray(dist, dtype=np.int32)).to(dev))

    def fill_table(dpd):
        # the other ranks' rows (not run here), interpolated with a ripple so
        # the smoother sees a table of the usual shape (bench.py's emulation)
        dpd = dpd.copy()
        for c in range(C):
            fin = np.isfinite(dpd[:, c])
            gap = ~fin & (np.arange(D) >= 4)
            gi = np.flatnonzero(gap)
            if fin.sum() >= 2 and gi.size:
                dpd[gap, c] = np.interp(gi, np.flatnonzero(fin), dpd[fin, c]) \
                    * (1 + 0.02 * np.sin(1.7 * gi + c))
        return dpd

    def time_share(d_sel, chroms, steps):
        """ms per step of one rank's share: estimate_disp on the pixels whose
        distance it owns, tables, lrt + BH on its chromosomes."""
        keep = d_sel[d_all]
        e = up(np.concatenate([p[0] for p in parts])[keep],
               np.concatenate([p[1] for p in parts])[keep], d_all[keep])
        own = [parts[i] for i in chroms]
        lr = up(np.concatenate([p[0] for p in own]),
                np.concatenate([p[1] for p in own]),
                np.concatenate([p[2] for p in own])) if own else None
        n_e, n_l = int(e[0].shape[0]), int(lr[0].shape[0]) if own else 0
        t_tab = torch.empty((D, C), dtype=torch.float64, device=dev)
        t_dpd = torch.empty((D, C), dtype=torch.float64, device=dev)
        o = torch.empty((3 + C, max(n_l, 1)), dtype=torch.float64, device=dev)
        q = torch.empty(max(n_l, 1), dtype=torch.float64, device=dev)
        torch.cuda.synchronize()

        def step():
            dpd = ctx.disp_per_dist_dev(e[0].data_ptr(), e[1].data_ptr(),
                                        e[2].data_ptr(), n_e, R, cond, C, D) \
                if n_e else np.full((D, C), np.nan)
            t_dpd.copy_(torch.from_numpy(fill_table(dpd)))
            ctx.disp_tables_dev(t_dpd.data_ptr(), D, C, t_tab.data_ptr())
            if n_l:
                ctx.lrt_dev_tab(lr[0].data_ptr(), lr[1].data_ptr(),
                                lr[2].data_ptr(), t_tab.data_ptr(), D, n_l, R,
                                cond, o[0].data_ptr(), o[1].data_ptr(),
                                o[2].data_ptr(), o[3].data_ptr())
                ctx.bh_dev(o[0].data_ptr(), n_l, q.data_ptr())
            else:
                ctx.disp_tables_wait()
        step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / steps * 1e3
        stats = ctx.disp_seg_stats(D, C) if n_e else None
        return ms, n_e, n_l, stats

    # N = 1: the whole genome, and the measured per-segment work
    all_d = np.ones(D, dtype=bool)
    ms1, n1, _, (qi, ev) = time_share(all_d, list(range(len(bins))),
                                      args.steps)
    ctx.profile_reset()
    ctx.profile(True, level=2)
    time_share(all_d, [], 1)
    ctx.profile(False)
    eq_ms, _, eq_b = ctx.profile_read('disp_work')
    nl_ms, _, nl_b = ctx.profile_read('disp_nll')
    # seconds per pixel-replicate: an equalize pass / one NLL evaluation
    k_eq = eq_ms / max(eq_b / 20.0, 1)
    k_nl = nl_ms / max(nl_b / 8.0, 1)
    work = (counts[:, None] * (qi * k_eq + ev * k_nl) * 2).sum(axis=1)
    model = parallel.distance_cost(counts,
                                   np.bincount(d_all, weights=np.concatenate(
                                       [p[0].sum(axis=1) for p in parts]),
                                       minlength=D)[:D], R)
    out = {'n1': {'ms': ms1, 'pixels': n1},
           'per_pixel_rep_ms': {'equalize': k_eq, 'nll_eval': k_nl},
           'seg_stats': {'qcml_iters_mean': float(qi[counts > 0].mean()),
                         'evals_mean': float(ev[counts > 0].mean())},
           'per_distance': {'pixels': counts.tolist(),
                            'measured_work_ms': work.tolist(),
                            'model': model.tolist(),
                            'qcml_iters': qi.tolist(), 'evals': ev.tolist()},
           'worlds': {}}
    print('N=1: %.2f ms/step over %d px; per pixel-rep equalize %.3g ms, NLL '
          'eval %.3g ms' % (ms1, n1, k_eq, k_nl), flush=True)
    assign_all = {}
    for N in [int(v) for v in args.worlds.split(',')]:
        assign = parallel.lpt_assign({i: b for i, b in enumerate(bins)}, N)
        assign_all[N] = assign
        res = {}
        for name, weight in (('pixels', counts), ('measured', work),
                             ('model', model)):
            owner = parallel.distance_owners(weight, N)
            ranks = []
            for r in range(N):
                ms, ne, nl, _ = time_share(owner == r, sorted(assign[r]),
                                           args.steps)
                ranks.append({'rank': r, 'ms': ms, 'disp_pixels': ne,
                              'lrt_pixels': nl})
                print('N=%d owners=%s rank %d: %.2f ms (%d disp px, %d lrt px)'
                      % (N, name, r, ms, ne, nl), flush=True)
            mx = max(x['ms'] for x in ranks)
            res[name] = {'ranks': ranks, 'max_ms': mx,
                         'speedup_vs_n1': ms1 / mx}
            print('N=%d owners=%s: max %.2f ms -> %.2fx of N=1 (%.1f%% '
                  'efficiency)' % (N, name, mx, ms1 / mx, 100 * ms1 / mx / N),
                  flush=True)
        best = min(res[k]['max_ms'] for k in ('pixels', 'measured', 'model'))
        res['collectives'] = collectives(parts, assign, counts, N, D, C,
                                         rec['compact'],
                                         res['pixels']['max_ms'], ms1, args)
        res['collectives']['best_owner_table_max_ms'] = best
        res['collectives_full_record'] = collectives(
            parts, assign, counts, N, D, C, rec['full'],
            res['pixels']['max_ms'], ms1, args)
        out['worlds'][str(N)] = res
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, 'w') as fh:
        json.dump(out, fh, indent=1)


if __name__ == '__main__':
    main()
