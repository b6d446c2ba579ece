"""Benchmark: pixels/sec through estimate_disp + lrt (BASELINE.json metric).

Workload (BASELINE.json configs[1], "cfg2"): per GPU one synthetic
chromosome of 20,000 bins, 4 replicates (2 + 2 conditions), dist_thresh_max
250 (SURVEY.md §8(d) generator, seed = rank). Untimed setup: generate the
input files, run the product's GPU prepare_data, upload raw / f / dist of the
disp pixels to HBM. One step = estimate_disp (qcml per distance x condition,
lowess smoothing table) + lrt (fused per-pixel GLM fits + LRT) on the
resident inputs, outputs left in HBM.

N > 1 (torchrun, one rank per GPU over RCCL): weak scaling — every rank owns
its own chromosome; the genome-wide per-distance pooling of estimate_disp is
kept by an all-reduce of the per-segment NLL sums each data pass.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

METRIC = ("pixels/sec through estimate_disp+lrt, 4 reps @10kb; "
          "max-|Δq| vs reference")


PMC_SUMMARY = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                           'profiles', 'pmc_traffic_default.json')


def pmc_traffic(kernel, bins, dmax):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (tools/pmc_passes.sh over this same default command: FETCH_SIZE x2
    gfx950 correction + WRITE_SIZE, each its own rocprofv3 pass).  Counters
    cannot be read inside the timed run, so the figure comes from that
    profile; None unless the workload is the one it was measured on."""
    try:
        d = json.load(open(PMC_SUMMARY))
    except (OSError, ValueError):
        return None
    if d.get('bins') != bins or d.get('dmax') != dmax:
        return None
    rd = wr = 0.0
    n = 0
    for key, e in d['kernels'].items():
        if kernel in key.split('[')[0]:
            rd += e.get('hbm_read_bytes_corrected', 0.0)
            wr += e.get('hbm_write_bytes', 0.0)
            n += e['dispatches']
    return (rd + wr) / n if n else None


def bytes_per_lrt_pixel(R, C):
    # raw int32 4R + f 8R + dist 4 in; p, llr, mu0 24 + mu1 8C + disp 8C out
    return 12 * R + 16 * C + 28


def make_workload(tmp, name, bins, dmax, seed):
    import pandas as pd
    from hic3defdr_amd import HiC3DeFDR, synthetic
    kw = synthetic.write_dataset(tmp, {name: bins}, dist_thresh_max=dmax,
                                 seed=seed)
    design = pd.DataFrame(kw['design'], index=kw['reps'], columns=kw['conds'])
    h = HiC3DeFDR(raw_npz_patterns=kw['raw_npz_patterns'],
                  bias_patterns=kw['bias_patterns'], chroms=kw['chroms'],
                  design=design, outdir=os.path.join(tmp, 'out'),
                  dist_thresh_max=dmax)
    return h, kw


def cpu_baseline(ctx, bins, dmax, seed=123):
    """The oracle (numpy/scipy restatement, fallback-fixed brentq) timed on a
    bounded sample of the same workload, 1 core; plus the GPU on the same
    sample for a parity figure."""
    import oracle
    from hic3defdr_amd import synthetic, _native
    tmp = tempfile.mkdtemp(prefix='h3dbench_cpu_')
    try:
        kw = synthetic.write_dataset(tmp, {'chrS': bins}, dist_thresh_max=dmax,
                                     seed=seed)
        design = kw['design']
        npz = [p.replace('<chrom>', 'chrS') for p in kw['raw_npz_patterns']]
        bfs = [p.replace('<chrom>', 'chrS') for p in kw['bias_patterns']]
        prep = oracle.prepare_chrom(npz, bfs, design, dist_thresh_max=dmax)
        bias = oracle.load_bias(bfs)
        di = prep['disp_idx']
        row, col = prep['row'][di], prep['col'][di]
        raw = prep['raw'][di]
        f = bias[row] * bias[col] * prep['size_factors'][di]
        t0 = time.time()
        disp, dpd, _ = oracle.estimate_disp([prep], [bias], design,
                                            dist_thresh_max=dmax)
        rp, _, _, _ = oracle.lrt(raw, f, np.dot(disp, design.T), design)
        dt = time.time() - t0
        n = len(raw)
        # GPU on the same sample
        cond = design.argmax(axis=1)
        C = design.shape[1]
        out = ctx.disp_per_dist(raw, f, col - row, cond, C, dmax + 1)
        tab = np.stack([_native.disp_table(out[:, c]) for c in range(C)], 1)
        p, _, _, _, _ = ctx.lrt(raw, f, col - row, tab, cond)
        qg = _native.bh(p)
        qo = oracle.adjust_pvalues(rp)
        with np.errstate(all='ignore'):
            dp = np.nanmax(np.abs(p - rp) / np.maximum(rp, 1e-300))
            dq = np.nanmax(np.abs(qg - qo))
        return {'value': n / dt, 'unit': 'pixels/s', 'cores': 1,
                'kind': 'port',
                'sample': 'oracle estimate_disp+lrt (numpy/scipy, brentq '
                          'fallback per failed pixel) on 1 synthetic chrom '
                          'of %d bins, dmax %d, 4 reps: %d disp pixels in '
                          '%.1f s' % (bins, dmax, n, dt)}, \
            {'sample_pixels': n, 'max_rel_dp_vs_oracle': float(dp),
             'max_abs_dq_vs_oracle': float(dq),
             'identical_calls_q<0.05': bool(np.array_equal(qg < 0.05,
                                                             qo < 0.05))}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--bins', type=int, default=20000)
    ap.add_argument('--dmax', type=int, default=250)
    ap.add_argument('--cpu-bins', type=int, default=1000)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    from hic3defdr_amd import _native, parallel
    ctx = _native.context(local)
    tmp = tempfile.mkdtemp(prefix='h3dbench_r%d_' % rank)
    try:
        h, kw = make_workload(tmp, 'chrB%d' % rank, args.bins, args.dmax, rank)
        h.prepare_data(verbose=False)
        raw, f, dist_np, _ = h._f_and_dist()
        design = kw['design']
        R, C = design.shape
        D = args.dmax + 1
        cond = design.argmax(axis=1).astype(np.int32)
        n = len(raw)
        dev = torch.device('cuda', local)
        t_raw = torch.from_numpy(raw.astype(np.int32)).to(dev).contiguous()
        t_f = torch.from_numpy(f).to(dev).contiguous()
        t_dist = torch.from_numpy(dist_np.astype(np.int32)).to(dev)
        t_p = torch.empty(n, dtype=torch.float64, device=dev)
        t_llr = torch.empty_like(t_p)
        t_mu0 = torch.empty_like(t_p)
        t_mu1 = torch.empty((n, C), dtype=torch.float64, device=dev)
        t_disp = torch.empty_like(t_mu1)
        torch.cuda.synchronize()
        ctx.set_stream(torch.cuda.current_stream().cuda_stream)
        reduce = parallel.make_allreduce() if world > 1 else None

        def step():
            dpd = ctx.disp_per_dist_dev(t_raw.data_ptr(), t_f.data_ptr(),
                                        t_dist.data_ptr(), n, R, cond, C, D,
                                        reduce=reduce)
            tab = _native.disp_tables(dpd)
            ctx.lrt_dev(t_raw.data_ptr(), t_f.data_ptr(), t_dist.data_ptr(),
                        tab, n, R, cond, t_p.data_ptr(), t_llr.data_ptr(),
                        t_mu0.data_ptr(), t_mu1.data_ptr(), t_disp.data_ptr())
            return dpd

        for _ in range(args.warmup):
            step()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        # timed region: HIP events around the roofline kernels only
        ctx.profile_reset()
        ctx.profile(True, level=1)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        ctx.profile(False)
        w_ms, w_n, w_bytes = ctx.profile_read('disp_work')
        l_ms, l_n, l_px = ctx.profile_read('lrt')
        # one more (untimed) step with every kernel scope timed, for the
        # per-kernel breakdown
        ctx.profile_reset()
        ctx.profile(True, level=2)
        step()
        torch.cuda.synchronize()
        ctx.profile(False)
        r_ms, r_n, _ = ctx.profile_read('disp_reduce')
        u_ms, u_n, _ = ctx.profile_read('disp_update')
        n_ms, n_n, n_bytes = ctx.profile_read('disp_nll')
        p_ms, p_n, _ = ctx.profile_read('disp_prep')
        b_ms, _, _ = ctx.profile_read('disp_work')
        b_lrt, _, _ = ctx.profile_read('lrt')
        tot_px = n
        if dist:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            t = torch.tensor([n], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            tot_px = int(t.item())
        value = tot_px * args.steps / elapsed
        if rank == 0:
            peak = 8000.0
            w_avg_s = (w_ms / max(w_n, 1)) / 1e3
            w_ach = (w_bytes / max(w_n, 1)) / w_avg_s / 1e9 if w_avg_s else 0.0
            l_avg_s = (l_ms / max(l_n, 1)) / 1e3
            l_ach = (n * bytes_per_lrt_pixel(R, C)) / l_avg_s / 1e9 \
                if l_avg_s else 0.0
            out = {
                'metric': METRIC, 'value': value, 'unit': 'pixels/s',
                'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
                'ms_per_step': elapsed / args.steps * 1e3,
                'higher_is_better': True, 'scaling': 'weak',
                'vs_baseline': None, 'dtype': 'f64',
                'data': 'synthetic (SURVEY.md 8(d) generator; no demo data '
                        'offline)',
                'config': {
                    'workload': 'cfg2: per GPU 1 chrom x %d bins, 4 reps '
                                '(2+2), dist_thresh_max %d, estimate_disp '
                                '(qcml) + lrt on HBM-resident inputs'
                                % (args.bins, args.dmax),
                    'disp_pixels_per_gpu': n, 'disp_pixels_total': tot_px,
                    'parallelism': 'dp%d (chromosome shards, per-pass '
                                   'NLL all-reduce)' % world},
                'roofline': {
                    'bound': 'hbm', 'kernel': 'k_disp_work',
                    'achieved': w_ach, 'peak': peak, 'unit': 'GB/s',
                    'frac': w_ach / peak,
                    # equalize instantiation <M=4, W=4, kEqualize>
                    'traffic': pmc_traffic('k_disp_work<4, 4, 0>', args.bins,
                                           args.dmax),
                    'traffic_source': 'profiles/pmc_traffic_default.json '
                                      '(HBM bytes per launch)',
                    'bytes_per_launch': w_bytes / max(w_n, 1),
                    'avg_launch_us': w_avg_s * 1e6, 'launches': w_n,
                    'note': 'FP64-VALU/transcendental bound (SURVEY.md '
                            'finding 3); bytes = 20 B per equalize '
                            'pixel-replicate (raw 4 + f 8 in, pseudodata 8 '
                            'out)'},
                'kernels_ms_per_step': {
                    'note': 'one extra untimed step, every kernel timed',
                    'disp_work': b_ms,
                    'disp_reduce': r_ms,
                    'disp_update': u_ms,
                    'disp_nll': n_ms,
                    'disp_prep': p_ms,
                    'lrt': b_lrt},
                'work_per_step': {
                    'equalize_pixel_reps': w_bytes / 20.0 / args.steps,
                    'nll_pixel_reps': n_bytes / 8.0,
                    'disp_launches': w_n / args.steps},
                'nll_roofline': {
                    'achieved': n_bytes / (n_ms / 1e3) / 1e9 if n_ms else 0.0,
                    'peak': peak, 'unit': 'GB/s',
                    'frac': n_bytes / (n_ms / 1e3) / 1e9 / peak if n_ms
                    else 0.0,
                    'bytes_per_pixel_rep': 8,
                    'avg_launch_us': n_ms / max(n_n, 1) * 1e3},
                'lrt_roofline': {'achieved': l_ach, 'peak': peak,
                                 'unit': 'GB/s', 'frac': l_ach / peak,
                                 'bytes_per_pixel': bytes_per_lrt_pixel(R, C),
                                 'avg_launch_us': l_avg_s * 1e6},
            }
            if world == 1 and not args.no_cpu_baseline:
                cb, par = cpu_baseline(ctx, args.cpu_bins, args.dmax)
                out['cpu_baseline'] = cb
                out['parity_sample'] = par
            print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
        if dist:
            dist.destroy_process_group()


if __name__ == '__main__':
    main()
