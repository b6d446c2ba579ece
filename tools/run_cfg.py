"""The hot path at the other north-star shapes (BASELINE.json configs /
SURVEY.md §8(d)) on one GPU, the way bench.py times cfg2: estimate_disp
(qcml per distance x condition + lowess table) + lrt on HBM-resident
inputs.

    cfg3: mouse genome at 10 kb -- 20 chromosomes, ~265k bins, R = 4 (2 + 2),
          dist_thresh_max 200, one genome-wide pooled estimate_disp
    cfg4: human chr1 at 5 kb -- 49,792 bins, R = 18 (6 + 6 + 6), C = 3,
          dist_thresh_max 400 (chi2 df = 2, k_lrt<32, 8>, the M = 8 disp path)

The pixels are drawn directly in the band (synthetic.draw_band: no files,
the SURVEY §8(d) generator's model with unit size factors). Prints one JSON
line.

    python tools/run_cfg.py --cfg 3 [--steps 3 --warmup 1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from hic3defdr_amd.synthetic import MM10_BINS  # noqa: E402

CFGS = {
    3: dict(chroms=MM10_BINS, npc=(2, 2), dmax=200),
    4: dict(chroms=[49792], npc=(6, 6, 6), dmax=400),
}


def draw(bins_list, npc, dmax, seed=0):
    from hic3defdr_amd import synthetic
    parts = []
    for i, n_bins in enumerate(bins_list):
        parts.append(synthetic.draw_band(n_bins, npc, dmax, seed=seed,
                                         chrom_index=i))
        print('  chrom of %d bins: %d disp px' % (n_bins, len(parts[-1][0])),
              file=sys.stderr, flush=True)
    cond = np.repeat(np.arange(len(npc)), npc).astype(np.int32)
    return (np.concatenate([p[0] for p in parts]),
            np.concatenate([p[1] for p in parts]),
            np.concatenate([p[2] for p in parts]), cond)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cfg', type=int, choices=sorted(CFGS), required=True)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    args = ap.parse_args()
    cfg = CFGS[args.cfg]
    t0 = time.time()
    raw, f, dist, cond = draw(cfg['chroms'], cfg['npc'], cfg['dmax'])
    gen_s = time.time() - t0
    import torch
    from hic3defdr_amd import _native
    torch.cuda.set_device(0)
    ctx = _native.context(0)
    dev = torch.device('cuda', 0)
    n, R = raw.shape
    C = len(cfg['npc'])
    D = cfg['dmax'] + 1
    t_raw = torch.from_numpy(raw).to(dev)
    t_f = torch.from_numpy(f).to(dev)
    t_d = torch.from_numpy(dist).to(dev)
    t_p = torch.empty(n, dtype=torch.float64, device=dev)
    t_llr, t_m0 = torch.empty_like(t_p), torch.empty_like(t_p)
    t_m1 = torch.empty((n, C), dtype=torch.float64, device=dev)
    t_disp = torch.empty_like(t_m1)
    torch.cuda.synchronize()   # the uploads ran on the default stream
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    from bench import table_lrt   # the bench step's table -> LRT
    tl = table_lrt(torch, dev, ctx, D, C)
    o = {'p': t_p, 'llr': t_llr, 'mu0': t_m0, 'mu1': t_m1, 'disp': t_disp}

    def step():
        dpd = tl.estimate(t_raw, t_f, t_d, n, R, cond)
        tl(dpd, t_raw, t_f, t_d, n, R, cond, o)
        return dpd

    first = None
    for _ in range(args.warmup):
        first = step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dpd = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ctx.profile_reset()
    ctx.profile(True, level=2)
    step()
    torch.cuda.synchronize()
    ctx.profile(False)
    ks = {k: ctx.profile_read(k)[0] for k in
          ('disp_work', 'disp_nll', 'disp_update', 'disp_prep', 'lrt')}
    p = t_p.cpu().numpy()
    present = np.isin(np.arange(D), dist)
    out = {
        'config': 'cfg%d' % args.cfg, 'bins': int(sum(cfg['chroms'])),
        'chroms': len(cfg['chroms']), 'reps': R, 'conds': C,
        'dist_thresh_max': cfg['dmax'], 'disp_pixels': int(n),
        'value': n * args.steps / el, 'unit': 'pixels/s',
        'ms_per_step': el / args.steps * 1e3, 'steps': args.steps,
        'kernels_ms_per_step': ks,
        'checks': {
            'disp_finite_where_present': bool(np.all(np.isfinite(
                dpd[present]))),
            'disp_nan_where_absent': bool(np.all(np.isnan(dpd[~present]))),
            'p_in_0_1': bool(np.all((p >= 0) & (p <= 1))),
            'deterministic_disp': None if first is None else bool(
                np.array_equal(first, dpd, equal_nan=True)),
            'frac_p_lt_0.05': float(np.mean(p < 0.05))},
        'generate_s': gen_s,
    }
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
