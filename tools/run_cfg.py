"""The hot path at the other north-star shapes (BASELINE.json configs /
SURVEY.md §8(d)) on one GPU, the way bench.py times cfg2: estimate_disp
(qcml per distance x condition + lowess table) + lrt on HBM-resident
inputs.

    cfg3: mouse genome at 10 kb -- 20 chromosomes, ~265k bins, R = 4 (2 + 2),
          dist_thresh_max 200, one genome-wide pooled estimate_disp
    cfg4: human chr1 at 5 kb -- 49,792 bins, R = 18 (6 + 6 + 6), C = 3,
          dist_thresh_max 400 (chi2 df = 2, k_lrt<32, 8>, the M = 8 disp path)

The pixels are drawn directly in the band (synthetic.draw_band: no files,
the SURVEY §8(d) generator's model with unit size factors); the step is
bench.py's (other_config, which the default bench also runs after the
headline). Prints one JSON line.

    python tools/run_cfg.py --cfg 3 [--steps 3 --warmup 1]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cfg', type=int, choices=(3, 4), required=True)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    args = ap.parse_args()
    import torch
    from bench import other_config
    from hic3defdr_amd import _native
    torch.cuda.set_device(0)
    ctx = _native.context(0)
    out = other_config(torch, ctx, torch.device('cuda', 0),
                       'cfg%d' % args.cfg, steps=args.steps,
                       warmup=args.warmup)
    out['config'] = 'cfg%d' % args.cfg
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
