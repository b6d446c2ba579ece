"""Repeatability of estimate_disp on one input: N calls, which segments
differ and by how much (tools/run_cfg.py shapes).
    python tools/determinism.py --cfg 4 [--calls 4]"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tools'))


def main():
    import run_cfg
    ap = argparse.ArgumentParser()
    ap.add_argument('--cfg', type=int, default=4)
    ap.add_argument('--calls', type=int, default=4)
    ap.add_argument('--bins', type=int, default=0)
    args = ap.parse_args()
    cfg = dict(run_cfg.CFGS[args.cfg])
    if args.bins:
        cfg['chroms'] = [args.bins]
    raw, f, dist, cond = run_cfg.draw(cfg['chroms'], cfg['npc'], cfg['dmax'])
    from hic3defdr_amd import _native
    ctx = _native.context(0)
    C, D = len(cfg['npc']), cfg['dmax'] + 1
    outs = [ctx.disp_per_dist(raw, f, dist, cond, C, D) for _ in range(args.calls)]
    for i in range(1, args.calls):
        a, b = outs[0], outs[i]
        diff = ~((a == b) | (np.isnan(a) & np.isnan(b)))
        idx = np.argwhere(diff)
        rel = np.abs(a - b)[diff] / np.abs(a[diff]) if diff.any() else []
        print('call 0 vs %d: %d segments differ, max rel %s, first %s' %
              (i, diff.sum(), np.max(rel) if len(rel) else 0, idx[:5].tolist()),
              flush=True)


if __name__ == '__main__':
    main()
