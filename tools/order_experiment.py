"""Which pixel order inside a distance segment minimises the equalize pass's
wave divergence? CPU-only experiment on the q2q_stats census (the work of
every pixel-replicate does not depend on the order, so one census is
re-evaluated under several within-segment orders with the wave cost model of
tools/q2q_stats.py).

    python tools/order_experiment.py [--bins 1500] [--dmax 250]
"""
import argparse
import ctypes
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import q2q_stats  # noqa: E402


def model(rec, fit, w=64, it_cost=18.0, call_cost=250.0, fit_cost=60.0):
    nw = len(rec) // w
    nr = rec.shape[1]
    rec = rec[:nw * w].reshape(nw, w, nr, 11)
    fit = fit[:nw * w].reshape(nw, w)
    ncall = rec[..., 0]
    its = rec[..., 1::2]
    paths = rec[..., 2::2]
    made = np.arange(5)[None, None, None, :] < ncall[..., None]
    itm = np.where(made, its, 0)
    cf = np.where(made & (paths == 0), itm, 0)
    se = np.where(made & (paths != 0), itm, 0)
    act = ((cf.max(1) + se.max(1)).sum(axis=(1, 2)) * it_cost +
           made.any(1).sum(axis=(1, 2)) * call_cost + fit.max(1) * fit_cost)
    ideal = (itm.sum(axis=(1, 2, 3)) / w * it_cost +
             made.sum(axis=(1, 2, 3)) / w * call_cost + fit.mean(1) * fit_cost)
    return act.sum(), ideal.sum()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--bins', type=int, default=1500)
    ap.add_argument('--dmax', type=int, default=250)
    args = ap.parse_args()
    import oracle
    from hic3defdr_amd import synthetic
    lib = q2q_stats.build()
    tmp = tempfile.mkdtemp(prefix='q2qo_')
    kw = synthetic.write_dataset(tmp, {'chrS': args.bins},
                                 dist_thresh_max=args.dmax, seed=123)
    design = kw['design']
    npz = [p.replace('<chrom>', 'chrS') for p in kw['raw_npz_patterns']]
    bfs = [p.replace('<chrom>', 'chrS') for p in kw['bias_patterns']]
    prep = oracle.prepare_chrom(npz, bfs, design, dist_thresh_max=args.dmax)
    bias = oracle.load_bias(bfs)
    di = prep['disp_idx']
    row, col = prep['row'][di], prep['col'][di]
    raw = np.ascontiguousarray(prep['raw'][di], dtype=np.int32)
    f = np.ascontiguousarray(bias[row] * bias[col] * prep['size_factors'][di])
    dist = col - row
    _, dpd, _ = oracle.estimate_disp([prep], [bias], design,
                                     dist_thresh_max=args.dmax)
    n, R = raw.shape
    cond = design.argmax(axis=1)
    P = ctypes.c_void_p
    lib.q2qs_wave_log.argtypes = [ctypes.c_int64, ctypes.c_int, P, P, P,
                                  ctypes.c_int, P, P, P]
    tot = {}
    for c in range(design.shape[1]):
        reps = np.flatnonzero(cond == c).astype(np.int32)
        nr = len(reps)
        alpha = np.ascontiguousarray(dpd[dist, c])
        rec = np.zeros((n, nr, 11))
        fit = np.zeros(n)
        lib.q2qs_wave_log(n, R, raw.ctypes.data, f.ctypes.data,
                          alpha.ctypes.data, nr, reps.ctypes.data,
                          rec.ctypes.data, fit.ctypes.data)
        ok = np.isfinite(alpha) & (alpha > 0)
        xc = raw[:, reps].astype(np.int64)
        qc = (raw[:, reps] / f[:, reps])
        its = np.where(np.arange(5)[None, None, :] < rec[..., :1],
                       rec[..., 1::2], 0).sum(axis=(1, 2))
        keys = {
            'dist only (position order)': (np.arange(n),),
            'total count (current)': (raw.sum(1),),
            'condition count': (xc.sum(1),),
            'condition counts lexicographic': tuple(xc.T[::-1]),
            'condition mean x/f': (qc.mean(1),),
            'condition min, max count': (xc.max(1), xc.min(1)),
            'iterations (oracle bound)': (its,),
        }
        # slots in descending-count order per pixel (the kernel may visit a
        # pixel's replicates in any order: only the mu_out clamp carries
        # across them, and it can be resolved first)
        rs = np.argsort(-xc, axis=1, kind='stable')
        rec_s = np.take_along_axis(rec, rs[:, :, None], axis=1)
        xs = np.take_along_axis(xc, rs, axis=1)
        keys['sorted slots: (max, min)'] = (xs[:, -1], xs[:, 0])
        keys['sorted slots: (log2 max, min)'] = (
            xs[:, -1], np.floor(np.log2(xs[:, 0] + 1)))
        keys['sorted slots: (min, max)'] = (xs[:, 0], xs[:, -1])
        for name, k in keys.items():
            order = np.lexsort(k + (dist,))
            order = order[ok[order]]
            r = rec_s if name.startswith('sorted slots') else rec
            a, i = model(r[order], fit[order])
            t = tot.setdefault(name, [0.0, 0.0])
            t[0] += a
            t[1] += i
    for name, (a, i) in tot.items():
        print('%-34s modelled cost %.3e  lane util %.3f' % (name, a, i / a))


if __name__ == '__main__':
    main()
