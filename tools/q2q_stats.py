"""Work census of the equalize pass on a cfg2-shaped sample (CPU only).

Builds tools/q2q_stats.cpp with g++, makes a synthetic chromosome with the
bench generator, estimates dispersions with the oracle, then runs the
instrumented equalize at the final per-distance dispersion, in the GPU's
(dist, count) pixel order, and reports per pixel-replicate work and a
64-lane wave divergence estimate (sum of per-wave max / sum of mean).

    python tools/q2q_stats.py [--bins 1500] [--dmax 250]
"""
import argparse
import ctypes
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def build():
    out = os.path.join(tempfile.gettempdir(), 'libq2qstats.so')
    src = os.path.join(HERE, 'q2q_stats.cpp')
    subprocess.check_call(['g++', '-O2', '-std=c++17', '-shared', '-fPIC',
                           '-ffp-contract=off', src, '-o', out])
    return ctypes.CDLL(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--bins', type=int, default=1500)
    ap.add_argument('--dmax', type=int, default=250)
    ap.add_argument('--key', choices=('maxmin', 'maxmin8', 'minmax', 'summax',
                                      'summin', 'total', 'ratio', 'sumratio',
                                      'maxratio', 'allmaxmin8'), default='maxmin')
    args = ap.parse_args()
    import oracle
    from hic3defdr_amd import synthetic
    lib = build()
    nf = lib.q2qs_fields()
    names = ('pq cf su ser cf_it su_it ser_it fac_l1 l1_it inv halley wh '
             'lgam lgam_small lgam_it fit fit_it').split()
    assert len(names) == nf
    tmp = tempfile.mkdtemp(prefix='q2qs_')
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
    cond = design.argmax(axis=1)
    raw0, f0, dist0 = raw, f, dist
    P = ctypes.c_void_p
    lib.q2qs_equalize.argtypes = [ctypes.c_int64, ctypes.c_int, P, P, P,
                                  ctypes.c_int, P, P, P]
    for c in range(design.shape[1]):
        # the kernel's pixel order: per condition (distance, max, min count
        # of the condition's replicates, each capped to 12 bits)
        # (k_dist_cond_keys); --key total: (distance, all replicates' total)
        rc = raw0[:, cond == c]
        mx, mn = np.minimum(rc.max(1), 4095), np.minimum(rc.min(1), 4095)
        sm = np.minimum(rc.sum(1), 4095)
        if args.key == 'total':
            order = np.lexsort((raw0.sum(1), dist0))
        elif args.key == 'minmax':
            order = np.lexsort((mx, mn, dist0))
        elif args.key == 'summax':
            order = np.lexsort((mx, sm, dist0))
        elif args.key == 'summin':
            order = np.lexsort((mn, sm, dist0))
        elif args.key in ('ratio', 'sumratio', 'maxratio'):
            # the replicates' normalized counts' log ratio (how far each
            # replicate sits from the pixel's mean: the tail position the
            # incomplete-gamma trip counts depend on), 4 bins per e-fold
            fc = f0[:, cond == c]
            nrm = (rc + 0.5) / fc
            lr = np.log(nrm.max(1) / nrm.min(1))
            rcode = np.minimum((lr * 4).astype(np.int64), 63)

            def code(v):
                v = np.asarray(v, dtype=np.int64)
                return np.where(v < 128, v, np.minimum(128 + (v - 128) // 8, 255))
            lead = {'ratio': code(rc.min(1)), 'sumratio': code(rc.sum(1)),
                    'maxratio': code(rc.max(1))}[args.key]
            order = np.lexsort((rcode, lead, dist0))
        elif args.key == 'allmaxmin8':
            # ONE order for every condition: the 8-bit codes of the max /
            # min count over ALL replicates (a prep with one sort and one
            # gather instead of one per condition)
            def code(v):
                v = np.asarray(v, dtype=np.int64)
                return np.where(v < 128, v, np.minimum(128 + (v - 128) // 8, 255))
            order = np.lexsort((code(raw0.min(1)), code(raw0.max(1)), dist0))
        elif args.key == 'maxmin8':
            # 8-bit count codes: exact below 128, then 8 counts per code up
            # to 1151 (k_dist_cond_keys' compressed key)
            def code(v):
                v = np.asarray(v, dtype=np.int64)
                return np.where(v < 128, v, np.minimum(128 + (v - 128) // 8, 255))
            order = np.lexsort((code(rc.min(1)), code(rc.max(1)), dist0))
        else:
            order = np.lexsort((mn, mx, dist0))
        raw, f, dist = raw0[order], np.ascontiguousarray(f0[order]), \
            dist0[order]
        n, R = raw.shape
        reps = np.flatnonzero(cond == c).astype(np.int32)
        nr = len(reps)
        alpha = np.ascontiguousarray(dpd[dist, c])
        ok = np.isfinite(alpha)
        rec = np.zeros((n, nr, nf), dtype=np.int64)
        out = np.zeros((n, nr))
        lib.q2qs_equalize(n, R, raw.ctypes.data, f.ctypes.data,
                          alpha.ctypes.data, nr, reps.ctypes.data,
                          rec.ctypes.data, out.ctypes.data)
        rec = rec[ok]
        m = ok.sum()
        print('condition %d: %d pixels x %d reps' % (c, m, nr))
        per = rec.sum(axis=(0, 1)) / (m * nr)
        for k, v in zip(names, per):
            print('  %-10s %8.3f / pixel-rep' % (k, v))
        # wave divergence: lanes = pixels (the rep loop is per lane)
        w = 64
        nw = m // w
        for k in ('cf_it', 'ser_it', 'su_it', 'halley', 'l1_it', 'lgam_it',
                  'fit_it'):
            j = names.index(k)
            v = rec[:nw * w, :, j].sum(1).reshape(nw, w)
            print('  wave %-8s mean %7.2f  max/mean %5.2f' %
                  (k, v.mean(), v.max(1).sum() / max(v.sum(1).sum() / w, 1)))
        # path mix per wave: waves that run both CF and series
        cfw = rec[:nw * w, :, names.index('cf')].sum(1).reshape(nw, w) > 0
        sew = (rec[:nw * w, :, names.index('ser')] +
               rec[:nw * w, :, names.index('su')]).sum(1).reshape(nw, w) > 0
        print('  waves with both CF and series lanes: %.1f%%' %
              (100 * np.mean(cfw.any(1) & sew.any(1))))
        hal = rec[:, :, names.index('halley')].ravel()
        print('  halley steps histogram:',
              np.bincount(hal, minlength=9)[:9] / hal.size)
        fit = rec[:, 0, names.index('fit_it')]
        print('  fit_mu iterations histogram:',
              np.bincount(fit, minlength=20)[:20] / fit.size)
        halley_report(lib, raw, f, dist, dpd, cond, c)
        pq_report(lib, raw, f, dist, dpd, cond, c)
        wave_report(lib, raw, f, dist, dpd, cond, c)




def halley_report(lib, raw, f, dist, dpd, cond, c):
    P = ctypes.c_void_p
    n, R = raw.shape
    reps = np.flatnonzero(cond == c).astype(np.int32)
    nr = len(reps)
    alpha = np.ascontiguousarray(dpd[dist, c])
    out = np.full((n, nr, 6), np.nan)
    lib.q2qs_halley.argtypes = [ctypes.c_int64, ctypes.c_int, P, P, P,
                                ctypes.c_int, P, P]
    lib.q2qs_halley(n, R, raw.ctypes.data, f.ctypes.data, alpha.ctypes.data,
                    nr, reps.ctypes.data, out.ctypes.data)
    o = out.reshape(-1, 6)
    o = o[np.isfinite(o[:, 0])]
    dx1, err1 = o[:, 0], o[:, 3]
    print('  halley: first-step |dx|/x quantiles 50/90/99/max:',
          np.quantile(dx1, [.5, .9, .99, 1]))
    for thr in (1e-6, 1e-5, 1e-4, 1e-3):
        sel = dx1 <= thr
        print('   stop after step 1 if dx<=%g: %.1f%% of lanes, max err %.2e'
              % (thr, 100 * sel.mean(), err1[sel].max() if sel.any() else 0))
    ratio = err1 / np.maximum(dx1, 1e-300) ** 3
    print('   err1/dx1^3 quantiles 50/99/max:',
          np.quantile(ratio[dx1 > 1e-5], [.5, .99, 1]))


def pq_report(lib, raw, f, dist, dpd, cond, c):
    P = ctypes.c_void_p
    n, R = raw.shape
    reps = np.flatnonzero(cond == c).astype(np.int32)
    alpha = np.ascontiguousarray(dpd[dist, c])
    cap = n * len(reps) * 6
    out = np.zeros((cap, 4))
    lib.q2qs_pq_log.restype = ctypes.c_int64
    lib.q2qs_pq_log.argtypes = [ctypes.c_int64, ctypes.c_int, P, P, P,
                                ctypes.c_int, P, P, ctypes.c_int64]
    m = lib.q2qs_pq_log(n, R, raw.ctypes.data, f.ctypes.data,
                        alpha.ctypes.data, len(reps), reps.ctypes.data,
                        out.ctypes.data, cap)
    a, x, it, path = out[:m].T
    print('  pq calls %d, mean iterations %.1f' % (m, it.mean()))
    for lo, hi in ((0, 1), (1, 5), (5, 20), (20, 100), (100, 1e9)):
        sel = (a >= lo) & (a < hi)
        print('   a in [%g, %g): %.1f%% of calls, %.1f%% of iterations, '
              'mean it %.1f' % (lo, hi, 100 * sel.mean(),
                                100 * it[sel].sum() / it.sum(),
                                it[sel].mean() if sel.any() else 0))
    temme = (a > 20) & (np.abs(x - a) / a < 0.3)
    print('   Temme region (a>20, |x-a|/a<0.3): %.1f%% of calls, %.1f%% of '
          'iterations' % (100 * temme.mean(), 100 * it[temme].sum() / it.sum()))


def wave_report(lib, raw, f, dist, dpd, cond, c, it_cost=18.0,
                call_cost=250.0, fit_cost=60.0, cf_factor=1.9):
    """Wave-level cost model of the equalize kernel: per slot, each pq-call
    position costs max-over-lanes iterations * it_cost (+ call_cost if any
    lane makes the call); fit_mu max iterations * fit_cost. Compared with
    the lane-mean (perfect utilisation)."""
    P = ctypes.c_void_p
    n, R = raw.shape
    reps = np.flatnonzero(cond == c).astype(np.int32)
    nr = len(reps)
    alpha = np.ascontiguousarray(dpd[dist, c])
    rec = np.zeros((n, nr, 11))
    fit = np.zeros(n)
    lib.q2qs_wave_log.argtypes = [ctypes.c_int64, ctypes.c_int, P, P, P,
                                  ctypes.c_int, P, P, P]
    lib.q2qs_wave_log(n, R, raw.ctypes.data, f.ctypes.data, alpha.ctypes.data,
                      nr, reps.ctypes.data, rec.ctypes.data, fit.ctypes.data)
    ok = np.isfinite(alpha) & (alpha > 0)
    rec, fit = rec[ok], fit[ok]
    w = 64
    nw = len(rec) // w
    rec = rec[:nw * w].reshape(nw, w, nr, 11)
    fit = fit[:nw * w].reshape(nw, w)
    parts = {}
    ncall = rec[..., 0]
    its = rec[..., 1::2]          # (nw, w, nr, 5)
    paths = rec[..., 2::2]
    made = np.arange(5)[None, None, None, :] < ncall[..., None]
    itm = np.where(made, its, 0)
    # actual: per slot j, call position c: max over lanes; CF and series
    # paths diverge -> pay both maxima
    cf = np.where(made & (paths == 0), itm, 0)
    se = np.where(made & (paths != 0), itm, 0)
    act_it = (cf_factor * cf.max(1) + se.max(1)).sum(axis=(1, 2)) * it_cost
    act_call = made.any(1).sum(axis=(1, 2)) * call_cost
    act_fit = fit.max(1) * fit_cost
    ideal_it = (cf_factor * np.where(paths == 0, itm, 0) +
                np.where(paths != 0, itm, 0)).sum(axis=(1, 2, 3)) / w * it_cost
    ideal_call = made.sum(axis=(1, 2, 3)) / w * call_cost
    ideal_fit = fit.mean(1) * fit_cost
    print('  wave model (cost units / wave): iterations %.0f (ideal %.0f), '
          'call overhead %.0f (ideal %.0f), fit %.0f (ideal %.0f)' % (
              act_it.mean(), ideal_it.mean(), act_call.mean(),
              ideal_call.mean(), act_fit.mean(), ideal_fit.mean()))
    # by call position
    for cpos in range(4):
        a = (cf[..., cpos].max(1) + se[..., cpos].max(1)).sum(1).mean()
        b = itm[..., cpos].sum(axis=(1, 2)).mean() / w
        frac = made[..., cpos].mean()
        both = ((cf[..., cpos] > 0).any(1) & (se[..., cpos] > 0).any(1)).mean()
        print('   call %d: lanes making it %.2f, wave iters %.1f vs mean %.1f,'
              ' slot-waves with both paths %.2f' % (cpos, frac, a, b, both))
    tot = act_it + act_call + act_fit
    ideal = ideal_it + ideal_call + ideal_fit
    print('  modelled lane utilisation %.2f' % (ideal.sum() / tot.sum()))
    # wave-local task sort: a wave's w x nr q2q tasks
    # sorted by a key, then run as nr rounds of w lanes -- the q2q loop
    # cost of each round is the max over its lanes per call position (CF and
    # series paths paid separately), as above
    tasks_it = itm.transpose(0, 2, 1, 3).reshape(nw, nr * w, 5)
    tasks_pa = paths.transpose(0, 2, 1, 3).reshape(nw, nr * w, 5)
    tasks_md = made.transpose(0, 2, 1, 3).reshape(nw, nr * w, 5)
    cost = (np.where(tasks_pa == 0, cf_factor, 1.0) * tasks_it).sum(2)

    def rounds(order):
        it = np.take_along_axis(tasks_it, order[..., None], 1)
        pa = np.take_along_axis(tasks_pa, order[..., None], 1)
        md = np.take_along_axis(tasks_md, order[..., None], 1)
        it = it.reshape(nw, nr, w, 5)
        pa = pa.reshape(nw, nr, w, 5)
        md = md.reshape(nw, nr, w, 5)
        c_ = np.where(md & (pa == 0), it, 0)
        s_ = np.where(md & (pa != 0), it, 0)
        return ((cf_factor * c_.max(2) + s_.max(2)).sum(axis=(1, 2)) * it_cost
                + md.any(2).sum(axis=(1, 2)) * call_cost)
    keys = {
        'oracle cost': cost,
        'fwd path, fwd iters': tasks_pa[..., 0] * 1000 + tasks_it[..., 0],
        'fwd path, inv path': tasks_pa[..., 0] * 10 + tasks_pa[..., 1],
        'fwd path': tasks_pa[..., 0].astype(float),
    }
    base = act_it + act_call
    for name, key in keys.items():
        order = np.argsort(key, axis=1, kind='stable')
        r = rounds(order)
        print('   wave-local sort by %-22s: q2q loop+call cost %.0f vs %.0f '
              '(%.1f%%)' % (name, r.mean(), base.mean(),
                            100 * (r.mean() / base.mean() - 1)))


if __name__ == '__main__':
    main()
