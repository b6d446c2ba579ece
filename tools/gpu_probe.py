"""Step-by-step GPU probe with flushed progress (diagnostics only)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests'))

import numpy as np  # noqa: E402


def log(*a):
    print('[probe %.1fs]' % (time.time() - T0), *a, flush=True)


T0 = time.time()
os.environ.setdefault('H3D_DEBUG', '1')
from hic3defdr_amd import _native  # noqa: E402
import oracle  # noqa: E402
from conftest import e2e_inputs  # noqa: E402

ctx = _native.context(0)
log('ctx open')
g, kw = e2e_inputs(sys.argv[1] if len(sys.argv) > 1 else 'small2')
chrom = kw['chroms'][0]
bias = oracle.load_bias([p.replace('<chrom>', chrom) for p in kw['bias_patterns']])
di = g['disp_idx__%s' % chrom]
row, col = g['row__%s' % chrom][di], g['col__%s' % chrom][di]
raw = g['raw__%s' % chrom][di]
f = bias[row] * bias[col] * g['size_factors__%s' % chrom][di]
dist = col - row
design = kw['design']
C = design.shape[1]
D = kw['dist_thresh_max'] + 1
cond = design.argmax(axis=1)
n = int(sys.argv[2]) if len(sys.argv) > 2 else len(raw)
sel = np.arange(len(raw)) < n
log('inputs', n, 'pixels')
tab = np.stack([_native.disp_table(g['disp_per_dist'][:, c]) for c in range(C)], 1)
p, llr, m0, m1, disp = ctx.lrt(raw[sel], f[sel], dist[sel], tab, cond)
log('lrt done', np.nanmax(p), np.nanmin(p))
dpd = ctx.disp_per_dist(raw[sel], f[sel], dist[sel], cond, C, D)
log('disp done')
ref = g['disp_per_dist']
fin = np.isfinite(ref) & np.isfinite(dpd)
log('disp max rel err (full only)', np.max(np.abs(dpd[fin] - ref[fin]) / ref[fin]))
