import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (gfx950)')


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def e2e_inputs(name):
    """Constructor kwargs for a golden e2e dataset (paths relocated to the
    repo checkout, so fixtures work on the GPU box too)."""
    g = golden('e2e_%s.npz' % name)
    base = os.path.join(GOLDEN, 'data', name)
    reps = [str(r) for r in g['meta_reps']]
    conds = [str(c) for c in g['meta_conds']]
    chroms = [str(c) for c in g['meta_chroms']]
    kw = dict(
        raw_npz_patterns=[os.path.join(base, r, '<chrom>_raw.npz')
                          for r in reps],
        bias_patterns=[os.path.join(base, r, '<chrom>_kr.bias')
                       for r in reps],
        chroms=chroms, reps=reps, conds=conds,
        design=g['meta_design'].astype(bool),
        dist_thresh_max=int(g['meta_dist_thresh_max']),
        loop_patterns=({c: os.path.join(base, 'clusters', '%s_<chrom>.json' % c)
                        for c in conds} if bool(g['meta_loops']) else None))
    return g, kw


def rel_err(a, b):
    a = np.atleast_1d(np.asarray(a, dtype=float))
    b = np.atleast_1d(np.asarray(b, dtype=float))
    both_nan = np.isnan(a) & np.isnan(b)
    same = (a == b) | both_nan
    with np.errstate(all='ignore'):
        r = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    r[same] = 0.0
    return float(np.max(r)) if r.size else 0.0


@pytest.fixture(scope='session')
def repo_root():
    return REPO
