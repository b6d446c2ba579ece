"""The generated log table (hic3defdr_amd/csrc/h3d_logtab.h) is what
tools/log_table.py produces, and the scheme it feeds (log_fast: 1024-step
mantissa table, degree-5 log1p) holds its documented accuracy against numpy's
80-bit log."""
import importlib.util
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gen():
    spec = importlib.util.spec_from_file_location(
        'log_table', os.path.join(REPO, 'tools', 'log_table.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_header_is_generated():
    mod = _gen()
    with open(mod.HEADER) as fh:
        assert fh.read() == mod.header(mod.table())


def test_log_fast_scheme_accuracy():
    mod = _gen()
    rows = mod.table()
    rng = np.random.default_rng(7)
    for xs, bar_abs, bar_rel in ((rng.uniform(0.3, 3, 200000), 3e-16, 4e-16),
                                 (rng.uniform(1, 1e4, 200000), 2e-15, 3e-16)):
        ref = np.log(xs.astype(np.longdouble))
        err = np.abs(mod.log_fast(xs, rows) - ref)
        rel = np.where(ref != 0, err / np.abs(ref), err)
        assert float(err.max()) < bar_abs
        assert float(rel.max()) < bar_rel
