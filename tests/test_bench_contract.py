"""bench.py host-side contract (no GPU): the roofline traffic figure comes
from the committed PMC summary of the default command and only for that
workload; the LRT byte count matches DESIGN.md's 108 B/px at R=4, C=2."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_pmc_summary_matches_default_workload():
    d = json.load(open(bench.PMC_SUMMARY))
    assert (d['bins'], d['dmax']) == (20000, 250)
    names = [k.split('[')[0] for k in d['kernels']]
    assert any('k_disp_work<4, 4, 0>' in k for k in names)


def test_pmc_traffic_per_launch():
    t = bench.pmc_traffic('k_disp_work<4, 4, 0>', 20000, 250)
    d = json.load(open(bench.PMC_SUMMARY))
    e = [v for k, v in d['kernels'].items() if 'k_disp_work<4, 4, 0>' in k][0]
    want = (e['hbm_read_bytes_corrected'] + e['hbm_write_bytes']) / e['dispatches']
    assert t == want and t > 0
    # other workloads were not profiled: traffic stays null
    assert bench.pmc_traffic('k_disp_work<4, 4, 0>', 1000, 250) is None
    assert bench.pmc_traffic('no_such_kernel', 20000, 250) is None


def test_lrt_bytes_per_pixel():
    assert bench.bytes_per_lrt_pixel(4, 2) == 108
