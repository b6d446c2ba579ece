"""Wraps a tools/pmc_passes.sh summary (gpurun_out/pmc_<tag>_summary.json)
into profiles/pmc_default.json, the file bench.py reads its counter-based
roofline figures from (FP64 flops, lane utilisation, HBM traffic per
launch). The passes must have run the default bench command.

    python tools/pmc_default.py <tag> [profile_dir]
"""
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
src = os.path.join(REPO, 'gpurun_out', 'pmc_%s_summary.json' % tag)
kernels = json.load(open(src))
out = {'bins': 20000, 'dmax': 250,
       'command': 'tools/pmc_passes.sh %s: rocprofv3 --pmc <pass> -- python3 '
                  'bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e '
                  '--no-other-configs --no-peaks (one pass '
                  'each: SQ, F64, FETCH_SIZE, WRITE_SIZE)' % tag,
       'units': 'hbm_read_bytes_corrected = FETCH_SIZE KB x1024 x2 (gfx950 '
                'correction); hbm_write_bytes = WRITE_SIZE KB x1024; SQ_* '
                'wave-level counts; totals over all dispatches',
       'kernels': kernels}
if len(sys.argv) > 2:
    d = os.path.join(REPO, sys.argv[2])
    os.makedirs(d, exist_ok=True)
    shutil.copy(src, os.path.join(d, 'pmc_summary.json'))
    out['source'] = os.path.join(sys.argv[2], 'pmc_summary.json')
json.dump(out, open(os.path.join(REPO, 'profiles', 'pmc_default.json'), 'w'),
          indent=1, sort_keys=True)
