#!/bin/bash
# tuning sweep of the disp_work register-budget knob (diagnostics); one bench
# process each: SWEEP="1 3 4" tools/sweep_disp.sh <tag>
set -e
tag=${1:-s}
for w in ${SWEEP:-1 2 3 4}; do
  H3D_DISP_W=$w timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_${tag}_w${w}.json
  python3 -c "import json; d=json.loads(open('gpurun_out/sweep_${tag}_w${w}.json').read().strip().splitlines()[-1]); print('W=$w', round(d['value']/1e6,2), 'Mpx/s', {k: (round(v,2) if isinstance(v, float) else v) for k,v in d['kernels_ms_per_step'].items()})"
done
