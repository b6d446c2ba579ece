#!/bin/bash
# tuning sweep of the disp_work knobs (diagnostics); one bench process each
set -e
for cfg in "1 0" "1 1" "3 1" "4 1"; do
  set -- $cfg
  H3D_DISP_W=$1 H3D_DISP_SORT=$2 timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_w$1_s$2.json
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_w$1_s$2.json').read().strip().splitlines()[-1]); print('W=$1 SORT=$2', round(d['value']/1e6,2), 'Mpx/s', {k: round(v,2) for k,v in d['kernels_ms_per_step'].items()})"
done
