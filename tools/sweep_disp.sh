#!/bin/bash
# tuning sweep of the disp_work knobs (diagnostics); one bench process each
set -e
for cfg in ${SWEEP:-"1 1" "3 1" "4 1"}; do
  w=${cfg% *}; s=${cfg#* }
  H3D_DISP_W=$w H3D_DISP_SORT=$s timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_w${w}_s${s}.json
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_w${w}_s${s}.json').read().strip().splitlines()[-1]); print('W=$w SORT=$s', round(d['value']/1e6,2), 'Mpx/s', {k: round(v,2) for k,v in d['kernels_ms_per_step'].items()})"
done
