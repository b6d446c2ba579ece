#!/bin/bash
# tuning sweep of the NLL-pass register-budget knob: SWEEP="1 2 4" tools/sweep_nll.sh <tag>
set -e
tag=${1:-s}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in ${SWEEP:-1 2 4}; do
  H3D_NLL_W=$w timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/sweepnll_${tag}_w${w}.json
  python3 -c "import json; d=json.loads(open('gpurun_out/sweepnll_${tag}_w${w}.json').read().strip().splitlines()[-1]); print('NLL_W=$w', round(d['value']/1e6,2), 'Mpx/s', {k: (round(v,2) if isinstance(v, float) else v) for k,v in d['kernels_ms_per_step'].items()})"
done
