#!/bin/bash
# cfg2 bench at H3D_DISP_W = 4, 5, 6 (equalize register budget, M = 4)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in 4 5 6; do
  H3D_DISP_W=$w timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/sw4_w$w.json 2> gpurun_out/sw4_w$w.err
done
grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/sw4_w*.json
