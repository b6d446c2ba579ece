#!/bin/bash
# cfg2 bench + cfg4 at H3D_DISP_W8 = 1..4 (equalize register budget, M = 8)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/sw_bench.json 2> gpurun_out/sw_bench.err
for w in 1 2 3 4; do
  H3D_DISP_W8=$w timeout -k 10 300 python3 -u tools/run_cfg.py --cfg 4 --steps 2 > gpurun_out/sw_cfg4_w$w.json 2> gpurun_out/sw_cfg4_w$w.err
done
tail -n 1 gpurun_out/sw_bench.json | cut -c1-400
grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/sw_cfg4_w*.json
