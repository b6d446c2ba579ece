#!/bin/bash
# r04y: the NLL log without a table (poly: 2 atanh series) vs the LDS table
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "tab:tab: poly:poly:" 3
for w in 1 4; do
  H3D_DISP_W8=$w timeout -k 10 300 python3 -u tools/run_cfg.py --cfg 4 --steps 2 --warmup 1 \
    > gpurun_out/r04y_cfg4_w$w.json 2> gpurun_out/r04y_cfg4_w$w.err
done
