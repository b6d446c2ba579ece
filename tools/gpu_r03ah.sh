#!/bin/bash
# equalize register budget re-swept on the current kernels (H3D_DISP_W2 4 /
# 5 / 6), then the full evidence pass (tools/gpu_final.sh)
tag=${1:-r}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab_summary.txt
bash tools/ab_env.sh "w4:cur: w5:cur:H3D_DISP_W2=5 w6:cur:H3D_DISP_W2=6" 2
cp gpurun_out/ab_summary.txt gpurun_out/${tag}_ab_w2.txt
bash tools/gpu_final.sh ${tag}
