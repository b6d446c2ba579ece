#!/bin/bash
# r04u: equalize at 3 waves / SIMD (168 VGPRs) vs 4
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "w4:cur:H3D_DISP_W2=4 w3:cur:H3D_DISP_W2=3" 3
