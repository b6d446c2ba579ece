#!/bin/bash
# r04r: equalize occupancy (H3D_DISP_W2) and Brent LDS staging re-swept on
# the current kernels
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "w4:cur:H3D_DISP_W2=4 w5:cur:H3D_DISP_W2=5 w6:cur:H3D_DISP_W2=6 l96:cur:H3D_BRENT_LDS_KB=96 l64:cur:H3D_BRENT_LDS_KB=64" 2
