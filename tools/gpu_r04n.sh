#!/bin/bash
# r04n: equalize task schedule A/B (H3D_EQ_STATIC8, per-XCD-group heads)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "e0:cur:H3D_EQ_STATIC8=0 e2:cur:H3D_EQ_STATIC8=2 e3:cur:H3D_EQ_STATIC8=3 e4:cur:H3D_EQ_STATIC8=4 e5:cur:H3D_EQ_STATIC8=5" 2
