#!/bin/bash
# k_brent workgroups of 512 threads, two per CU (each with half the LDS
# staging), vs one 1024-thread workgroup per CU: interleaved A/B on cfg2
tag=${1:-r}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab_summary.txt
bash tools/ab_env.sh "b512:b512:H3D_BRENT_LDS_KB=72 b512s:b512:H3D_BRENT_LDS_KB=56 base:base:" 2
