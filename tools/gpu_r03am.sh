#!/bin/bash
# k_brent LDS staging re-swept with the log table in LDS (144 / 96 / 0 KB)
tag=${1:-r}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab_summary.txt
bash tools/ab_env.sh "lds64:cur:H3D_BRENT_LDS_KB=64 lds80:cur:H3D_BRENT_LDS_KB=80 lds96:cur:H3D_BRENT_LDS_KB=96 lds112:cur:H3D_BRENT_LDS_KB=112 lds128:cur:H3D_BRENT_LDS_KB=128" 2
