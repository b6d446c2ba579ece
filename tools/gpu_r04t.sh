#!/bin/bash
# r04t: the Brent LDS head with a pixel's replicates adjacent (ilv) vs the
# per-replicate rows (old), LDS staging 128 / 144 / 152 KB
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "old:old: ilv:ilv: i144:ilv:H3D_BRENT_LDS_KB=144 i152:ilv:H3D_BRENT_LDS_KB=152 i96:ilv:H3D_BRENT_LDS_KB=96" 2
