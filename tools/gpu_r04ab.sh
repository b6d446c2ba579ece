#!/bin/bash
# r04ab: the Brent serial step run twice (dbl) -- its share of k_brent
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "cur:cur: dbl:dbl:" 3
