#!/bin/bash
# r04af: Brent pixels per trip for the mid / large NLL forms (3, 4) vs 2
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "cur:cur: pf3:pf3: pf4:pf4:" 3
