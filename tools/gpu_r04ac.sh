#!/bin/bash
# r04ac: the Brent serial step inlined (inl) vs out of line (cur)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "cur:cur: inl:inl:" 3
