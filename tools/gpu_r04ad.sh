#!/bin/bash
# r04ad: Brent serial step inlined with the two NLL-constant lgammas on two
# lanes (par) vs inlined (inl) vs out of line (cur)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "cur:cur: inl:inl: par:par:" 3
