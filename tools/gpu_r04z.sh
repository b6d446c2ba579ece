#!/bin/bash
# r04z: cfg3 end to end through the class with the stages under cProfile
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/run_e2e.py --chroms 20 --workers 16 --profile 40 \
  > gpurun_out/r04z_e2e_cfg3.json 2> gpurun_out/r04z_e2e_cfg3.err
