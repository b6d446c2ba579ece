#!/bin/bash
# r04b: GPU suite + smoke (tools/gpu_tests.sh), the default bench without the
# CPU rows, the e2e profile of the product class
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests.sh r04b
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err
timeout -k 10 300 python3 -u tools/e2e_profile.py --top 30 > gpurun_out/r04b_e2eprof.log 2>&1
