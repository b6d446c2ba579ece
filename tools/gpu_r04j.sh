#!/bin/bash
# r04j: the whole GPU suite + smoke at HEAD, then the default bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_tests.sh r04j || exit $?
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/r04j_bench.json 2> gpurun_out/r04j_bench.err
