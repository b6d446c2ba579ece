#!/bin/bash
# Perf iteration on the GPU box: the disp/lrt parity tests, one bench line
# (no CPU baseline) and a rocprofv3 kernel-stats pass of the same bench
# command. Each step has its own time limit; the first failure ends the run.
#   tools/gpu_iter.sh <tag>
set -e
tag=${1:-i}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py \
  -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_tests.log; exit 1; }
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --no-cpu-baseline \
  > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
tail -n 3 gpurun_out/${tag}_tests.log
tail -n 1 gpurun_out/${tag}_bench.json
