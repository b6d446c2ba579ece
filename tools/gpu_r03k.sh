#!/bin/bash
# GPU tests + the default bench (its e2e leg reads the NPZ inputs natively)
#   tools/gpu_r03k.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 300 python3 -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
tail -n 2 gpurun_out/${tag}_gpu_tests.log
tail -n 1 gpurun_out/${tag}_bench.json | cut -c1-300
