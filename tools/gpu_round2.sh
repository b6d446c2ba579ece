#!/bin/bash
# Round-end style GPU pass: every -m gpu test, smoke(), the DEFAULT bench
# command (CPU baseline + parity sample + e2e wall time), rocprofv3 kernel
# stats of the bench. Each step under its own limit; stops at the first
# failure.   tools/gpu_round2.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 600 python3 -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --no-cpu-baseline --no-e2e \
  > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
tail -n 3 gpurun_out/${tag}_gpu_tests.log
tail -n 1 gpurun_out/${tag}_bench.json
