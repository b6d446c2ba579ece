#!/bin/bash
# One GPU-box pass: parity tests, smoke, default bench, rocprofv3 kernel stats
# of the same bench command.  Usage (via gpurun): tools/gpu_round.sh <tag>
# Every GPU step has its own time limit and the steps stop at the first failure.
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 300 python3 -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --no-cpu-baseline \
  > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
tail -n 1 gpurun_out/${tag}_bench.json
