#!/bin/bash
# r04v: kernel trace of the default bench step -> idle gaps per step
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04v_trace -o run -- \
  python3 -u bench.py --no-cpu-baseline --no-e2e --no-other-configs --steps 10 --warmup 3 > gpurun_out/r04v_bench.json 2> gpurun_out/r04v_bench.err
f=$(find gpurun_out/r04v_trace -name '*kernel_trace.csv' | head -1)
python3 tools/trace_gaps.py "$f" 5 > gpurun_out/r04v_gaps.txt
rm -rf gpurun_out/r04v_trace
