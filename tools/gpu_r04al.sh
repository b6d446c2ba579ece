#!/bin/bash
# r04al: kernel trace of the default bench step at HEAD and its idle gaps
# (tools/trace_gaps.py), the trace csv kept small (bench steps only)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/r04al_prof -o run -- python3 -u bench.py --no-cpu-baseline --no-e2e --no-other-configs \
  > gpurun_out/r04al_prof_bench.json 2> gpurun_out/r04al_prof.err
f=$(find gpurun_out/r04al_prof -name '*kernel_trace.csv' | head -n 1)
python3 tools/trace_gaps.py "$f" 5 > gpurun_out/r04al_gaps.txt
python3 tools/trace_gaps.py "$f" 1 > gpurun_out/r04al_gaps_1us.txt
