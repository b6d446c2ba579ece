#!/bin/bash
# r04w: the driver's default bench command (CPU rows, e2e, other configs)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
t0=$(date +%s)
timeout -k 10 900 python3 -u bench.py > gpurun_out/r04w_bench.json 2> gpurun_out/r04w_bench.err
echo "bench wall $(( $(date +%s) - t0 )) s" > gpurun_out/r04w_wall.txt
