#!/bin/bash
# r04d: the GPU suite + smoke (tools/gpu_tests.sh), then the default bench
# without the CPU rows -- each step under its own limit; the bench runs even
# when a test failed (its numbers are read separately)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_tests.sh r04d; trc=$?
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e \
  > gpurun_out/r04d_bench.json 2> gpurun_out/r04d_bench.err || exit $?
exit $trc
