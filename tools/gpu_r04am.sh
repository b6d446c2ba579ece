#!/bin/bash
# r04am: the round-end check at HEAD -- the whole GPU suite + smoke, then the
# driver's default bench command (CPU baseline rows, e2e, cfg3 / cfg4 lines)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_tests.sh r04am || exit $?
timeout -k 10 900 python3 -u bench.py > gpurun_out/r04am_bench.json 2> gpurun_out/r04am_bench.err
