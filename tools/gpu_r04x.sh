#!/bin/bash
# r04x: the slowest N = 8 rank's share (6/8) with its kernel breakdown, the
# N = 1 cfg3 step for reference, then the whole GPU suite + smoke at HEAD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
H3D_BENCH_EMULATE=6/8 timeout -k 10 400 python3 -u bench.py --config cfg3 --steps 5 --warmup 2 \
  > gpurun_out/r04x_emu6of8.json 2> gpurun_out/r04x_emu6of8.err || exit 1
timeout -k 10 400 python3 -u bench.py --config cfg3 --steps 3 --warmup 1 \
  > gpurun_out/r04x_cfg3_n1.json 2> gpurun_out/r04x_cfg3_n1.err || exit 1
bash tools/gpu_tests.sh r04x || exit $?
