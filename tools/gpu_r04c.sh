#!/bin/bash
# r04c: the default bench (no CPU rows), the e2e profile of the product
# class, every rank's share of N = 2 / 4 / 8 cfg3 runs
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err
timeout -k 10 300 python3 -u tools/e2e_profile.py --top 30 > gpurun_out/r04c_e2eprof.log 2>&1
timeout -k 10 400 python3 -u tools/emulate_ranks.py --steps 3 \
  --out gpurun_out/r04c_emulate_ranks.json > gpurun_out/r04c_emulate.log 2>&1
