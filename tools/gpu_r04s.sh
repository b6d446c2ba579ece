#!/bin/bash
# r04s: the round's final measurements at HEAD: PMC passes + rocprofv3 kernel
# stats of the default bench command (-> profiles/r04/s, pmc_default.json),
# every rank of N = 2 / 4 / 8 emulated, cfg3 end to end through the class,
# cfg4, and the default bench with its CPU baseline rows
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/pmc_passes.sh r04s
bash tools/gpu_prof_bench.sh r04s > gpurun_out/r04s_prof_top.txt
find gpurun_out/r04s_prof -name '*kernel_trace.csv' -delete
timeout -k 10 400 python3 -u tools/emulate_ranks.py --steps 3 \
  --out gpurun_out/r04s_emulate_ranks.json > gpurun_out/r04s_emulate.log 2>&1
timeout -k 10 400 python3 -u tools/run_cfg.py --cfg 4 --steps 2 --warmup 1 \
  > gpurun_out/r04s_cfg4.json 2> gpurun_out/r04s_cfg4.err
timeout -k 10 400 python3 -u tools/run_cfg.py --cfg 3 --steps 3 --warmup 1 \
  > gpurun_out/r04s_cfg3.json 2> gpurun_out/r04s_cfg3.err
timeout -k 10 600 python3 -u tools/run_e2e.py --chroms 20 --workers 16 \
  > gpurun_out/r04s_e2e_cfg3.json 2> gpurun_out/r04s_e2e_cfg3.err
timeout -k 10 600 python3 -u bench.py > gpurun_out/r04s_bench.json 2> gpurun_out/r04s_bench.err
