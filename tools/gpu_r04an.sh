#!/bin/bash
# r04an: the round's final profiles at HEAD: PMC passes + rocprofv3 kernel
# stats of the default bench command (-> profiles/r04/an,
# profiles/pmc_default.json), every rank of N = 2 / 4 / 8 emulated, cfg3 end
# to end through the class
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/pmc_passes.sh r04an
bash tools/gpu_prof_bench.sh r04an > gpurun_out/r04an_prof_top.txt
find gpurun_out/r04an_prof -name '*kernel_trace.csv' -delete
timeout -k 10 400 python3 -u tools/emulate_ranks.py --steps 3 \
  --out gpurun_out/r04an_emulate_ranks.json > gpurun_out/r04an_emulate.log 2>&1
timeout -k 10 600 python3 -u tools/run_e2e.py --chroms 20 --workers 16 \
  > gpurun_out/r04an_e2e_cfg3.json 2> gpurun_out/r04an_e2e_cfg3.err
