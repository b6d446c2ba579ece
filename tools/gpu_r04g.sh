#!/bin/bash
# r04g: PMC passes + rocprofv3 kernel stats of the default bench command at
# HEAD (-> profiles/r04/g, profiles/pmc_default.json), then cfg3 end to end
# through the class, files included (tools/run_e2e.py). Each step under its
# own limit; the first failure ends the script.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/pmc_passes.sh r04g
bash tools/gpu_prof_bench.sh r04g > gpurun_out/r04g_prof_top.txt
timeout -k 10 600 python3 -u tools/run_e2e.py --chroms 20 --workers 16 \
  > gpurun_out/r04g_e2e_cfg3.json 2> gpurun_out/r04g_e2e_cfg3.err
# keep the merge-back small: the stats csv only
find gpurun_out/r04g_prof -name '*kernel_trace.csv' -delete
