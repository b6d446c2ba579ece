#!/bin/bash
# PMC counter passes over one step (each pass its own rocprofv3 run,
# counters only -- never combined with runtime / sys traces):
#   tools/pmc_passes.sh <tag> [2|3|4]  -> gpurun_out/pmc_<tag>_summary.json
# workload: 2 = the default cfg2 bench step (default), 3 / 4 = tools/run_cfg.py
set -e
tag=${1:-r}
cfg=${2:-2}
if [ "$cfg" = 2 ]; then
  cmd="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-other-configs --no-peaks"
else
  cmd="tools/run_cfg.py --cfg $cfg --steps 1 --warmup 0"
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  timeout -k 10 300 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/pmc_${tag}_$1 -o run -- \
    python3 -u $cmd > gpurun_out/pmc_${tag}_$1.log 2>&1
}
run sq "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU"
run f64 "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
run fetch "FETCH_SIZE"
run write "WRITE_SIZE"
python3 tools/pmc_summary.py $tag > gpurun_out/pmc_${tag}_summary.json
# keep the merge-back small: summaries + logs only
rm -rf gpurun_out/pmc_${tag}_sq gpurun_out/pmc_${tag}_f64 gpurun_out/pmc_${tag}_fetch gpurun_out/pmc_${tag}_write
