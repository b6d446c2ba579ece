#!/bin/bash
# cfg4 (human chr1 at 5 kb, R = 18, C = 3, dmax 400) at HEAD: the timed run,
# rocprofv3 kernel stats, and the four PMC passes of tools/pmc_passes.sh
# over one step -> gpurun_out/pmc_<tag>_summary.json
#   tools/gpu_cfg4_pmc.sh <tag>
set -e
tag=${1:-cfg4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/run_cfg.py --cfg 4 --steps 3 --warmup 1 \
  > gpurun_out/${tag}_run.json 2> gpurun_out/${tag}_run.err
tail -n 1 gpurun_out/${tag}_run.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 -u tools/run_cfg.py --cfg 4 --steps 1 --warmup 0 > gpurun_out/${tag}_prof.json 2> gpurun_out/${tag}_prof.err
s=$(find gpurun_out/${tag}_prof -name '*kernel_stats.csv' -print -quit)
cp $s gpurun_out/${tag}_kernel_stats.csv
rm -rf gpurun_out/${tag}_prof
run() {
  timeout -k 10 300 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/pmc_${tag}_$1 -o run -- \
    python3 -u tools/run_cfg.py --cfg 4 --steps 1 --warmup 0 > gpurun_out/pmc_${tag}_$1.log 2>&1
}
run sq "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU"
run f64 "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
run fetch "FETCH_SIZE"
run write "WRITE_SIZE"
python3 tools/pmc_summary.py $tag > gpurun_out/pmc_${tag}_summary.json
rm -rf gpurun_out/pmc_${tag}_sq gpurun_out/pmc_${tag}_f64 gpurun_out/pmc_${tag}_fetch gpurun_out/pmc_${tag}_write
echo done
