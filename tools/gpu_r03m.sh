#!/bin/bash
# interleaved A/B of the step with the device vs host smoother, then a
# kernel trace of the device-table bench (per-step gaps)
#   tools/gpu_r03m.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in 1 0; do
    H3D_DEV_TABLE=$v timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-e2e > gpurun_out/${tag}_ab_dev${v}_$i.json 2>> gpurun_out/${tag}_ab.err
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']/1e6,1),round(d['ms_per_step'],3))" gpurun_out/${tag}_ab_dev${v}_$i.json
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --no-cpu-baseline --no-e2e --steps 5 \
  > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
f=$(find gpurun_out/${tag}_prof -name '*kernel_trace.csv' -print -quit)
python3 tools/trace_gaps.py $f 15 > gpurun_out/${tag}_trace_gaps.txt
s=$(find gpurun_out/${tag}_prof -name '*kernel_stats.csv' -print -quit)
cp $s gpurun_out/${tag}_kernel_stats.csv
rm -rf gpurun_out/${tag}_prof
cat gpurun_out/${tag}_trace_gaps.txt | head -n 30
