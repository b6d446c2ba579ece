#!/bin/bash
# Perf iteration on the GPU box: one bench line (no parity tests, no CPU
# baseline) + FETCH_SIZE / WRITE_SIZE PMC passes of one step.
#   tools/gpu_perf.sh <tag>
set -e
tag=${1:-p}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${tag}_$c -o run -- \
    python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_${tag}_$c.log 2>&1
done
python3 tools/pmc_summary.py $tag > gpurun_out/pmc_${tag}_summary.json
rm -rf gpurun_out/pmc_${tag}_FETCH_SIZE gpurun_out/pmc_${tag}_WRITE_SIZE
tail -n 1 gpurun_out/${tag}_bench.json
