#!/bin/bash
# Round-3 evidence pass: -m gpu tests, smoke, the default bench, PMC passes
# (tools/pmc_passes.sh) and rocprofv3 kernel stats of the bench.
#   tools/gpu_r03g.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
# the full-size cfg2 parity metrics (printed by the test)
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_scale.py -m gpu -rP -q --timeout 180 \
  --timeout-method thread > gpurun_out/${tag}_scale_metrics.log 2>&1
timeout -k 10 300 python3 -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --no-cpu-baseline --no-e2e \
  > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
bash tools/pmc_passes.sh ${tag}
tail -n 2 gpurun_out/${tag}_gpu_tests.log
tail -n 1 gpurun_out/${tag}_bench.json | cut -c1-300
