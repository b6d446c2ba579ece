#!/bin/bash
# Full GPU-box pass: every -m gpu test, smoke(), one bench line (no CPU
# baseline), the rocprofv3 kernel stats of the same bench command, then the
# PMC counter passes (tools/pmc_passes.sh). Each step under its own limit;
# the first failing step ends the run.   tools/gpu_full.sh <tag>
set -e
tag=${1:-f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --no-cpu-baseline \
  > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
bash tools/pmc_passes.sh ${tag}
tail -n 3 gpurun_out/${tag}_gpu_tests.log
tail -n 1 gpurun_out/${tag}_bench.json
