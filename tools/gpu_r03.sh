#!/bin/bash
# Round-3 GPU pass: every -m gpu test, smoke(), the default bench (cfg2:
# CPU baseline + parity sample + e2e), an A/B of the Brent kernel
# (H3D_BRENT=0: one workgroup per segment), cfg3 on one GPU, rocprofv3
# kernel stats of the bench. Each step under its own limit; stops at the
# first failure.   tools/gpu_r03.sh <tag> [skip-tests]
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
fi
timeout -k 10 300 python3 -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
H3D_BRENT=0 timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-e2e \
  > gpurun_out/${tag}_bench_plain.json 2> gpurun_out/${tag}_bench_plain.err
timeout -k 10 200 python3 -u bench.py --config cfg3 \
  > gpurun_out/${tag}_cfg3.json 2> gpurun_out/${tag}_cfg3.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --no-cpu-baseline --no-e2e \
  > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
tail -n 3 gpurun_out/${tag}_gpu_tests.log || true
tail -n 1 gpurun_out/${tag}_bench.json
