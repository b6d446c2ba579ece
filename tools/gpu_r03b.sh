#!/bin/bash
# A/B (base = last commit's kernels; cur = this tree; plain = this tree with
# the one-workgroup Brent), then the -m gpu tests, smoke, the default bench
# and cfg3 on one GPU.   tools/gpu_r03b.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "base:base: cur:cur: plain:cur:H3D_BRENT=0" 2
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 300 python3 -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 200 python3 -u bench.py --config cfg3 \
  > gpurun_out/${tag}_cfg3.json 2> gpurun_out/${tag}_cfg3.err
tail -n 3 gpurun_out/${tag}_gpu_tests.log
tail -n 1 gpurun_out/${tag}_bench.json | cut -c1-400
