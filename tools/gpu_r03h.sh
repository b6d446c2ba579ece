#!/bin/bash
# k_brent LDS staging A/B (144 / 96 / 0 KB), cfg4 on one GPU, -m gpu tests,
# smoke.   tools/gpu_r03h.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "lds144:cur: lds0:cur:H3D_BRENT_LDS_KB=0 lds96:cur:H3D_BRENT_LDS_KB=96" 2
H3D_TIMING=1 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-e2e \
  > gpurun_out/${tag}_timing.json 2> gpurun_out/${tag}_timing.err
timeout -k 10 300 python3 -u tools/run_cfg.py --cfg 4 > gpurun_out/${tag}_cfg4.json 2> gpurun_out/${tag}_cfg4.err
tail -n 1 gpurun_out/${tag}_cfg4.json
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
tail -n 2 gpurun_out/${tag}_gpu_tests.log
