#!/bin/bash
# A/B (base = round 2, cur = this tree), cfg4, host stamps, the N = 2 cfg3
# rehearsal over gloo on this GPU, -m gpu tests, smoke.  tools/gpu_r03i.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "next:next: cur:cur: base:base:" 2
H3D_TIMING=1 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-e2e \
  > gpurun_out/${tag}_timing.json 2> gpurun_out/${tag}_timing.err
timeout -k 10 300 python3 -u tools/run_cfg.py --cfg 4 > gpurun_out/${tag}_cfg4.json 2> gpurun_out/${tag}_cfg4.err
tail -n 1 gpurun_out/${tag}_cfg4.json | cut -c1-300
bash tools/gpu_n2_rehearsal.sh ${tag}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
tail -n 2 gpurun_out/${tag}_gpu_tests.log
