#!/bin/bash
# device-side Brent mode choice (k_brent / k_brent_gang by live segments):
# interleaved A/B against one workgroup per segment (H3D_BRENT=0), cfg3 at
# N = 1 both ways, then the whole -m gpu suite.   tools/gpu_r03w.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "spec:spec: plain:spec:H3D_BRENT=0" 3
for v in 1 0; do
  H3D_BRENT=$v timeout -k 10 300 python3 -u bench.py --config cfg3 --steps 3 --warmup 1 \
    > gpurun_out/${tag}_cfg3_b$v.json 2> gpurun_out/${tag}_cfg3_b$v.err
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg3_b$v.json').read().splitlines()[-1]); print('cfg3 brent=$v', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
done
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 60 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
