#!/bin/bash
# one rank's share of an N-GPU cfg3 run (N = 8, 4, 2; the live-segment hint
# keeps its Brent searches in gangs), cfg3 at N = 1, then the multi-rank GPU
# tests.   tools/gpu_r03v.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for N in 8 4 2; do
  H3D_BENCH_EMULATE=0/$N timeout -k 10 300 python3 -u bench.py --config cfg3 --steps 3 --warmup 1 \
    > gpurun_out/${tag}_emu$N.json 2> gpurun_out/${tag}_emu$N.err
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_emu$N.json').read().splitlines()[-1]); print('emu0of$N', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
done
timeout -k 10 300 python3 -u bench.py --config cfg3 --steps 3 --warmup 1 \
  > gpurun_out/${tag}_cfg3.json 2> gpurun_out/${tag}_cfg3.err
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg3.json').read().splitlines()[-1]); print('cfg3', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_mr_tests.log 2>&1 || \
  { tail -n 60 gpurun_out/${tag}_mr_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_mr_tests.log
