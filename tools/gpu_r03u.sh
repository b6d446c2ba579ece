#!/bin/bash
# sharded BH: the multi-rank GPU tests (incl. bh_sharded vs h3d_bh_dev), the
# driver's N = 2 path rehearsed over gloo on one GPU, rank 0's share of an
# N = 8 cfg3 run emulated, and cfg3 at N = 1.   tools/gpu_r03u.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_mr_tests.log 2>&1 || \
  { tail -n 60 gpurun_out/${tag}_mr_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_mr_tests.log
bash tools/gpu_n2_rehearsal.sh ${tag}
H3D_BENCH_EMULATE=0/8 timeout -k 10 300 python3 -u bench.py --config cfg3 --steps 3 --warmup 1 \
  > gpurun_out/${tag}_emu8.json 2> gpurun_out/${tag}_emu8.err
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_emu8.json').read().splitlines()[-1]); print('emu0of8', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
timeout -k 10 300 python3 -u bench.py --config cfg3 --steps 3 --warmup 1 \
  > gpurun_out/${tag}_cfg3.json 2> gpurun_out/${tag}_cfg3.err
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg3.json').read().splitlines()[-1]); print('cfg3', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
