#!/bin/bash
# the committed tree: -m gpu suite, default bench line, one rank of an
# N = 8 / 4 cfg3 run, the driver's N = 2 command rehearsed over gloo
tag=${1:-r}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 60 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_bench.json').read().splitlines()[-1]); print('bench', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
for N in 8 4; do
  H3D_BENCH_EMULATE=0/$N timeout -k 10 300 python3 -u bench.py --config cfg3 --steps 3 --warmup 1 \
    > gpurun_out/${tag}_emu$N.json 2> gpurun_out/${tag}_emu$N.err
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_emu$N.json').read().splitlines()[-1]); print('emu0of$N', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
done
bash tools/gpu_n2_rehearsal.sh ${tag}
