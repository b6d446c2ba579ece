#!/bin/bash
# the multi-GPU path at HEAD: cfg3 at N = 1 through bench.py (BH included),
# one rank's share of an N = 8 / 4 / 2 run, the driver's N = 2 command over
# gloo on one GPU
tag=${1:-r}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --config cfg3 --steps 3 --warmup 1 \
  > gpurun_out/${tag}_cfg3.json 2> gpurun_out/${tag}_cfg3.err
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg3.json').read().splitlines()[-1]); print('cfg3', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
for N in 8 4 2; do
  H3D_BENCH_EMULATE=0/$N timeout -k 10 300 python3 -u bench.py --config cfg3 --steps 3 --warmup 1 \
    > gpurun_out/${tag}_emu$N.json 2> gpurun_out/${tag}_emu$N.err
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_emu$N.json').read().splitlines()[-1]); print('emu0of$N', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
done
bash tools/gpu_n2_rehearsal.sh ${tag}
