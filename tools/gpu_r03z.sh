#!/bin/bash
# rocprofv3 kernel trace of the default cfg2 bench (the device-chosen Brent
# mode per qcml iteration), and one rank of an N = 8 cfg3 run with the
# host-built gangs vs the device tables + device-chosen mode
tag=${1:-r}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_prof_bench.sh ${tag}
for v in 0 1; do
  for i in 1 2; do
    env $( [ $v = 1 ] && echo H3D_DEV_TABLES_ANY=1 ) H3D_BENCH_EMULATE=0/8 timeout -k 10 300 python3 -u bench.py --config cfg3 --steps 3 --warmup 1 \
      > gpurun_out/${tag}_emu8_any$v.json 2> gpurun_out/${tag}_emu8_any$v.err
    python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_emu8_any$v.json').read().splitlines()[-1]); print('emu0of8 any=$v', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
  done
done
