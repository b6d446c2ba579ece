#!/bin/bash
# gang slice size: the default cfg2 bench and one rank of an N = 8 cfg3 run
# (device tables) at H3D_GANG_P = default / 1024 / 512 / 256, kernel stats
# of the tail launches from a short trace at each
tag=${1:-r}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for P in 0 1024 512 256; do
  H3D_GANG_P=$P timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-e2e --steps 10 \
    > gpurun_out/${tag}_cfg2_p$P.json 2> gpurun_out/${tag}_cfg2_p$P.err
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg2_p$P.json').read().splitlines()[-1]); print('cfg2 P=$P', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
  H3D_GANG_P=$P H3D_DEV_TABLES_ANY=1 H3D_BENCH_EMULATE=0/8 timeout -k 10 300 python3 -u bench.py --config cfg3 --steps 3 --warmup 1 \
    > gpurun_out/${tag}_emu8_p$P.json 2> gpurun_out/${tag}_emu8_p$P.err
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_emu8_p$P.json').read().splitlines()[-1]); print('emu0of8 P=$P', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
done
