#!/bin/bash
# M = 2 equalize path (R_c <= 2) vs M = 4, and its W; cfg4 with the
# spill-free k_brent<8>.   tools/sweep_m2.sh <tag>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${1:-m2}
for cfg in "M2=0" "M2=1 W2=4" "M2=1 W2=5" "M2=1 W2=6" "M2=0" "M2=1 W2=4"; do
  set -- $cfg
  m2=${1#M2=}; w2=${2#W2=}; w2=${w2:-4}
  H3D_DISP_M2=$m2 H3D_DISP_W2=$w2 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-e2e \
    --steps 10 > gpurun_out/${tag}_b.json 2> gpurun_out/${tag}_b.err
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_b.json').read().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$cfg', round(d['value']/1e6,1), round(d['ms_per_step'],3), round(k['disp_work'],3), round(k['disp_nll'],3))"
done
timeout -k 10 300 python3 -u tools/run_cfg.py --cfg 4 --steps 2 --warmup 1 > gpurun_out/${tag}_cfg4.json 2> gpurun_out/${tag}_cfg4.err
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg4.json').read()); print('cfg4', d['ms_per_step'], d['kernels_ms_per_step'], d['checks']['deterministic_disp'])"
