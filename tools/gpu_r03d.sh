#!/bin/bash
# cfg2 A/B (plain / forced gang / last commit), cfg3 on one GPU (auto /
# forced gang), one rank of an 8-GPU cfg3 run emulated (auto = gang / plain),
# then the -m gpu tests and smoke.   tools/gpu_r03d.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "plain:cur:H3D_BRENT=0 gang:cur:H3D_BRENT=2 base:base:" 1
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); k=d['kernels_ms_per_step']; print(sys.argv[2], round(d['value']/1e6,1), round(d['ms_per_step'],3), {a: round(b,3) for a, b in k.items() if a != 'note'}, d.get('emulated', {}).get('disp_pixels_estimate_disp'))" "$1" "$2" | tee -a gpurun_out/${tag}_summary.txt; }
for v in 1 2 0; do
  H3D_BRENT=$v timeout -k 10 200 python3 -u bench.py --config cfg3 \
    > gpurun_out/${tag}_cfg3_b$v.json 2> gpurun_out/${tag}_cfg3_b$v.err
  summ gpurun_out/${tag}_cfg3_b$v.json cfg3_brent$v
done
for v in 1 0; do
  H3D_BENCH_EMULATE=0/8 H3D_BRENT=$v timeout -k 10 200 python3 -u bench.py --config cfg3 \
    > gpurun_out/${tag}_emu8_b$v.json 2> gpurun_out/${tag}_emu8_b$v.err
  summ gpurun_out/${tag}_emu8_b$v.json emu0of8_brent$v
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
tail -n 2 gpurun_out/${tag}_gpu_tests.log
