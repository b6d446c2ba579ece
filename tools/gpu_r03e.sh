#!/bin/bash
# k_brent prefetch A/B (cfg2), one rank of an N-GPU cfg3 run emulated on
# this GPU (N = 2, 4, 8; Brent auto / one workgroup per segment / gang),
# cfg3 on one GPU, then the -m gpu tests and smoke.  tools/gpu_r03e.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
# (prefetch A/B done in r03e: k_brent 3.07 vs 2.84 ms with it -- reverted)
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); k=d['kernels_ms_per_step']; print(sys.argv[2], round(d['value']/1e6,1), round(d['ms_per_step'],3), {a: round(b,3) for a, b in k.items() if a != 'note'}, d.get('emulated', {}).get('disp_pixels_estimate_disp'))" "$1" "$2" | tee -a gpurun_out/${tag}_summary.txt; }
for e in 8:1 8:0 8:2 4:1 2:1; do
  N=${e%%:*}; v=${e##*:}
  H3D_BENCH_EMULATE=0/$N H3D_BRENT=$v timeout -k 10 200 python3 -u bench.py --config cfg3 \
    > gpurun_out/${tag}_emu${N}_b$v.json 2> gpurun_out/${tag}_emu${N}_b$v.err
  summ gpurun_out/${tag}_emu${N}_b$v.json emu0of${N}_brent$v
done
timeout -k 10 200 python3 -u bench.py --config cfg3 \
  > gpurun_out/${tag}_cfg3.json 2> gpurun_out/${tag}_cfg3.err
summ gpurun_out/${tag}_cfg3.json cfg3_auto
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
tail -n 2 gpurun_out/${tag}_gpu_tests.log
