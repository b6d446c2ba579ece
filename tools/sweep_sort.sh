#!/bin/bash
# Pixel-order A/B (H3D_DISP_SORT 1 = (dist, total count), 2 = per-condition
# (dist, max, min)): parity tests under 2, then bench and cfg4 under each.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${1:-sort}
H3D_DISP_SORT=2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_e2e.py tests/test_gpu_scale.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/${tag}_tests2.log 2>&1 || \
  { tail -n 30 gpurun_out/${tag}_tests2.log; exit 1; }
tail -n 2 gpurun_out/${tag}_tests2.log
for s in 1 2 1 2; do
  H3D_DISP_SORT=$s timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-e2e \
    --steps 10 > gpurun_out/${tag}_bench_s$s.json 2> gpurun_out/${tag}_bench_s$s.err
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${tag}_bench_s$s.json').read().splitlines()[-1]); print('sort $s', d['value'], d['ms_per_step'], d['kernels_ms_per_step'])"
done
for s in 1 2; do
  H3D_DISP_SORT=$s timeout -k 10 300 python3 -u tools/run_cfg.py --cfg 4 --steps 2 \
    --warmup 1 > gpurun_out/${tag}_cfg4_s$s.json 2> gpurun_out/${tag}_cfg4_s$s.err
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg4_s$s.json').read()); print('cfg4 sort $s', d['ms_per_step'], d['kernels_ms_per_step'], d['checks'])"
done
