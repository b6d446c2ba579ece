#!/bin/bash
# every -m gpu test, a 10-step default bench (no CPU baseline / e2e) and
# cfg4.   tools/gpu_quick2.sh <tag>
set -e
tag=${1:-q}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
for i in 1 2; do
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-e2e --steps 10 \
  > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_bench.json').read().splitlines()[-1]); print('cfg2', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
done
timeout -k 10 300 python3 -u tools/run_cfg.py --cfg 4 --steps 2 --warmup 1 \
  > gpurun_out/${tag}_cfg4.json 2> gpurun_out/${tag}_cfg4.err
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg4.json').read()); print('cfg4', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: round(v,2) for k, v in d['kernels_ms_per_step'].items()}, d['checks']['deterministic_disp'])"
