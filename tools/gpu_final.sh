#!/bin/bash
# Full evidence pass of the committed tree: -m gpu tests, smoke(), the
# default bench (CPU baseline, parity sample, e2e), rocprofv3 kernel stats of
# the bench, the four PMC passes, then cfg4 and cfg3 with kernel stats. Every
# GPU step under its own limit; the first failure ends the call.
#   tools/gpu_final.sh <tag>
set -e
tag=${1:-f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 600 python3 -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_bench.json').read().splitlines()[-1]); print('bench', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --no-cpu-baseline --no-e2e \
  > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
bash tools/pmc_passes.sh ${tag}
for c in 4 3; do
  timeout -k 10 400 python3 -u tools/run_cfg.py --cfg $c > gpurun_out/${tag}_cfg$c.json 2> gpurun_out/${tag}_cfg$c.err
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg$c.json').read()); print('cfg$c', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: round(v,2) for k, v in d['kernels_ms_per_step'].items()}, d['checks'])"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/${tag}_prof_cfg$c -o run -- python3 -u tools/run_cfg.py --cfg $c --steps 1 \
    > gpurun_out/${tag}_prof_cfg$c.json 2> gpurun_out/${tag}_prof_cfg$c.err
done
