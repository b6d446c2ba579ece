#!/bin/bash
# fused estimate_disp + device smoother: table tests, then an interleaved
# A/B of the bench step over H3D_DEV_TABLE 2 / 1 / 0
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_table.py -m gpu -v --timeout 200 \
  --timeout-method thread > gpurun_out/${tag}_table_tests.log 2>&1 || \
  { tail -n 60 gpurun_out/${tag}_table_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_table_tests.log
for i in 1 2 3; do
  for v in 2 1 0; do
    H3D_DEV_TABLE=$v timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-e2e > gpurun_out/${tag}_ab_tab${v}_$i.json 2>> gpurun_out/${tag}_ab.err
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']/1e6,1),round(d['ms_per_step'],3))" gpurun_out/${tag}_ab_tab${v}_$i.json
  done
done
