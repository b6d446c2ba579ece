#!/bin/bash
# device-built segment tables: GPU suite, then an interleaved A/B of the
# bench step (H3D_DEV_SEG_TABLES 1 / 0)
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
for i in 1 2 3; do
  for v in 1 0; do
    H3D_DEV_SEG_TABLES=$v timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-e2e > gpurun_out/${tag}_ab_seg${v}_$i.json 2>> gpurun_out/${tag}_ab.err
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']/1e6,1),round(d['ms_per_step'],3))" gpurun_out/${tag}_ab_seg${v}_$i.json
  done
done
