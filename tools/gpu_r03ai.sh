#!/bin/bash
# the grouped LRT (k_lrt8, R > 8) with the table log from LDS: cfg4
# interleaved A/B, then the LRT / e2e GPU tests on the new build
tag=${1:-r}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in lrt8tab base; do
    H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_$v.so timeout -k 10 400 python3 -u tools/run_cfg.py --cfg 4 \
      > gpurun_out/${tag}_cfg4_$v.json 2> gpurun_out/${tag}_cfg4_$v.err
    python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg4_$v.json').read()); print('cfg4 $v', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: round(v,2) for k, v in d['kernels_ms_per_step'].items()})"
  done
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 60 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
