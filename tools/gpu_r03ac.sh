#!/bin/bash
# 24-bit (distance, min / max count code) sort key vs the 32-bit one:
# interleaved A/B on cfg2, cfg4 on the new key, then the -m gpu suite on it
tag=${1:-r}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab_summary.txt
bash tools/ab_env.sh "key8:key8: base:base:" 3
timeout -k 10 400 python3 -u tools/run_cfg.py --cfg 4 > gpurun_out/${tag}_cfg4.json 2> gpurun_out/${tag}_cfg4.err
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg4.json').read()); print('cfg4', round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: round(v,2) for k, v in d['kernels_ms_per_step'].items()}, d['checks'])"
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 60 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
