#!/bin/bash
# every -m gpu test, then cfg4 (run_cfg) plain and under rocprofv3 kernel
# stats; prints the top kernels.   tools/gpu_cfg4_prof.sh <tag>
set -e
tag=${1:-c4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python3 -u tools/run_cfg.py --cfg 4 --steps 2 --warmup 1 \
  > gpurun_out/${tag}_cfg4.json 2> gpurun_out/${tag}_cfg4.err
python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_cfg4.json').read()); print('cfg4', d['value']/1e6, d['ms_per_step'], d['kernels_ms_per_step'], d['checks'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/${tag}_cfg4prof -o run -- python3 -u tools/run_cfg.py --cfg 4 --steps 1 --warmup 0 \
  > gpurun_out/${tag}_cfg4prof.json 2> gpurun_out/${tag}_cfg4prof.err
python3 - "$tag" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
f = glob.glob('gpurun_out/%s_cfg4prof/**/*kernel_stats.csv' % tag, recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print('%-64s %5s %10.1f %9.1f' % (r['Name'][:64], r['Calls'], float(r['TotalDurationNs']) / 1e3, float(r['AverageNs']) / 1e3))
PY
