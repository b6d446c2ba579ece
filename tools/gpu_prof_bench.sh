#!/bin/bash
# rocprofv3 kernel trace + stats of the default bench step (no CPU baseline,
# no e2e); prints the top kernels.   tools/gpu_prof_bench.sh <tag>
set -e
tag=${1:-prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --no-cpu-baseline --no-e2e --no-other-configs --no-peaks \
  > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err
python3 - "$tag" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
f = glob.glob('gpurun_out/%s_prof/**/*kernel_stats.csv' % tag, recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:25]:
    print('%-70s %6s %12.1f %10.1f' % (r['Name'][:70], r['Calls'], float(r['TotalDurationNs']) / 1e3, float(r['AverageNs']) / 1e3))
PY
tail -n 1 gpurun_out/${tag}_prof_bench.json | cut -c1-300
