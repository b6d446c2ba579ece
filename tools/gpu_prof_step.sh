#!/bin/bash
# rocprofv3 kernel trace + stats of the default cfg2 bench step, the top
# kernels and the per-step idle gaps (tools/trace_gaps.py).
#   tools/gpu_prof_step.sh <tag>
set -o pipefail
tag=${1:-prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/${tag}_prof -o run -- python3 -u bench.py --no-cpu-baseline --no-e2e --no-other-configs --no-peaks \
  > gpurun_out/${tag}_prof_bench.json 2> gpurun_out/${tag}_prof.err || exit 1
s=$(find gpurun_out/${tag}_prof -name '*kernel_stats.csv' -print -quit)
t=$(find gpurun_out/${tag}_prof -name '*kernel_trace.csv' -print -quit)
cp "$s" gpurun_out/${tag}_kernel_stats.csv
cp "$t" gpurun_out/${tag}_kernel_trace.csv
python3 tools/trace_gaps.py "$t" 10 > gpurun_out/${tag}_gaps.txt
python3 - "$tag" <<'PY'
import csv, sys
tag = sys.argv[1]
rows = list(csv.DictReader(open('gpurun_out/%s_kernel_stats.csv' % tag)))
for r in rows[:30]:
    print('%-90s %6s %12.1f %10.1f' % (r['Name'][:90], r['Calls'], float(r['TotalDurationNs']) / 1e3, float(r['AverageNs']) / 1e3))
PY
rm -rf gpurun_out/${tag}_prof
