#!/bin/bash
# The operator / simulation GPU tests, then the cfg3 and cfg4 shapes
# (tools/run_cfg.py) each with a rocprofv3 kernel-stats pass.
#   tools/gpu_cfgs.sh <tag>
set -e
tag=${1:-c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in 4 3; do
  timeout -k 10 400 python3 -u tools/run_cfg.py --cfg $c > gpurun_out/${tag}_cfg$c.json 2> gpurun_out/${tag}_cfg$c.err
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/${tag}_prof_cfg$c -o run -- python3 -u tools/run_cfg.py --cfg $c --steps 1 \
    > gpurun_out/${tag}_prof_cfg$c.json 2> gpurun_out/${tag}_prof_cfg$c.err
done
cat gpurun_out/${tag}_cfg4.json gpurun_out/${tag}_cfg3.json
