#!/bin/bash
# GPU-box pass: the whole -m gpu suite (no -x: every failure is reported) and
# smoke(); each step under its own time limit, stopping at the first step
# that fails.   tools/gpu_tests.sh <tag> [pytest args...]
set -e
tag=${1:-t}
shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -rP --timeout 300 \
  --timeout-method thread "$@" > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
tail -n 3 gpurun_out/${tag}_gpu_tests.log
