#!/bin/bash
# The whole -m gpu suite and smoke() (each under its own limit, stopping at
# the first failure).   tools/gpu_suite.sh <tag> [pytest args...]
set -o pipefail
tag=${1:-t}
shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v -rP --timeout 300 \
  --timeout-method thread "$@" > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/${tag}_smoke.log 2>&1
tail -n 3 gpurun_out/${tag}_gpu_tests.log
