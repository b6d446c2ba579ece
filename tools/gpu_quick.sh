#!/bin/bash
# Quick GPU check: parity tests + one bench line (no profiler).
#   tools/gpu_quick.sh <tag> [bench args...]
set -e
tag=${1:-q}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
timeout -k 10 300 python3 -u bench.py "$@" > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
tail -n 1 gpurun_out/${tag}_bench.json
