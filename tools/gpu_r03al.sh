#!/bin/bash
# k_brent's DiDonato-Morris guess out of line vs inlined: interleaved A/B on cfg2, then the
# Brent-related GPU tests on the new build
tag=${1:-r}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab_summary.txt
bash tools/ab_env.sh "cold:cold: base:base:" 3
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 60 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
