#!/bin/bash
# the GPU tests before test_gpu_cfg3 in suite order, then it, H3D_DEBUG on
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
H3D_DEBUG=1 timeout -k 10 400 python3 -u -m pytest tests/test_alternatives.py tests/test_gpu_cfg3.py \
  -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/${tag}_seq.log 2>&1
rc=$?; echo "rc=$rc"
grep -E "launch error|pending|PASSED|FAILED|H3DError" gpurun_out/${tag}_seq.log | head -20
