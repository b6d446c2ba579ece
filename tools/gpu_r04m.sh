#!/bin/bash
# r04m: equalize task-schedule A/B (H3D_EQ_STATIC8), then the disp parity tests
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "e6:cur:H3D_EQ_STATIC8=6 e8:cur:H3D_EQ_STATIC8=8 e4:cur:H3D_EQ_STATIC8=4 nolpt:cur:H3D_BRENT_LPT=0" 2
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_multirank.py \
  -m gpu -q -rP --timeout 300 --timeout-method thread > gpurun_out/r04m_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/r04m_tests.log; exit 1; }
tail -n 2 gpurun_out/r04m_tests.log
