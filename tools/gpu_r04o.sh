#!/bin/bash
# r04o: the mid-r NLL path A/B (mid vs cur, both at H3D_EQ_STATIC8=4), then
# the special-function unit tests on gfx950 and the disp parity tests
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "mid:mid:H3D_EQ_STATIC8=4 cur:cur:H3D_EQ_STATIC8=4" 3
timeout -k 10 600 python3 -u -m pytest tests/test_special_host.py tests/test_gpu_parity.py tests/test_gpu_scale.py \
  tests/test_gpu_cfg1.py -m gpu -q -rP --timeout 300 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/r04o_tests.log; exit 1; }
tail -n 2 gpurun_out/r04o_tests.log
