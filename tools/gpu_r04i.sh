#!/bin/bash
# r04i: the resident-path tests and the e2e goldens, then cfg3 end to end
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_resident.py tests/test_gpu_e2e.py \
  -m gpu -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04i_tests.log 2>&1 || \
  { tail -n 40 gpurun_out/r04i_tests.log; exit 1; }
tail -n 2 gpurun_out/r04i_tests.log
timeout -k 10 600 python3 -u tools/run_e2e.py --chroms 20 --workers 16 --profile 30 \
  > gpurun_out/r04i_e2e_cfg3.json 2> gpurun_out/r04i_e2e_cfg3.err
cat gpurun_out/r04i_e2e_cfg3.json
