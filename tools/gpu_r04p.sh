#!/bin/bash
# r04p: the special-function tests first in their own process (the runtime
# order), then the whole GPU suite + smoke, then the default bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_special_host.py tests/test_gpu_parity.py -m gpu -q \
  --timeout 200 --timeout-method thread > gpurun_out/r04p_order.log 2>&1 || { tail -n 30 gpurun_out/r04p_order.log; exit 1; }
tail -n 1 gpurun_out/r04p_order.log
bash tools/gpu_tests.sh r04p || exit $?
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/r04p_bench.json 2> gpurun_out/r04p_bench.err
