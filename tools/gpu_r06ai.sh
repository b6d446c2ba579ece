set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_operators.py tests/test_gpu_scale.py -v --timeout 300 --timeout-method thread > gpurun_out/r06ai_tests.log 2>&1 || { tail -30 gpurun_out/r06ai_tests.log; exit 1; }
tail -3 gpurun_out/r06ai_tests.log
bash tools/ab_lib.sh -r 1 "cur::" > gpurun_out/r06ai_ab.txt 2>&1 || exit 1
cat gpurun_out/r06ai_ab.txt
