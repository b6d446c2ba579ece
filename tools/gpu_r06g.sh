set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_resident.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r06g_tests.log 2>&1 && \
bash tools/gpu_prof_step.sh r06g > gpurun_out/r06g_top.txt 2>&1 && \
timeout -k 10 400 python -u tools/smoother_census.py > gpurun_out/r06g_census.json 2> gpurun_out/r06g_census.err
