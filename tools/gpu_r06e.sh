set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-r06e}
timeout -k 10 300 python -u tools/class_stamps.py --runs 5 > gpurun_out/${tag}_stamps.json 2> gpurun_out/${tag}_stamps.err && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_resident.py tests/test_gpu_cfg1.py tests/test_gpu_simulation.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${tag}_tests.log 2>&1
