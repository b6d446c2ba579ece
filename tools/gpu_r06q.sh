set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u bench.py > gpurun_out/r06q_bench.json 2> gpurun_out/r06q_bench.err || exit 1
bash tools/gpu_suite.sh r06q
