set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_lib.sh -r 2 -p "ahead:: noahead:noahead:" > gpurun_out/r06r_ab.txt 2>&1 || exit 1
bash tools/gpu_suite.sh r06r || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/r06r_bench.json 2> gpurun_out/r06r_bench.err
