set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_lib.sh -r 3 "fold:: base:base:" > gpurun_out/r06al_ab.txt 2>&1 || { cat gpurun_out/r06al_ab.txt; exit 1; }
cat gpurun_out/r06al_ab.txt
bash tools/gpu_suite.sh r06al || exit 1
