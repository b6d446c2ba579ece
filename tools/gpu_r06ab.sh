set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_suite.sh r06ab || exit 1
bash tools/gpu_n2_rehearsal.sh r06ab || exit 1
