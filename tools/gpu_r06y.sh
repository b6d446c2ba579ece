set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_lib.sh -r 2 "prio1:: prio2:prio2:" > gpurun_out/r06y_ab.txt 2>&1 || exit 1
cat gpurun_out/r06y_ab.txt
bash tools/gpu_r06x.sh
