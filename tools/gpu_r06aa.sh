set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_lib.sh -r 3 "split:: split0:split0:" > gpurun_out/r06aa_ab.txt 2>&1 || exit 1
cat gpurun_out/r06aa_ab.txt
bash tools/ab_lib.sh -c 4 -r 1 "split:: split0:split0:" > gpurun_out/r06aa_ab4.txt 2>&1 || exit 1
cat gpurun_out/r06aa_ab4.txt
