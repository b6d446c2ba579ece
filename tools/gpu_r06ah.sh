set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_lib.sh -r 2 "l128::H3D_BRENT_LDS_KB=128 l144::H3D_BRENT_LDS_KB=144 l148::H3D_BRENT_LDS_KB=148" > gpurun_out/r06ah_ab.txt 2>&1 || exit 1
cat gpurun_out/r06ah_ab.txt
