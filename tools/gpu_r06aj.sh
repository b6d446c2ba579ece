set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_lib.sh -r 2 "bkt::H3D_BUCKET_SORT=1 rad::H3D_BUCKET_SORT=0" > gpurun_out/r06aj_ab.txt 2>&1 || { cat gpurun_out/r06aj_ab.txt; tail -20 gpurun_out/ab_bkt.err; exit 1; }
cat gpurun_out/r06aj_ab.txt
bash tools/gpu_suite.sh r06aj || exit 1
