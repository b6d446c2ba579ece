set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_prof_step.sh r06p > gpurun_out/r06p_top.txt 2>&1 && \
bash tools/pmc_passes.sh r06p
