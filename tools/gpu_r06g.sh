# round-6 final kernel stats + PMC passes of the default bench command, then
# the full default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_prof_step.sh r06g > gpurun_out/r06g_top.txt 2>&1 || exit 1
bash tools/pmc_passes.sh r06g || exit 1
timeout -k 10 900 python3 -u bench.py > gpurun_out/r06g_bench.json 2> gpurun_out/r06g_bench.err || exit 1
head -12 gpurun_out/r06g_top.txt
