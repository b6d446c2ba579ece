set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/class_stamps.py --runs 3 --no-flush > gpurun_out/r06t_stamps_noflush.json 2> gpurun_out/r06t_stamps.err || exit 1
timeout -k 10 300 python3 -u tools/class_stamps.py --runs 3 > gpurun_out/r06t_stamps_flush.json 2>> gpurun_out/r06t_stamps.err || exit 1
