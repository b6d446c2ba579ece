set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-r06a}
timeout -k 10 900 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
