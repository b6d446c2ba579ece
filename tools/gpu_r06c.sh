set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-r06c}
timeout -k 10 120 python -u -c "
import torch, json, sys
sys.path.insert(0, '.')
import bench
print(json.dumps(bench.measured_peaks(0)))
" > gpurun_out/${tag}_peaks.json 2>&1 && \
timeout -k 10 300 python -u tools/class_stamps.py --runs 5 > gpurun_out/${tag}_stamps.json 2> gpurun_out/${tag}_stamps.err
