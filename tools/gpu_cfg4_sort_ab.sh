#!/bin/bash
# cfg4: the disp pixel order inside a distance segment (H3D_DISP_SORT 0 / 1 / 2)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 2 1 0 2; do
  H3D_DISP_SORT=$v timeout -k 10 300 python3 -u tools/run_cfg.py --cfg 4 --steps 2 --warmup 1 \
    > gpurun_out/cfg4_sort$v.json 2> gpurun_out/cfg4_sort$v.err
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],round(d['value']/1e6,2),round(d['ms_per_step'],2),{k:round(x,2) for k,x in d['kernels_ms_per_step'].items()})" gpurun_out/cfg4_sort$v.json $v
done
