#!/bin/bash
# cfg4: k_brent<8>'s LDS staging size (H3D_BRENT_LDS_KB) vs occupancy
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 144 0 48 72 144; do
  H3D_BRENT_LDS_KB=$v timeout -k 10 300 python3 -u tools/run_cfg.py --cfg 4 --steps 2 --warmup 1 \
    > gpurun_out/cfg4_lds$v.json 2> gpurun_out/cfg4_lds$v.err
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],round(d['value']/1e6,2),round(d['ms_per_step'],2),{k:round(x,2) for k,x in d['kernels_ms_per_step'].items()})" gpurun_out/cfg4_lds$v.json $v
done
for v in 144 0 48; do
  H3D_BRENT_LDS_KB=$v timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/cfg2_lds$v.json 2>/dev/null
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('cfg2',sys.argv[2],round(d['value']/1e6,1),round(d['ms_per_step'],3))" gpurun_out/cfg2_lds$v.json $v
done
