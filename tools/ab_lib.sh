#!/bin/bash
# A/B of libh3d variants (hic3defdr_amd/lib/variants/libh3d_<v>.so) on the
# default bench, interleaved; then the -m gpu tests on the variant named
# first.   tools/ab_lib.sh "<v1> <v2> ..."
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
vs=${1:-"base s"}
first=${vs%% *}
for rep in 1 2; do
for v in $vs; do
  H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_$v.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-e2e --no-other-configs --steps 10 \
    > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$v', round(d['value']/1e6,1), round(d['ms_per_step'],3), {a: round(b,3) for a, b in k.items() if a != 'note'})"
done
done
H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_$first.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -rP --timeout 300 \
  --timeout-method thread > gpurun_out/ab_gpu_tests.log 2>&1 || { tail -n 40 gpurun_out/ab_gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/ab_gpu_tests.log
