#!/bin/bash
# the log table in LDS for k_brent_gang and k_lrt too: interleaved A/B on
# cfg2 and on one rank of an N = 8 cfg3 run (gangs), then the -m gpu suite
tag=${1:-r}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab_summary.txt
bash tools/ab_env.sh "tab2:tab2: base:base:" 3
for v in tab2 base; do
  H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_$v.so H3D_BENCH_EMULATE=0/8 timeout -k 10 300 \
    python3 -u bench.py --config cfg3 --steps 3 --warmup 1 > gpurun_out/${tag}_emu8_$v.json 2> gpurun_out/${tag}_emu8_$v.err
  python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_emu8_$v.json').read().splitlines()[-1]); print('emu0of8 $v', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['kernels_ms_per_step'].items() if k != 'note'})"
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || \
  { tail -n 60 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_gpu_tests.log
