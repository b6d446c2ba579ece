#!/bin/bash
# Interleaved A/B of (library variant, environment) pairs on the default
# cfg2 bench (no CPU baseline, no e2e): each spec is name:lib:ENV=VAL[,..]
# with lib = hic3defdr_amd/lib/variants/libh3d_<lib>.so.
#   tools/ab_env.sh "base:base: cur:cur: plain:cur:H3D_BRENT=0" [reps]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
specs=$1
reps=${2:-2}
for rep in $(seq $reps); do
for sp in $specs; do
  name=${sp%%:*}; rest=${sp#*:}; lib=${rest%%:*}; envs=${rest#*:}
  env $(echo "$envs" | tr ',' ' ') H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_$lib.so \
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-e2e --no-other-configs --steps 10 \
    > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$name.json').read().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$name', round(d['value']/1e6,1), round(d['ms_per_step'],3), {a: round(b,3) for a, b in k.items() if a != 'note'})" | tee -a gpurun_out/ab_summary.txt
done
done
