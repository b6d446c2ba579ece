#!/bin/bash
# Interleaved A/B of (libh3d variant, environment) pairs -- the one runner for
# every measured comparison (library variants, the H3D_* knobs, cfg2 / cfg3 /
# cfg4). Each spec is name:lib:ENV=VAL[,ENV=VAL...]; lib = a variant built by
# hic3defdr_amd/build.py build_variant (lib/variants/libh3d_<lib>.so), empty
# for the default libh3d.so.
#   tools/ab_lib.sh [-c 2|3|4] [-r reps] [-s steps] [-t] [-p] "spec spec ..."
#     -c  workload: 2 = bench.py cfg2 (default), 3 / 4 = tools/run_cfg.py
#     -r  interleaved repetitions (default 2)
#     -s  timed steps per run (default 10 for cfg2, 2 for cfg3 / cfg4)
#     -t  then the -m gpu suite on the first spec (stops the script on a fail)
#     -p  each run under rocprofv3 --kernel-trace --stats (kernel stats kept
#         as gpurun_out/ab_<name>_kernel_stats.csv)
# Examples: tools/ab_lib.sh "base:base: cur:cur:"
#           tools/ab_lib.sh "w3::H3D_DISP_W=3 w4::H3D_DISP_W=4"
#           tools/ab_lib.sh -c 4 "s2::H3D_DISP_SORT=2 s0::H3D_DISP_SORT=0"
set -e
cfg=2; reps=2; steps=; tests=0; prof=0
while getopts "c:r:s:tp" o; do
  case $o in
    c) cfg=$OPTARG ;; r) reps=$OPTARG ;; s) steps=$OPTARG ;;
    t) tests=1 ;; p) prof=1 ;; *) exit 2 ;;
  esac
done
shift $((OPTIND - 1))
specs=${1:?"specs"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "$cfg" = 2 ]; then
  cmd="bench.py --no-cpu-baseline --no-e2e --no-other-configs --no-peaks --steps ${steps:-10}"
else
  cmd="tools/run_cfg.py --cfg $cfg --steps ${steps:-2} --warmup 1"
fi
first=
for rep in $(seq $reps); do
for sp in $specs; do
  name=${sp%%:*}; rest=${sp#*:}; lib=${rest%%:*}; envs=${rest#*:}
  first=${first:-$sp}
  libenv=
  [ -n "$lib" ] && libenv=H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_$lib.so
  if [ "$prof" = 1 ]; then
    env $(echo "$envs" | tr ',' ' ') $libenv timeout -k 10 400 rocprofv3 --kernel-trace --stats \
      --output-format csv -d gpurun_out/ab_${name}_prof -o run -- python3 -u $cmd \
      > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
    s=$(find gpurun_out/ab_${name}_prof -name '*kernel_stats.csv' -print -quit)
    cp "$s" gpurun_out/ab_${name}_kernel_stats.csv && rm -rf gpurun_out/ab_${name}_prof
  else
    env $(echo "$envs" | tr ',' ' ') $libenv timeout -k 10 400 python3 -u $cmd \
      > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  fi
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$name.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$name', round(d['value']/1e6,1), round(d['ms_per_step'],3), d.get('result_sha16'), {a: round(b,3) for a, b in k.items() if a != 'note'})" | tee -a gpurun_out/ab_summary.txt
done
done
if [ "$tests" = 1 ]; then
  name=${first%%:*}; rest=${first#*:}; lib=${rest%%:*}; envs=${rest#*:}
  libenv=
  [ -n "$lib" ] && libenv=H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_$lib.so
  env $(echo "$envs" | tr ',' ' ') $libenv timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rP \
    --timeout 300 --timeout-method thread > gpurun_out/ab_gpu_tests.log 2>&1 || \
    { tail -n 40 gpurun_out/ab_gpu_tests.log; exit 1; }
  tail -n 2 gpurun_out/ab_gpu_tests.log
fi
