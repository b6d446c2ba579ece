#!/bin/bash
# The GPU-box recipes of the measurements DESIGN.md cites, one entry point:
#   tools/gpu_runs.sh <recipe> <tag> [args]      (on the box, via gpurun)
# recipes:
#   final    rocprofv3 kernel stats + trace gaps of the default bench command
#            (tools/gpu_prof_step.sh), its PMC passes (tools/pmc_passes.sh),
#            then the full default bench line -> gpurun_out/<tag>_bench.json
#            (r06f, r06g; tools/pmc_default.py <tag> profiles/r06/<x> then
#            makes the summary the bench's default)
#   suite    the -m gpu suite and smoke() (tools/gpu_suite.sh)
#   ab       interleaved A/B of libh3d variants / H3D_* knobs on cfg2
#            (tools/ab_lib.sh "<specs>"; args: -r reps -p ...), then the suite
#   e2e      the bench's end-to-end legs only (cfg2 + cfg3 from files), for
#            each "name:ENV=VAL" spec in $3, $4 reps (r06u, r06x, r06ad, r06ag)
#   n2       the driver's N = 2 command rehearsed over gloo on one GPU
# Round-6 runs (the variants they compared were removed
# once measured): r06r tail prefetch A/B, r06s / r06v / r06w H3D_BRENT_CLOCK
# builds, r06w / r06y / r06z / r06aa / r06ae / r06ah / r06al kernel A/Bs,
# r06aj / r06ak bucket sort, r06x NUMA binding, r06ac prepare_data profile.
set -o pipefail
recipe=${1:?recipe}
tag=${2:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
case $recipe in
  final)
    bash tools/gpu_prof_step.sh "$tag" > gpurun_out/${tag}_top.txt 2>&1 || exit 1
    bash tools/pmc_passes.sh "$tag" || exit 1
    timeout -k 10 900 python3 -u bench.py > gpurun_out/${tag}_bench.json \
      2> gpurun_out/${tag}_bench.err || exit 1
    head -12 gpurun_out/${tag}_top.txt ;;
  suite)
    bash tools/gpu_suite.sh "$tag" ;;
  ab)
    shift 2
    bash tools/ab_lib.sh "$@" > gpurun_out/${tag}_ab.txt 2>&1 || \
      { cat gpurun_out/${tag}_ab.txt; exit 1; }
    cat gpurun_out/${tag}_ab.txt
    bash tools/gpu_suite.sh "$tag" ;;
  e2e)
    specs=${3:?specs}; reps=${4:-2}
    for rep in $(seq "$reps"); do
      for spec in $specs; do
        name=${spec%%:*}; envs=${spec#*:}
        env $envs timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 \
          --no-cpu-baseline --no-other-configs --no-cpu-cfg3 --no-peaks \
          > gpurun_out/${tag}_$name$rep.json 2> gpurun_out/${tag}_$name$rep.err || exit 1
        python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_$name$rep.json').read().strip().splitlines()[-1]); f=lambda e: {k: (round(v*1e3,1) if isinstance(v,float) else v) for k,v in e.items() if k not in ('note','first_run','runs_total_s','gc_collections')}; print('$name', f(d['e2e_run_to_qvalues'])); print('$name', f(d['e2e_cfg3_run_to_qvalues']))"
      done
    done ;;
  n2)
    bash tools/gpu_n2_rehearsal.sh "$tag" ;;
  *) echo "unknown recipe $recipe"; exit 2 ;;
esac
