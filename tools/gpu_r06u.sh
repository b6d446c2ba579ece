# e2e legs of bench.py only, host knobs A/B (estimate_disp through the class)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for spec in base: pin0:H3D_NPZ_PINNED=0 ahead0:H3D_PREP_AHEAD=0; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-other-configs --no-cpu-cfg3 --no-peaks > gpurun_out/r06u_$name.json 2> gpurun_out/r06u_$name.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r06u_$name.json').read().strip().splitlines()[-1]); e=d['e2e_run_to_qvalues']; c=d['e2e_cfg3_run_to_qvalues']; f=lambda e: {k: round(v*1e3,2) for k,v in e.items() if isinstance(v,float)}; print('$name', f(e), [round(x,3) for x in e['runs_total_s']], f(c))"
done
