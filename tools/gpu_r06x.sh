# cfg2 end to end through the class, NUMA binding A/B (interleaved processes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2 3; do
for spec in bind:H3D_NUMA_BIND=1 free:H3D_NUMA_BIND=0; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs --no-e2e-cfg3 --no-peaks > gpurun_out/r06x_$name$rep.json 2> gpurun_out/r06x_$name$rep.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r06x_$name$rep.json').read().strip().splitlines()[-1]); e=d['e2e_run_to_qvalues']; f=lambda e: {k: round(v*1e3,2) for k,v in e.items() if isinstance(v,float)}; print('$name', d.get('numa_bind'), round(d['value']/1e6,1), f(e), [round(x,3) for x in e['runs_total_s']])"
done
done
