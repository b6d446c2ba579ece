# class end to end (cfg2 + cfg3 from files): reader-thread nice A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for spec in n0:H3D_READER_NICE=0 n5:H3D_READER_NICE=5 n15:H3D_READER_NICE=15; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-other-configs --no-cpu-cfg3 --no-peaks > gpurun_out/r06ad_$name$rep.json 2> gpurun_out/r06ad_$name$rep.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r06ad_$name$rep.json').read().strip().splitlines()[-1]); e=d['e2e_run_to_qvalues']; c=d['e2e_cfg3_run_to_qvalues']; f=lambda e: {k: round(v*1e3,1) for k,v in e.items() if isinstance(v,float)}; print('$name', f(e), f(c))"
done
done
