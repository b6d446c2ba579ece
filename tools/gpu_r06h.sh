set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u bench.py > gpurun_out/r06t_bench.json 2> gpurun_out/r06t_bench.err || exit 1
python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06t_bench.json').read().strip().splitlines()[-1]); e=d['e2e_run_to_qvalues']; print({k: round(v*1e3,2) for k,v in e.items() if isinstance(v,float)}, [round(x,3) for x in e['runs_total_s']]); print(d['value']/1e6, d['e2e_cfg3_run_to_qvalues']['total_s'])"
