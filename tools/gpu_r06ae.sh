set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_lib.sh -r 3 "sl:: sl0:sl0:" > gpurun_out/r06ae_ab.txt 2>&1 || exit 1
cat gpurun_out/r06ae_ab.txt
timeout -k 10 900 python3 -u bench.py > gpurun_out/r06ae_bench.json 2> gpurun_out/r06ae_bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r06ae_bench.json').read().strip().splitlines()[-1]); e=d['e2e_run_to_qvalues']; c=d['e2e_cfg3_run_to_qvalues']; f=lambda e: {k: (round(v*1e3,1) if isinstance(v,float) else v) for k,v in e.items() if k not in ('note','first_run')}; print(round(d['value']/1e6,1), f(e)); print(f(c))"
