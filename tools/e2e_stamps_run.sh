cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for b in 0 1; do
H3D_E2E_STAMPS=1 H3D_NUMA_BIND=$b timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-other-configs --no-e2e-cfg3 --no-peaks > gpurun_out/r06an_b$b.json 2> gpurun_out/r06an_b$b.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/r06an_b$b.json').read().strip().splitlines()[-1]); e=d['e2e_run_to_qvalues']
print('bind $b', round(e['estimate_disp_s']*1e3,1), [round(x,3) for x in e['runs_total_s']])
for st in e['estimate_disp_stamps_ms']: print('  ', {k:v for k,v in sorted(st.items(), key=lambda kv:-kv[1]) if v>0.2})
"
done
