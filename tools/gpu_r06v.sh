# class e2e after the stream-only syncs: stamps (no flush) + bench e2e legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/class_stamps.py --runs 3 --no-flush > gpurun_out/r06v_stamps_noflush.json 2> gpurun_out/r06v_stamps.err || exit 1
for k in 1 2; do
timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-other-configs --no-cpu-cfg3 --no-peaks > gpurun_out/r06v_e2e$k.json 2> gpurun_out/r06v_e2e$k.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r06v_e2e$k.json').read().strip().splitlines()[-1]); e=d['e2e_run_to_qvalues']; c=d['e2e_cfg3_run_to_qvalues']; f=lambda e: {k: round(v*1e3,2) for k,v in e.items() if isinstance(v,float)}; print('e2e$k', f(e), [round(x,3) for x in e['runs_total_s']], f(c))"
done
H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_bclk.so timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-other-configs --no-peaks > gpurun_out/r06v_bclk.json 2> gpurun_out/r06v_bclk.err || exit 1
grep brent_clk_wave gpurun_out/r06v_bclk.err | tail -1
