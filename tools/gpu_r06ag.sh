# class end to end: NPZ CRC threads A/B with the cgroup's throttled time
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max 2>/dev/null
for rep in 1 2; do
for spec in crc8:H3D_NPZ_CRC_THREADS=8 crc1:H3D_NPZ_CRC_THREADS=1; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-other-configs --no-cpu-cfg3 --no-peaks > gpurun_out/r06ag_$name$rep.json 2> gpurun_out/r06ag_$name$rep.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r06ag_$name$rep.json').read().strip().splitlines()[-1]); e=d['e2e_run_to_qvalues']; c=d['e2e_cfg3_run_to_qvalues']; f=lambda e: {k: (round(v*1e3,1) if isinstance(v,float) else v) for k,v in e.items() if k not in ('note','first_run','runs_total_s','gc_collections','write_genome_s','chromosomes')}; print('$name', f(e)); print('$name', f(c))"
done
done
