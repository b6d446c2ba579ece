set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_bclk.so timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-other-configs --no-peaks > gpurun_out/r06s_bclk.json 2> gpurun_out/r06s_bclk.err || exit 1
grep brent_clk gpurun_out/r06s_bclk.err | tail -3
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_r06s_lds -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-other-configs --no-peaks > gpurun_out/pmc_r06s_lds.log 2>&1 || exit 1
f=$(find gpurun_out/pmc_r06s_lds -name '*counter_collection.csv' -print -quit)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name'][:60]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in agg.items():
    if 'brent' in k or 'disp_work' in k or 'k_lrt' in k:
        print(k, dict(v))
PY
cp "$f" gpurun_out/pmc_r06s_lds.csv; rm -rf gpurun_out/pmc_r06s_lds
