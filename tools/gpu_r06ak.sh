set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_lib.sh -r 1 -p "bkt::H3D_BUCKET_SORT=1" > gpurun_out/r06ak_ab.txt 2>&1 || exit 1
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/ab_bkt_kernel_stats.csv')))
for r in rows:
    if 'bkt' in r['Name'] or 'gather_pack2' in r['Name'] or 'keys_pack2' in r['Name']:
        print('%-60s %5s %9.1f %8.1f' % (r['Name'][:60], r['Calls'], float(r['TotalDurationNs'])/1e3, float(r['AverageNs'])/1e3))
PY
