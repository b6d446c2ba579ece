set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
for v in "old H3D_PREP_AHEAD=1 H3D_NPZ_PINNED=0 H3D_REAP_MADVISE=0" "a1 H3D_PREP_AHEAD=1" "a2 H3D_PREP_AHEAD=2" "a3 H3D_PREP_AHEAD=3"; do
  set -- $v; name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/run_e2e.py > gpurun_out/r06m_$name.json 2> gpurun_out/r06m_$name.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['run_to_qvalues_s'],3), {k: round(v,3) for k,v in d['stages'].items()})" gpurun_out/r06m_$name.json $name
done
done
