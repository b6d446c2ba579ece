set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/prep_profile.py --genome --runs 2 > gpurun_out/r06l_prep.json 2> gpurun_out/r06l_prep.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r06l_prep.json')); print({k: round(v['median_ms_per_run'],1) for k,v in d.items()})"
for rep in 1 2; do
for v in "old H3D_PREP_AHEAD=1 H3D_NPZ_PINNED=0 H3D_REAP_MADVISE=0" "new H3D_PREP_AHEAD=3"; do
  set -- $v; name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/run_e2e.py > gpurun_out/r06l_$name.json 2> gpurun_out/r06l_$name.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['run_to_qvalues_s'],3), {k: round(v,3) for k,v in d['stages'].items()}, 'collect', round(d['collect_s'],3))" gpurun_out/r06l_$name.json $name
done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_cfg1.py tests/test_gpu_cfg3.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r06l_tests.log 2>&1; tail -2 gpurun_out/r06l_tests.log
