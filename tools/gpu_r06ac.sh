set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
H3D_NUMA_BIND=1 timeout -k 10 400 python3 -u tools/prep_profile.py --genome --runs 3 --cprofile 40 > gpurun_out/r06ac_prep_genome.json 2> gpurun_out/r06ac_prep_genome.err || exit 1
cat gpurun_out/r06ac_prep_genome.json
