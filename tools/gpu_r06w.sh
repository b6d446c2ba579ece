set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_lib.sh -r 2 "prio:: prio0:prio0:" > gpurun_out/r06w_ab.txt 2>&1 || exit 1
H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_bclk.so timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-other-configs --no-peaks > gpurun_out/r06w_bclk.json 2> gpurun_out/r06w_bclk.err || exit 1
grep brent_clk gpurun_out/r06w_bclk.err | tail -2
