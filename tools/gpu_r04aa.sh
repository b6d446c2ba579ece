#!/bin/bash
# r04aa: small launches dealt statically (no head probes) vs HEAD, cfg2 and
# the N = 8 rank share (its launches are small)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "head:head: small:small:" 3
for v in head small; do
  H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_$v.so H3D_BENCH_EMULATE=6/8 timeout -k 10 300 \
    python3 -u bench.py --config cfg3 --steps 5 --warmup 2 > gpurun_out/r04aa_emu_$v.json 2> gpurun_out/r04aa_emu_$v.err
done
