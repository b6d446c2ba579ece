#!/bin/bash
# r04q: the one-log llr + grouped Halley A/B (llr vs mid), the prep sort
# A/B (H3D_DISP_SORT 2 vs 3 on the current library), cfg4 through run_cfg
# for the grouped LRT, then the whole GPU suite + smoke
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env.sh "llr:llr: mid:mid: s2:cur:H3D_DISP_SORT=2 s3:cur:H3D_DISP_SORT=3" 2 || exit 1
for v in llr mid; do
  H3D_LIB=$PWD/hic3defdr_amd/lib/variants/libh3d_$v.so timeout -k 10 400 python3 -u tools/run_cfg.py --cfg 4 \
    --steps 2 --warmup 1 > gpurun_out/r04q_cfg4_$v.json 2> gpurun_out/r04q_cfg4_$v.err || exit 1
done
bash tools/gpu_tests.sh r04q || exit $?
