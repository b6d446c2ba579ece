#!/bin/bash
# locate the pending HIP error behind test_gpu_cfg3's h3d_lrt failure: the
# test on each library variant / mode, H3D_DEBUG on
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for spec in "cur::" "cur:H3D_BRENT=0:" "dual::" "nopre::"; do
  v=${spec%%:*}; rest=${spec#*:}; e=${rest%%:*}
  lib=$PWD/hic3defdr_amd/lib/libh3d.so
  [ "$v" != cur ] && lib=$PWD/hic3defdr_amd/lib/variants/libh3d_$v.so
  echo "== $v $e"
  env $e H3D_DEBUG=1 H3D_LIB=$lib timeout -k 10 240 python3 -u -m pytest tests/test_gpu_cfg3.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/${tag}_${v}_$e.log 2>&1
  rc=$?
  echo "rc=$rc"; grep -E "pending|passed|failed|H3DError" gpurun_out/${tag}_${v}_$e.log | head -5
  case $rc in 124|134|137|139) exit $rc;; esac
done
