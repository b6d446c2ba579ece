#!/bin/bash
# The driver's N > 1 bench path (cfg3, strong scaling) rehearsed with 2 ranks
# on this one GPU over gloo (RCCL needs one GPU per rank): torchrun exactly
# as the driver launches it, plus H3D_DEVICE / H3D_BENCH_BACKEND.
#   tools/gpu_n2_rehearsal.sh <tag>
set -e
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
H3D_DEVICE=0 H3D_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 \
  bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/${tag}_n2.json 2> gpurun_out/${tag}_n2.err
tail -n 1 gpurun_out/${tag}_n2.json | cut -c1-600
