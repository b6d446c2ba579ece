set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export H3D_DEVICE=0 OMP_NUM_THREADS=1 TORCH_DISTRIBUTED_DEBUG=DETAIL H3D_DEBUG=1
timeout -k 10 120 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 --redirects 3 --log-dir gpurun_out/distlogs tests/dist_product_main.py small2 /tmp/h3dout > gpurun_out/dist_run.log 2>&1 || { echo FAILED; tail -50 gpurun_out/dist_run.log; find gpurun_out/distlogs -name "*.log" | xargs tail -30; exit 1; }
tail -20 gpurun_out/dist_run.log
