# 2 ranks on the box's one GPU (gloo for the barrier/all-reduce): the bench's
# multi-process path end to end.  The 8-GPU run is the driver's (RCCL).
set -e
mkdir -p gpurun_out
MM2G_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu \
  > gpurun_out/mr2.json 2> gpurun_out/mr2.err
