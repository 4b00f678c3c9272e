#!/bin/bash
# Round 5, call r: the N-GPU bench path on the final tree, rehearsed as two
# ranks sharing the box's one GPU (--share-gpu: gloo, RCCL refuses two ranks on one device; the driver's 8-GPU
# node is not ours to launch) -- torchrun as the driver launches it.
# usage (on the GPU box): bash tools/r05/gpu_r05r.sh <tag>
set -e
tag=${1:-r05r}
mkdir -p gpurun_out
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-box-state --share-gpu \
    > gpurun_out/bench2_$tag.json 2> gpurun_out/bench2_$tag.err
