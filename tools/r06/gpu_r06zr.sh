#!/bin/bash
# r06zr: the final tree's 2-rank shared-GPU rehearsal, launched as the driver
# launches N > 1 (torchrun, default steps and CPU baseline), each rank
# dumping its stack every 60 s if it stalls.
set -e
tag=${1:-r06zr}
mkdir -p gpurun_out
export DQDK_BENCH_WATCHDOG=60
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29519 bench.py --gpus 2 --share-gpu --no-configs > gpurun_out/bench_2rank_$tag.json \
    2> gpurun_out/bench_2rank_$tag.err
