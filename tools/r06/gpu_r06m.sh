#!/bin/bash
# r06m: the 2-rank shared-GPU rehearsal (r06l went silent after both ranks'
# 9000 B warm-up and was killed): first in round 5's form (--steps 5, no CPU
# baseline), then the default form, each rank dumping its stack every 60 s
# (DQDK_BENCH_WATCHDOG) so a stall names its line.
set -e
tag=${1:-r06m}
mkdir -p gpurun_out
export DQDK_BENCH_WATCHDOG=60
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-box-state --share-gpu \
    --no-configs > gpurun_out/bench2a_$tag.json 2> gpurun_out/bench2a_$tag.err
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 2 --share-gpu --no-configs > gpurun_out/bench2b_$tag.json \
    2> gpurun_out/bench2b_$tag.err
