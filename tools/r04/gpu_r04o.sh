#!/bin/bash
# Round 4, call o: rx_part2's last block re-zeroes the slot's per-batch
# counters (no memset launch per batch): every GPU test, then A/B on one box
# against the memset form (DQDK_GPU_P2ZERO=0), 1500 B and 9000 B, twice.
# usage (on the GPU box): bash tools/r04/gpu_r04o.sh <tag>
set -e
tag=${1:-r04o}
mkdir -p gpurun_out/ab_$tag
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
b="--no-9000 --no-box-state --no-cpu-baseline"
for r in 1 2; do
    for z in 1 0; do
        DQDK_GPU_P2ZERO=$z timeout -k 10 200 python3 bench.py $b > gpurun_out/ab_$tag/z${z}_1500_$r.json \
            2>> gpurun_out/ab_$tag/err.log
    done
done
for z in 1 0; do
    DQDK_GPU_P2ZERO=$z timeout -k 10 200 python3 bench.py --frame-len 9000 $b > gpurun_out/ab_$tag/z${z}_9000.json \
        2>> gpurun_out/ab_$tag/err.log
done
