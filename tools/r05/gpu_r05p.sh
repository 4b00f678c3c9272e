#!/bin/bash
# Round 5, call p: a 5-window load ring (DQDK_FRINGW=5: one more window in
# flight across each round flush; rounds of 25 / 20 windows) against HEAD's
# 4 (head).
# usage (on the GPU box): bash tools/r05/gpu_r05p.sh <tag>
set -e
tag=${1:-r05p}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
for r in 1 2; do
    for L in 1500 9000; do
        for v in head r5; do
            DQDK_GPU_LIB=$PWD/build/ab/$v.so timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 \
                --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/${v}_$r.json \
                2> gpurun_out/ab_${tag}_$L/${v}_$r.err
        done
    done
done
