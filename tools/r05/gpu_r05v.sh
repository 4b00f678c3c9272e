#!/bin/bash
# Round 5, call v: streaming (non-temporal) stores for the decode's pieces
# (fnt: DQDK_FST_AUX=2) and for rx_part2's output (pnt: DQDK_P2ST_AUX=2)
# against HEAD (head).
# usage (on the GPU box): bash tools/r05/gpu_r05v.sh <tag>
set -e
tag=${1:-r05v}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
for r in 1 2; do
    for L in 1500 9000; do
        for v in head fnt pnt; do
            DQDK_GPU_LIB=$PWD/build/ab/$v.so timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 \
                --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/${v}_$r.json \
                2> gpurun_out/ab_${tag}_$L/${v}_$r.err
        done
    done
done
