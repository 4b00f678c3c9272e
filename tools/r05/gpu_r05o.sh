#!/bin/bash
# Round 5, call o: where the packed-stage decode's time goes -- timing-only
# builds (tables wrong; tools/r05/r05o_diag.patch): noor = staged keys not
# OR-ed into the stage, nofl = round flushes drop the round's keys (no
# stores, no LDS work; barriers kept), noboth = both; against HEAD (head).
# usage (on the GPU box): bash tools/r05/gpu_r05o.sh <tag>
set -e
tag=${1:-r05o}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
for r in 1 2; do
    for L in 1500 9000; do
        for v in head noor nofl noboth; do
            DQDK_GPU_LIB=$PWD/build/ab/$v.so timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 \
                --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/${v}_$r.json \
                2> gpurun_out/ab_${tag}_$L/${v}_$r.err
        done
    done
done
