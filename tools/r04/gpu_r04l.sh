#!/bin/bash
# Round 4, call l: where the first-line hand-off's time goes (timing builds,
# same box, interleaved): cur = the hand-off (policy 6) and the round-4
# default (policy 2) from one build; shnone = the hand-off geometry with
# phase B reading the straddling dword itself; shload0 = the register dword
# shifted in but lane 0 loading at the grid offset (wrong bytes: timing only).
# usage (on the GPU box): bash tools/r04/gpu_r04l.sh <tag>
set -e
tag=${1:-r04l}
mkdir -p gpurun_out/ab_$tag
b="--no-9000 --no-box-state --no-cpu-baseline --steps 16 --warmup 2"
for r in 1 2; do
    for v in "cur 6" "cur 2" "shnone 6" "shload0 6"; do
        set -- $v
        DQDK_GPU_LIB=$PWD/build/ab/$1.so DQDK_GPU_FUSED_POLICY=$2 timeout -k 10 200 python3 bench.py $b \
            > gpurun_out/ab_$tag/$1_p$2_$r.json 2>> gpurun_out/ab_$tag/err.log
    done
done
