#!/bin/bash
# Round 5, call q: the first-line hand-off (fused policy 6: phase A decodes
# the events of each frame's first 128 B, phase B never re-reads that line)
# on the packed stage -- the A/B build of the tree (wt), policy 2 vs 6 at
# 1500 B, interleaved, three rounds.
# usage (on the GPU box): bash tools/r05/gpu_r05q.sh <tag>
set -e
tag=${1:-r05q}
mkdir -p gpurun_out/ab_${tag}_1500
for r in 1 2 3; do
    for p in 2 6; do
        DQDK_GPU_LIB=$PWD/build/ab/wt.so DQDK_GPU_FUSED_POLICY=$p timeout -k 10 200 python3 bench.py --frame-len 1500 \
            --steps 10 --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_1500/p${p}_$r.json \
            2> gpurun_out/ab_${tag}_1500/p${p}_$r.err
    done
done
