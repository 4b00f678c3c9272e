#!/bin/bash
# Round 5, call y: 9000 B under fused policy 3 (whole-line flushes with
# non-temporal frame loads) against policy 1 (temporal loads; the default),
# the A/B build of the tree, interleaved, three rounds -- a second box for
# r05x's p3 row.
# usage (on the GPU box): bash tools/r05/gpu_r05y.sh <tag>
set -e
tag=${1:-r05y}
mkdir -p gpurun_out/ab_${tag}_9000
for r in 1 2 3; do
    for p in 1 3; do
        DQDK_GPU_LIB=$PWD/build/ab/wt.so DQDK_GPU_FUSED_POLICY=$p timeout -k 10 200 python3 bench.py --frame-len 9000 \
            --steps 10 --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_9000/p${p}_$r.json \
            2> gpurun_out/ab_${tag}_9000/p${p}_$r.err
    done
done
