#!/bin/bash
# Round 5, call k: rx_part2's per-phase cycles (s_memtime stamps at its
# barriers, diagnostic build p2t = DQDK_P2_TIMING=1), printed per launch by
# its last block, at both sizes; the same bench with head for the kernel's
# uninstrumented time.
# usage (on the GPU box): bash tools/r05/gpu_r05k.sh <tag>
set -e
tag=${1:-r05k}
mkdir -p gpurun_out/$tag
for L in 1500 9000; do
    for v in head p2t; do
        DQDK_GPU_LIB=$PWD/build/ab/$v.so timeout -k 10 200 python3 bench.py --frame-len $L --steps 5 \
            --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/$tag/${v}_$L.out \
            2> gpurun_out/$tag/${v}_$L.err
    done
done
