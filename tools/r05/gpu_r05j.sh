#!/bin/bash
# Round 5, call j: the next round's first windows touched into L2 (LDS-DMA
# loads into a junk word block, no VGPRs) before each round flush, so the
# ring restarts from L2 after it -- A/B builds t4 / t8 (DQDK_TOUCH=4 / 8
# windows) against HEAD (head).
#   1. fused-path parity of t8;
#   2. interleaved bench runs, both sizes, two rounds.
# usage (on the GPU box): bash tools/r05/gpu_r05j.sh <tag>
set -e
tag=${1:-r05j}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
DQDK_GPU_LIB=$PWD/build/ab/t8.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py \
    tests/test_gpu_parity.py tests/test_gpu_fused_head.py -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_${tag}_t8.log 2>&1
for r in 1 2; do
    for L in 1500 9000; do
        for v in head t4 t8; do
            DQDK_GPU_LIB=$PWD/build/ab/$v.so timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 \
                --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/${v}_$r.json \
                2> gpurun_out/ab_${tag}_$L/${v}_$r.err
        done
    done
done
