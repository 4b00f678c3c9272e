#!/bin/bash
# Round 5, call u: the next super-tile's descriptors (addr, len) loaded two
# ring steps before this one ends, so phase A starts with one dependent load
# fewer (dpf = DQDK_DESC_PF=1), and their header lines touched into L2 by
# LDS-DMA one step before (hpf = + DQDK_HDR_PF=1) against HEAD (head).
# usage (on the GPU box): bash tools/r05/gpu_r05u.sh <tag>
set -e
tag=${1:-r05u}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
DQDK_GPU_LIB=$PWD/build/ab/hpf.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py \
    tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
for r in 1 2; do
    for L in 1500 9000; do
        for v in head dpf hpf; do
            DQDK_GPU_LIB=$PWD/build/ab/$v.so timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 \
                --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/${v}_$r.json \
                2> gpurun_out/ab_${tag}_$L/${v}_$r.err
        done
    done
done
