#!/bin/bash
# Round 4, call j: rx_part2 with its ranks kept in registers from the count
# to the scatter (no LDS round trip; 94 VGPRs, one 16-wave block per CU:
# build/ab/p2rreg.so) against the working tree (build/ab/base.so), same box,
# interleaved, both frame sizes; its parity on the partitioned tests first.
# usage (on the GPU box): bash tools/r04/gpu_r04j.sh <tag>
set -e
tag=${1:-r04j}
mkdir -p gpurun_out
DQDK_GPU_LIB=$PWD/build/ab/p2rreg.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    -k "partitioned or fused or skewed" --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
bash tools/ab_run.sh ${tag}_1500 "--no-9000 --no-box-state" base p2rreg
bash tools/ab_run.sh ${tag}_9000 "--frame-len 9000 --no-9000 --no-box-state" base p2rreg
