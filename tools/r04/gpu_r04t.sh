#!/bin/bash
# Round 4, call t: where the fused decode's waves spend their cycles (timing
# build build/ab/diagt.so, -DDQDK_DIAG_TIMING: s_memtime sums of phase A and
# of the round flushes per wave, printed at queue destroy), 1500 / 9000 B.
# usage (on the GPU box): bash tools/r04/gpu_r04t.sh <tag>
set -e
tag=${1:-r04t}
mkdir -p gpurun_out
for L in 1500 9000; do
    DQDK_GPU_LIB=$PWD/build/ab/diagt.so timeout -k 10 200 python3 bench.py --frame-len $L --no-9000 --no-cpu-baseline \
        --no-box-state --steps 16 > gpurun_out/diagt_${tag}_$L.json 2> gpurun_out/diagt_${tag}_$L.err
    grep diag_timing gpurun_out/diagt_${tag}_$L.err || true
done
