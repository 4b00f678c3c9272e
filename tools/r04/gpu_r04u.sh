#!/bin/bash
# Round 4, call u: the ring-buffer stage (no carry copies in the flush):
# every GPU test on it, then same-box A/B against the previous commit (base)
# at 1500 B and 9000 B, whole-line flushes at 1500 B on the ring, and the
# timing build's cycle shares.
# usage (on the GPU box): bash tools/r04/gpu_r04u.sh <tag>
set -e
tag=${1:-r04u}
mkdir -p gpurun_out/ab_$tag
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
b="--no-9000 --no-box-state --no-cpu-baseline"
for r in 1 2; do
    for n in base ring; do
        DQDK_GPU_LIB=$PWD/build/ab/$n.so timeout -k 10 200 python3 bench.py $b > gpurun_out/ab_$tag/${n}_1500_$r.json \
            2>> gpurun_out/ab_$tag/err.log
        DQDK_GPU_LIB=$PWD/build/ab/$n.so timeout -k 10 200 python3 bench.py --frame-len 9000 $b \
            > gpurun_out/ab_$tag/${n}_9000_$r.json 2>> gpurun_out/ab_$tag/err.log
    done
    DQDK_GPU_LIB=$PWD/build/ab/ring.so DQDK_GPU_FUSED_POLICY=3 DQDK_GPU_FUSED_FILL=46 timeout -k 10 200 python3 bench.py $b \
        > gpurun_out/ab_$tag/ringlines_1500_$r.json 2>> gpurun_out/ab_$tag/err.log
done
for L in 1500 9000; do
    DQDK_GPU_LIB=$PWD/build/ab/diagt.so timeout -k 10 200 python3 bench.py --frame-len $L $b --steps 16 \
        > gpurun_out/ab_$tag/diagt_$L.json 2> gpurun_out/ab_$tag/diagt_$L.err
    grep diag_timing gpurun_out/ab_$tag/diagt_$L.err || true
done
