#!/bin/bash
# Round 5, call m: the packed stage's round size.  pk = the working tree
# (fill 70 at 1500 B: W = 28 windows; 65 at 9000 B: W = 16) against HEAD
# (head), and pk at fill 80 (W = 32) at 1500 B / fill 50 (W = 12) at 9000 B.
# usage (on the GPU box): bash tools/r05/gpu_r05m.sh <tag>
set -e
tag=${1:-r05m}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
for r in 1 2; do
    for L in 1500 9000; do
        alt=80; [ $L = 9000 ] && alt=50
        for v in head pk pk_alt; do
            lib=${v%_alt}; env=""
            [ "$v" = pk_alt ] && env="DQDK_GPU_FUSED_FILL=$alt"
            env DQDK_GPU_LIB=$PWD/build/ab/$lib.so $env timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 \
                --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/${v}_$r.json \
                2> gpurun_out/ab_${tag}_$L/${v}_$r.err
        done
    done
done
