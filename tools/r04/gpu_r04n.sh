#!/bin/bash
# Round 4, call n: the first-line hand-off with phase A's keys staged in one
# LDS round trip (cur, policy 6) against policy 2 from the same build, and a
# timing build whose phase A drops those keys (noastage: where the hand-off's
# cost sits); same box, interleaved; the hand-off parity tests first.
# usage (on the GPU box): bash tools/r04/gpu_r04n.sh <tag>
set -e
tag=${1:-r04n}
mkdir -p gpurun_out/ab_$tag
DQDK_GPU_LIB=$PWD/build/ab/cur.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused_head.py -x -q \
    -k handoff --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
b="--no-9000 --no-box-state --no-cpu-baseline --steps 16 --warmup 2"
for r in 1 2; do
    for v in "cur 6" "cur 2" "noastage 6"; do
        set -- $v
        DQDK_GPU_LIB=$PWD/build/ab/$1.so DQDK_GPU_FUSED_POLICY=$2 timeout -k 10 200 python3 bench.py $b \
            > gpurun_out/ab_$tag/$1_p$2_$r.json 2>> gpurun_out/ab_$tag/err.log || true
    done
done
