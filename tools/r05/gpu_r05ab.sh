#!/bin/bash
# Round 5, call ab: rx_part2 loads item i + 2's piece starts at the end of
# item i - 1 (in flight with item i + 1's triples), not after item i's cursor
# barrier = the in-tree build and build/ab/wt.so, against HEAD (head).
#   1. the -m gpu suite on the in-tree build;
#   2. interleaved bench runs, both sizes, three rounds.
# usage (on the GPU box): bash tools/r05/gpu_r05ab.sh <tag>
set -e
tag=${1:-r05ab}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
for r in 1 2 3; do
    for L in 1500 9000; do
        for v in head wt; do
            DQDK_GPU_LIB=$PWD/build/ab/$v.so timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 \
                --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/${v}_$r.json \
                2> gpurun_out/ab_${tag}_$L/${v}_$r.err
        done
    done
done
