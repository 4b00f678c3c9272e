#!/bin/bash
# Round 5, call z4: fused policy 3 (whole-line flushes, non-temporal frame
# loads) as the default from 128 events per frame = the in-tree build:
#   1. the -m gpu suite on it;
#   2. interleaved 9000 B bench runs against HEAD (head), three rounds.
# usage (on the GPU box): bash tools/r05/gpu_r05z4.sh <tag>
set -e
tag=${1:-r05z4}
mkdir -p gpurun_out/ab_${tag}_9000
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
for r in 1 2 3; do
    for v in head wt; do
        DQDK_GPU_LIB=$PWD/build/ab/$v.so timeout -k 10 200 python3 bench.py --frame-len 9000 --steps 10 \
            --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_9000/${v}_$r.json \
            2> gpurun_out/ab_${tag}_9000/${v}_$r.err
    done
done
