#!/bin/bash
# Round 5, call ad: the slice pass gathers with two register sets in turn
# (group g + 1's loads in flight while group g is counted), two items per
# wave group (kNI 2: 61 VGPRs, no scratch; the kNI 3 form of call ac spilled),
# the low-byte plane loaded after the gather = the in-tree build and
# build/ab/wt.so, against HEAD (head).
#   1. interleaved bench runs, both sizes, three rounds;
#   2. the -m gpu suite on the in-tree build (last: call ac's suite hit an
#      illegal address surfacing at test_gpu_pinned's first copy).
# usage (on the GPU box): bash tools/r05/gpu_r05ad.sh <tag>
set -e
tag=${1:-r05ad}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
for r in 1 2 3; do
    for L in 1500 9000; do
        for v in head wt; do
            DQDK_GPU_LIB=$PWD/build/ab/$v.so timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 \
                --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/${v}_$r.json \
                2> gpurun_out/ab_${tag}_$L/${v}_$r.err
        done
    done
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
