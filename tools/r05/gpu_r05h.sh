#!/bin/bash
# Round 5, call h: the fused decode in two 8-wave blocks per CU (64-key
# stages, four buckets per flush store; their round flushes need not
# coincide) -- DQDK_GPU_FUSED_GEO=2 on the A/B build of the working tree
# (wt), which at the default geometry must equal HEAD (head).
#   1. the -m gpu suite on the in-tree build (default geometry);
#   2. interleaved bench runs: head, wt, wt at geometry 2, both sizes.
# (geometry 2's parity run, r05h first try: 101 fused-path tests green, then
# an illegal address reported at the next test's first copy -- see DESIGN §9)
# usage (on the GPU box): bash tools/r05/gpu_r05h.sh <tag>
set -e
tag=${1:-r05h}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
for r in 1 2; do
    for L in 1500 9000; do
        for v in head wt wt_geo2; do
            lib=${v%_geo2}; env=""
            [ "$v" = wt_geo2 ] && env="DQDK_GPU_FUSED_GEO=2 DQDK_GPU_FUSED_POLICY=2"
            env DQDK_GPU_LIB=$PWD/build/ab/$lib.so $env timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 \
                --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/${v}_$r.json \
                2> gpurun_out/ab_${tag}_$L/${v}_$r.err
        done
    done
done
