#!/bin/bash
# Round 5, call i: double-buffered decode rounds (fused policy 10, A/B build
# wt: two 67-key stage halves, one streamed into while the other is flushed
# between the windows) against HEAD (head) and wt's default policy.
#   1. parity of policy 10 on every fused-path test, launches and copies
#      serialised (a fault names its operation);
#   2. the A/B variants' own edge-frame tests on wt (policies 1, 2, 10, ...);
#   3. interleaved bench runs: head, wt, wt at policy 10 (1500 B), and
#      head / wt at 9000 B.
# usage (on the GPU box): bash tools/r05/gpu_r05i.sh <tag>
set -e
tag=${1:-r05i}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
DQDK_GPU_LIB=$PWD/build/ab/wt.so DQDK_GPU_FUSED_POLICY=10 AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 \
    timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py \
    tests/test_gpu_fused_head.py tests/test_gpu_pinned.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "not handoff and not frame_maps" > gpurun_out/pytest_${tag}_db.log 2>&1
DQDK_GPU_LIB=$PWD/build/ab/wt.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fused_head.py -m gpu -x -q \
    --timeout 240 --timeout-method thread > gpurun_out/pytest_${tag}_variants.log 2>&1
for r in 1 2; do
    for v in head wt wt_db; do
        lib=${v%_db}; env=""
        [ "$v" = wt_db ] && env="DQDK_GPU_FUSED_POLICY=10"
        env DQDK_GPU_LIB=$PWD/build/ab/$lib.so $env timeout -k 10 200 python3 bench.py --frame-len 1500 --steps 10 \
            --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_1500/${v}_$r.json \
            2> gpurun_out/ab_${tag}_1500/${v}_$r.err
    done
    for v in head wt; do
        DQDK_GPU_LIB=$PWD/build/ab/$v.so timeout -k 10 200 python3 bench.py --frame-len 9000 --steps 10 \
            --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_9000/${v}_$r.json \
            2> gpurun_out/ab_${tag}_9000/${v}_$r.err
    done
done
