#!/bin/bash
# Round 4, call b: the new full-size / configs / harness tests first (verbose,
# with the 8-queue test's latency line), then the rest of the -m gpu suite,
# the drop-in latency sweep and the default bench line (with box_state).
# usage (on the GPU box): bash tools/r04/gpu_r04b.sh <tag>
set -e
tag=${1:-r04b}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_c_harness.py \
    -m gpu -x -v -s --timeout 240 --timeout-method thread > gpurun_out/pytest_new_$tag.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    --deselect tests/test_gpu_fullsize.py --deselect tests/test_gpu_configs.py --deselect tests/test_c_harness.py \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
timeout -k 10 600 python3 -u tools/dropin_latency.py --out gpurun_out/dropin_$tag.jsonl > gpurun_out/dropin_$tag.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
