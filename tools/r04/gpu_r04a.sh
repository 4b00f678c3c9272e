#!/bin/bash
# Round 4, call a: the plugin (frame-processor) harness tests and the egress
# tests first, then the whole -m gpu suite, the drop-in latency sweep and the
# default bench line.  usage (on the GPU box): bash tools/r04/gpu_r04a.sh <tag>
set -e
tag=${1:-r04a}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_c_harness.py tests/test_gpu_egress.py -m gpu -x -v \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_fp_$tag.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    --deselect tests/test_c_harness.py --deselect tests/test_gpu_egress.py > gpurun_out/pytest_gpu_$tag.log 2>&1
timeout -k 10 600 python3 -u tools/dropin_latency.py --out gpurun_out/dropin_$tag.jsonl > gpurun_out/dropin_$tag.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
