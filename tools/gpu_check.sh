#!/bin/bash
# GPU tests then one bench line per frame size (no profiling).
# usage (on the GPU box): bash tools/gpu_check.sh <tag>
set -e
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$tag.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_${tag}_1500.json 2> gpurun_out/bench_${tag}_1500.err
timeout -k 10 300 python3 bench.py --frame-len 9000 --no-cpu-baseline > gpurun_out/bench_${tag}_9000.json 2> gpurun_out/bench_${tag}_9000.err
