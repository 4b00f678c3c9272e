#!/bin/bash
# Quick GPU check: GPU tests + both bench lines (no profiler passes).
# usage: bash tools/gpu_quick.sh <tag>
set -e
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$tag.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_${tag}_1500.json 2> gpurun_out/bench_${tag}_1500.err
timeout -k 10 300 python3 bench.py --frame-len 9000 --no-cpu-baseline > gpurun_out/bench_${tag}_9000.json 2> gpurun_out/bench_${tag}_9000.err
