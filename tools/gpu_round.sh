#!/bin/bash
# One GPU-box session: GPU tests, bench lines, rocprof kernel stats, PMC.
# usage: bash tools/gpu_round.sh <tag> [skip-tests]
set -e
tag=${1:-run}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
    timeout -k 10 1200 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$tag.log 2>&1
fi
timeout -k 10 300 python3 bench.py > gpurun_out/bench_${tag}_1500.json 2> gpurun_out/bench_${tag}_1500.err
timeout -k 10 300 python3 bench.py --frame-len 9000 --cpu-baseline-sec 5 > gpurun_out/bench_${tag}_9000.json 2> gpurun_out/bench_${tag}_9000.err
bash tools/prof.sh $tag
bash tools/pmc.sh $tag 1500
bash tools/pmc.sh $tag 9000
