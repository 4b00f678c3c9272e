#!/bin/bash
# Round-end measurement on the GPU box: GPU tests, PMC passes (both frame
# sizes) merged into the bench's traffic summary, the default bench line
# (1500 B + 9000 B) reading that traffic, rocprof kernel stats of the bench.
# usage: bash tools/gpu_final.sh <tag>
set -e
tag=${1:-final}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$tag.log 2>&1
cp profiles/pmc_summary.json gpurun_out/pmc_summary.json
bash tools/pmc.sh $tag 1500
bash tools/pmc.sh $tag 9000
timeout -k 10 400 python3 bench.py --pmc gpurun_out/pmc_summary.json > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
bash tools/prof.sh $tag
