#!/bin/bash
# PMC traffic for the non-default bench configs (tools/gpu_configs.sh), merged
# into a copy of profiles/pmc_summary.json, then their bench lines with it.
# usage (on the GPU box): bash tools/gpu_configs_pmc.sh <tag>
set -e
tag=${1:-run}
mkdir -p gpurun_out
cp profiles/pmc_summary.json gpurun_out/pmc_summary.json
FRAMES=262144 bash tools/pmc.sh ${tag}_cfg1 1500 --no-histo --no-records
FRAMES=262144 bash tools/pmc.sh ${tag}_cfg2 9000
bash tools/pmc.sh ${tag}_mixed 0
P=gpurun_out/pmc_summary.json
timeout -k 10 300 python3 bench.py --frames 262144 --no-histo --no-records --cpu-baseline-sec 5 --pmc $P \
    > gpurun_out/bench_${tag}_cfg1_parse.json 2> gpurun_out/bench_${tag}_cfg1_parse.err
timeout -k 10 300 python3 bench.py --frame-len 9000 --frames 262144 --cpu-baseline-sec 5 --pmc $P \
    > gpurun_out/bench_${tag}_cfg2_9000_256k.json 2> gpurun_out/bench_${tag}_cfg2_9000_256k.err
timeout -k 10 300 python3 bench.py --frame-len 0 --cpu-baseline-sec 5 --pmc $P \
    > gpurun_out/bench_${tag}_mixed.json 2> gpurun_out/bench_${tag}_mixed.err
