#!/bin/bash
# Round-3 end measurement: PMC passes (both frame sizes) into the bench's
# traffic summary, the default bench line reading it, rocprof kernel stats.
set -e
mkdir -p gpurun_out
cp profiles/pmc_summary.json gpurun_out/pmc_summary.json
bash tools/pmc.sh r03 1500
bash tools/pmc.sh r03 9000
timeout -k 10 400 python3 bench.py --pmc gpurun_out/pmc_summary.json > gpurun_out/bench_r03.json 2> gpurun_out/bench_r03.err
bash tools/prof.sh r03
