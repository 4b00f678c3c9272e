#!/bin/bash
# Bench lines for BASELINE.json's other single-GPU configs:
# configs[1] (256K x 1500 B, parse + checksum only) and configs[3]'s frame
# mix (1M frames, 1500/9000 B by a seeded coin flip), plus rocprof stats of the mix.
# usage (on the GPU box): bash tools/gpu_configs.sh <tag>
set -e
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --frames 262144 --no-histo --no-records --cpu-baseline-sec 5 \
    > gpurun_out/bench_${tag}_cfg1_parse.json 2> gpurun_out/bench_${tag}_cfg1_parse.err
timeout -k 10 300 python3 bench.py --frame-len 9000 --frames 262144 --cpu-baseline-sec 5 \
    > gpurun_out/bench_${tag}_cfg2_9000_256k.json 2> gpurun_out/bench_${tag}_cfg2_9000_256k.err
timeout -k 10 300 python3 bench.py --frame-len 0 --cpu-baseline-sec 5 \
    > gpurun_out/bench_${tag}_mixed.json 2> gpurun_out/bench_${tag}_mixed.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_mixed -o run --output-format csv -- \
    python3 bench.py --frame-len 0 --no-cpu-baseline > gpurun_out/prof_${tag}_mixed.log 2>&1
