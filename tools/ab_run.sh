#!/bin/bash
# Same-box A/B: bench.py with each build/ab/<name>.so, interleaved rounds.
# usage: bash tools/ab_run.sh <tag> "<bench args>" name1 name2 ...
set -e
tag=$1; bargs=$2; shift 2
mkdir -p gpurun_out/ab_$tag
for r in 1 2; do
    for n in "$@"; do
        DQDK_GPU_LIB=$PWD/build/ab/$n.so timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline $bargs \
            > gpurun_out/ab_$tag/${n}_$r.json 2> gpurun_out/ab_$tag/${n}_$r.err
    done
done
