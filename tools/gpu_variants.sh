#!/bin/bash
# Sensitivity sweep of the decode kernel: one bench line per variant.
# usage: bash tools/gpu_variants.sh <tag> [frame_len]
set -e
tag=${1:-run}; L=${2:-1500}
mkdir -p gpurun_out/var_$tag
i=0
while read -r name args; do
    i=$((i+1))
    timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 --warmup 2 --no-cpu-baseline $args \
        > gpurun_out/var_$tag/$name.json 2> gpurun_out/var_$tag/$name.err
done <<'LIST'
default
nohisto --no-histo
nocsum_nohisto --no-csum --no-histo
waveform --mode waveform
parse_only --mode waveform --no-csum
packed --stride 1536
LIST
