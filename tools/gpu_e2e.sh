#!/bin/bash
# PCIe-inclusive pipeline rates for DESIGN.md §7 (both frame sizes, both H2D forms, +records D2H).
# usage (on the GPU box): bash tools/gpu_e2e.sh <tag>
set -e
tag=${1:-run}
mkdir -p gpurun_out
o=gpurun_out/e2e_$tag.jsonl
: > $o
timeout -k 10 240 python3 tools/e2e_pipeline.py --frame-len 1500 --copy frames >> $o
timeout -k 10 240 python3 tools/e2e_pipeline.py --frame-len 1500 --copy frames --records --no-zero-copy >> $o
timeout -k 10 240 python3 tools/e2e_pipeline.py --frame-len 1500 --copy image --no-zero-copy >> $o
timeout -k 10 240 python3 tools/e2e_pipeline.py --frame-len 9000 --copy frames >> $o
timeout -k 10 240 python3 tools/e2e_pipeline.py --frame-len 9000 --copy frames --records --no-zero-copy >> $o
