#!/bin/bash
# Packed-UMEM variant: frames at stride roundup(L, 128)
# instead of the UMEM chunk size, to separate the stride's cost from the kernel's.
# usage (on the GPU box): bash tools/gpu_packed.sh <tag>
set -e
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --stride 1536 --no-cpu-baseline > gpurun_out/bench_${tag}_packed_1500.json 2> gpurun_out/bench_${tag}_packed_1500.err
timeout -k 10 300 python3 bench.py --frame-len 9000 --stride 9088 --no-cpu-baseline > gpurun_out/bench_${tag}_packed_9000.json 2> gpurun_out/bench_${tag}_packed_9000.err
