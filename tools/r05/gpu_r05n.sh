#!/bin/bash
# Round 5, call n: with the packed stage, each size under the other size's
# flush policy (1 = whole 128-B lines, 2 = whole words) at a few fills;
# the in-tree build, interleaved, two rounds.
# usage (on the GPU box): bash tools/r05/gpu_r05n.sh <tag>
set -e
tag=${1:-r05n}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
run() {  # size name env...
    local L=$1 v=$2; shift 2
    env "$@" timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 --warmup 2 --no-cpu-baseline \
        --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/$v.json 2> gpurun_out/ab_${tag}_$L/$v.err
}
for r in 1 2; do
    run 1500 def_$r X=0
    run 1500 p1f70_$r DQDK_GPU_FUSED_POLICY=1 DQDK_GPU_FUSED_FILL=70
    run 1500 p1f80_$r DQDK_GPU_FUSED_POLICY=1 DQDK_GPU_FUSED_FILL=80
    run 9000 def_$r X=0
    run 9000 p2f65_$r DQDK_GPU_FUSED_POLICY=2 DQDK_GPU_FUSED_FILL=65
    run 9000 p2f75_$r DQDK_GPU_FUSED_POLICY=2 DQDK_GPU_FUSED_FILL=75
done
