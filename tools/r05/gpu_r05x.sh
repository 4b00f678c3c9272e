#!/bin/bash
# Round 5, call x: more streaming -- the slice gather's loads (snt:
# DQDK_SLICE_LD_AUX=2) at both sizes, and at 9000 B the frames streamed too
# (fused policy 3 = lines + non-temporal loads, A/B build wt) -- against the
# tree's defaults (wt).
# usage (on the GPU box): bash tools/r05/gpu_r05x.sh <tag>
set -e
tag=${1:-r05x}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000
run() {  # size name lib env...
    local L=$1 v=$2 lib=$3; shift 3
    env DQDK_GPU_LIB=$PWD/build/ab/$lib.so "$@" timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 \
        --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/$v.json \
        2> gpurun_out/ab_${tag}_$L/$v.err
}
for r in 1 2; do
    run 1500 wt_$r wt X=0
    run 1500 snt_$r snt X=0
    run 9000 wt_$r wt X=0
    run 9000 snt_$r snt X=0
    run 9000 p3_$r wt DQDK_GPU_FUSED_POLICY=3
done
