#!/bin/bash
# Round 4, call i: the fused decode's first-line hand-off (policy bit 2).
#   its edge-case parity tests and the folded counters'; A/B on one box by
#   DQDK_GPU_FUSED_POLICY / DQDK_GPU_FOLD (1500 B: 6 = hand-off vs 2 =
#   round-4 default, folded counters vs rx_abort + rx_count, interleaved frame
#   map, twice; 9000 B: 5 vs 1, frame maps);
#   PMC traffic passes of the new default at 1500 B; then every GPU test.
# usage (on the GPU box): bash tools/r04/gpu_r04i.sh <tag>
set -e
tag=${1:-r04i}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused_head.py tests/test_gpu_egress.py -x -q --timeout 120 \
    --timeout-method thread \
    > gpurun_out/pytest_${tag}_head.log 2>&1
b="--no-9000 --no-box-state --no-cpu-baseline"
for r in 1 2; do
    for v in "6 1 0" "2 1 0" "6 0 0" "2 0 0"; do
        set -- $v
        DQDK_GPU_FUSED_POLICY=$1 DQDK_GPU_FOLD=$2 DQDK_GPU_FRAME_MAP=$3 timeout -k 10 300 python3 bench.py $b \
            > gpurun_out/ab_${tag}_1500_p$1_f$2_m$3_$r.json 2>> gpurun_out/ab_$tag.err
    done
done
for v in "5 0" "1 0"; do
    set -- $v
    DQDK_GPU_FUSED_POLICY=$1 DQDK_GPU_FRAME_MAP=$2 timeout -k 10 300 python3 bench.py --frame-len 9000 $b \
        > gpurun_out/ab_${tag}_9000_p$1_m$2.json 2>> gpurun_out/ab_$tag.err
done
cp profiles/pmc_summary.json gpurun_out/pmc_summary.json
bash tools/pmc.sh $tag 1500
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
