#!/bin/bash
# Round 4, call k: the first-line hand-off with the straddling dword carried
# in a register (policy 6) against the round-4 default (2), folded counters
# on, same box, twice; its parity tests first; PMC traffic of policy 6.
# usage (on the GPU box): bash tools/r04/gpu_r04k.sh <tag>
set -e
tag=${1:-r04k}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused_head.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_${tag}_head.log 2>&1
b="--no-9000 --no-box-state --no-cpu-baseline"
for r in 1 2; do
    for p in 6 2; do
        DQDK_GPU_FUSED_POLICY=$p timeout -k 10 300 python3 bench.py $b > gpurun_out/ab_${tag}_1500_p${p}_$r.json \
            2>> gpurun_out/ab_$tag.err
    done
done
cp profiles/pmc_summary.json gpurun_out/pmc_summary.json
DQDK_GPU_FUSED_POLICY=6 bash tools/pmc.sh $tag 1500
