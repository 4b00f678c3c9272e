#!/bin/bash
# Round 4, call p: whole-line flushes at 1500 B with rounds small enough for
# their carries (fill 46 % -> 12 windows, 40 % -> 8) against the default
# (triples, 16 windows), same box, twice; plus PMC writes of the best guess.
# usage (on the GPU box): bash tools/r04/gpu_r04p.sh <tag>
set -e
tag=${1:-r04p}
mkdir -p gpurun_out/ab_$tag
b="--no-9000 --no-box-state --no-cpu-baseline"
for r in 1 2; do
    for v in "2 61" "3 46" "3 40" "1 46"; do
        set -- $v
        DQDK_GPU_FUSED_POLICY=$1 DQDK_GPU_FUSED_FILL=$2 timeout -k 10 200 python3 bench.py $b \
            > gpurun_out/ab_$tag/p$1_f$2_$r.json 2>> gpurun_out/ab_$tag/err.log
    done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
DQDK_GPU_FUSED_POLICY=3 DQDK_GPU_FUSED_FILL=46 timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/ab_$tag/pmcw -o run \
    --output-format csv -- python3 bench.py --steps 3 --warmup 1 $b > gpurun_out/ab_$tag/pmcw.log 2>&1
