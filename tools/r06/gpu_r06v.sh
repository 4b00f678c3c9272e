#!/bin/bash
# r06v: phase A's header loads non-temporal (-DDQDK_PHA_NT=1) vs plain:
# same-box A/B at 1500 and 9000 B, then PMC traffic of each variant (1500 B).
set -e
tag=${1:-r06v}
mkdir -p gpurun_out
bash tools/ab_run.sh phant_$tag "--no-9000 --no-configs --no-box-state" base phant
bash tools/ab_run.sh phant9_$tag "--frame-len 9000 --no-configs --no-box-state" base phant
for n in base phant; do
    DQDK_GPU_LIB=$PWD/build/ab/$n.so bash tools/pmc.sh ${tag}_$n 1500 --no-configs --no-box-state
done
