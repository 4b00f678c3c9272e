#!/bin/bash
# Round 4, call w: the final tree's default bench line (both legs, box state,
# CPU baseline) and the rocprofv3 kernel-trace summary of the same command.
# usage (on the GPU box): bash tools/r04/gpu_r04w.sh <tag>
set -e
tag=${1:-r04w}
mkdir -p gpurun_out/$tag
timeout -k 10 400 python3 bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$tag/prof -o run \
    -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/$tag/prof_bench.json \
    2> $GRAFT_REPO_ROOT/gpurun_out/$tag/prof.err
