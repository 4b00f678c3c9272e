#!/bin/bash
# rocprofv3 kernel-trace summaries of the bench command for both frame sizes.
# usage (on the GPU box): bash tools/prof.sh <tag>
set -e
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_1500 -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-9000 > gpurun_out/prof_${tag}_1500.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_9000 -o run --output-format csv -- \
    python3 bench.py --frame-len 9000 --no-cpu-baseline > gpurun_out/prof_${tag}_9000.log 2>&1
