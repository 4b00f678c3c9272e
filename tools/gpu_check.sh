#!/bin/bash
# One GPU call: the full -m gpu suite (new full-size / configs tests first),
# the default bench line and rocprof kernel stats of the 1500 B bench.
# usage (on the GPU box): bash tools/gpu_check.sh <tag>
set -e
tag=${1:-chk}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_configs.py -m gpu -x -v \
    --timeout 240 --timeout-method thread > gpurun_out/pytest_new_$tag.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    --deselect tests/test_gpu_fullsize.py --deselect tests/test_gpu_configs.py > gpurun_out/pytest_gpu_$tag.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_1500 -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-9000 > gpurun_out/prof_${tag}_1500.log 2>&1
