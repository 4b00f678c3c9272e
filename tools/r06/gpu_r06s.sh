#!/bin/bash
# r06s: records-path tiles read a frame's second 64 B only when its headers
# reach them (kHalf): the -m gpu suite, then the default bench line.
set -e
tag=${1:-r06s}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
