#!/bin/bash
# r06z2: eight staging candidates (DQDK_GPU_PROBE_CANDS 8): the probe tests,
# then the default bench line.
set -e
tag=${1:-r06z2}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fullsize.py -m gpu -k staging_probe -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/pytest_probe_$tag.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
