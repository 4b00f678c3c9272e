#!/bin/bash
# r06z8: the staging probe timing every candidate twice, in order and in
# reverse order (drift-robust): the probe tests, the 1500 B headline with the
# probe on and off interleaved, then the default bench line.
set -e
tag=${1:-r06z8}
mkdir -p gpurun_out/ab_probe_$tag
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fullsize.py -m gpu -k staging_probe -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/pytest_probe_$tag.log 2>&1
for r in 1 2 3; do
    for v in 1 0; do
        DQDK_GPU_STAGING_PROBE=$v timeout -k 10 200 python3 bench.py --steps 32 --warmup 3 --no-cpu-baseline --no-9000 \
            --no-configs --no-box-state > gpurun_out/ab_probe_$tag/probe${v}_$r.json 2> gpurun_out/ab_probe_$tag/probe${v}_$r.err
    done
done
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
