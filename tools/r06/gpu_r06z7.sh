#!/bin/bash
# r06z7: the staging probe's worth at 1500 B -- the headline with the probe
# on (eight candidates) and off (DQDK_GPU_STAGING_PROBE=0), interleaved.
set -e
tag=${1:-r06z7}
mkdir -p gpurun_out/ab_probe_$tag
for r in 1 2 3; do
    for v in 1 0; do
        DQDK_GPU_STAGING_PROBE=$v timeout -k 10 200 python3 bench.py --steps 32 --warmup 3 --no-cpu-baseline --no-9000 \
            --no-configs --no-box-state > gpurun_out/ab_probe_$tag/probe${v}_$r.json 2> gpurun_out/ab_probe_$tag/probe${v}_$r.err
    done
done
