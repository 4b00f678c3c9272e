#!/bin/bash
# r06k: decode-only batches with the records-path decode's first-line
# hand-off (configs[1]): the -m gpu suite once (new edge-frame parity cases),
# then configs[1] same-box A/B, DQDK_GPU_HEAD_A 1 (default) / 0, three rounds.
set -e
tag=${1:-r06k}
d=gpurun_out/ab_head_$tag
mkdir -p $d
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
for r in 1 2 3; do
    for h in 1 0; do
        DQDK_GPU_HEAD_A=$h timeout -k 10 200 python3 bench.py --frames 262144 --no-histo --no-records --rotate 4 \
            --no-9000 --no-configs --no-box-state --steps 32 --warmup 2 --no-cpu-baseline > $d/h${h}_$r.json 2> $d/h${h}_$r.err
    done
done
