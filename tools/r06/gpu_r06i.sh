#!/bin/bash
# r06i: rx_part1's launch removed from the fused path (the decode takes back
# checksum-failed frames in its phase C and adds its overflow keys by device
# atomics; rx_part2 scans the piece sizes itself): the -m gpu suite once on
# the working tree, then same-box A/B vs HEAD (p1launch), 1500 B and 9000 B,
# --steps 32, two interleaved rounds.
set -e
tag=${1:-r06i}
mkdir -p gpurun_out gpurun_out/ab_p1_$tag
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
for r in 1 2; do
    for n in p1launch nop1; do
        DQDK_GPU_LIB=$PWD/build/ab/$n.so timeout -k 10 300 python3 bench.py --steps 32 --warmup 2 --no-cpu-baseline \
            --no-configs --no-box-state > gpurun_out/ab_p1_$tag/${n}_$r.json 2> gpurun_out/ab_p1_$tag/${n}_$r.err
    done
done
