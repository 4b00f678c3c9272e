#!/bin/bash
# r06g: the slice pass with the wave's next group's runs touched into L2
# (LDS-DMA dwords, one per 128-B line, inline asm) while this group is
# counted (-DDQDK_SLICE_TOUCH=1) vs without; same box, 1500 B and 9000 B,
# --steps 32 (one whole slice pass at 1500 B), two interleaved rounds.
set -e
tag=${1:-r06g}
mkdir -p gpurun_out/ab_touch_$tag
for r in 1 2; do
    for n in t0 t1; do
        DQDK_GPU_LIB=$PWD/build/ab/$n.so timeout -k 10 300 python3 bench.py --steps 32 --warmup 2 --no-cpu-baseline \
            --no-configs --no-box-state > gpurun_out/ab_touch_$tag/${n}_$r.json 2> gpurun_out/ab_touch_$tag/${n}_$r.err
    done
done
