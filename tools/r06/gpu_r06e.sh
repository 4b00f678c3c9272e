#!/bin/bash
# r06e: configs[1] (256K x 1500 B parse + checksum, 4 rotated images): the
# records-path decode's wave tile (DQDK_GPU_TILE_FRAMES 64 = shipped / 32 /
# 16: with 64 every wave runs one tile, so every wave's phase A falls at the
# same moment; smaller tiles put some waves' phase A under others' streams).
set -e
tag=${1:-r06e}
d=gpurun_out/ab_tile_$tag
mkdir -p $d
for r in 1 2; do
    for t in 64 32 16; do
        DQDK_GPU_TILE_FRAMES=$t timeout -k 10 200 python3 bench.py --frames 262144 --no-histo --no-records --rotate 4 \
            --no-9000 --no-configs --no-box-state --steps 20 --warmup 2 --no-cpu-baseline > $d/t${t}_$r.json 2> $d/t${t}_$r.err
    done
done
