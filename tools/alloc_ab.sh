#!/bin/bash
# A/B of the device allocation kinds (dqdk_gpu.hip dev_alloc): the queue's own
# buffers (DQDK_GPU_ALLOC) x the UMEM images (DQDK_GPU_IMAGE_ALLOC), default
# bench (1500 B + 9000 B), separate processes, interleaved rounds.
# usage (GPU box): bash tools/alloc_ab.sh <tag> [rounds]
tag=${1:-alloc}; rounds=${2:-2}
d=gpurun_out/ab_$tag
mkdir -p $d
for r in $(seq 1 $rounds); do
    for combo in plain:contig auto:contig contig:contig; do
        i=${combo%%:*}; m=${combo##*:}
        DQDK_GPU_ALLOC=$i DQDK_GPU_IMAGE_ALLOC=$m timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline \
            > $d/${i}-${m}_$r.json 2> $d/${i}-${m}_$r.err || exit $?
    done
done
