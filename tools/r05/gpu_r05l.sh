#!/bin/bash
# Round 5, call l: the packed stage (keys staged three to an 8-B word, as
# the pieces hold them: 198 keys a bucket instead of 134; rounds of 24 / 16
# windows running on across super-tiles; the flush copies words) = the
# in-tree build and build/ab/pk.so, against HEAD (head).
#   1. the -m gpu suite on the in-tree build;
#   2. interleaved bench runs: head, pk, pk at fill 70, both sizes, two rounds;
#   3. rx_part2's per-phase cycles (diagnostic build p2t, HEAD's decode).
# usage (on the GPU box): bash tools/r05/gpu_r05l.sh <tag>
set -e
tag=${1:-r05l}
mkdir -p gpurun_out/ab_${tag}_1500 gpurun_out/ab_${tag}_9000 gpurun_out/${tag}_p2t
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
for r in 1 2; do
    for L in 1500 9000; do
        for v in head pk pk_f70; do
            lib=${v%_f70}; env=""
            [ "$v" = pk_f70 ] && env="DQDK_GPU_FUSED_FILL=70"
            env DQDK_GPU_LIB=$PWD/build/ab/$lib.so $env timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 \
                --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/ab_${tag}_$L/${v}_$r.json \
                2> gpurun_out/ab_${tag}_$L/${v}_$r.err
        done
    done
done
for L in 1500 9000; do
    DQDK_GPU_LIB=$PWD/build/ab/p2t.so timeout -k 10 200 python3 bench.py --frame-len $L --steps 5 \
        --warmup 2 --no-cpu-baseline --no-9000 --no-box-state > gpurun_out/${tag}_p2t/p2t_$L.out \
        2> gpurun_out/${tag}_p2t/p2t_$L.err
done
