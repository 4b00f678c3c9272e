#!/bin/bash
# r06c: the -m gpu suite once on the working tree (records-path counters
# folded into rx_decode; rx_part2's balanced items), then same-box A/Bs:
#  - configs[1] (256K x 1500 B parse + checksum, 4 rotated images): HEAD
#    (rx_abort + rx_count) / folded / folded with 6- and 8-window rings;
#  - 1M x 1500 B default path: rx_part2 items balanced (default) / not
#    (DQDK_GPU_P2_BALANCE=0), interleaved, two rounds.
set -e
tag=${1:-r06c}
mkdir -p gpurun_out gpurun_out/ab_p2_$tag
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
bash tools/ab_run.sh cfg1_$tag "--frames 262144 --no-histo --no-records --rotate 4 --no-9000 --no-configs --no-box-state" \
    p1base p1fold p1ring6 p1ring8
for r in 1 2; do
    for v in 1 0; do
        DQDK_GPU_P2_BALANCE=$v timeout -k 10 200 python3 bench.py --steps 32 --warmup 2 --no-cpu-baseline --no-9000 \
            --no-configs --no-box-state > gpurun_out/ab_p2_$tag/bal${v}_$r.json 2> gpurun_out/ab_p2_$tag/bal${v}_$r.err
    done
done
