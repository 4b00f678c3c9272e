#!/bin/bash
# r06b: the records-path decode with its counters folded (no rx_abort /
# rx_count launches): the whole -m gpu suite once, then configs[1] (256K x
# 1500 B parse + checksum, no event work, 4 rotated images) same-box A/B:
# HEAD (abort + count) / folded / folded with 6- and 8-window rings.
set -e
tag=${1:-r06b}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
bash tools/ab_run.sh cfg1_$tag "--frames 262144 --no-histo --no-records --rotate 4 --no-9000 --no-configs --no-box-state" \
    p1base p1fold p1ring6 p1ring8
