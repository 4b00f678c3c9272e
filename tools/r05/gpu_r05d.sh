#!/bin/bash
# Round 5, call d: rx_part2 writing item i's stage after item i+1's count
# (fixed two 16-B stores per thread, issued before the next loads: the
# count's waits no longer drain them) = p2ro (working tree) vs p2pf (HEAD);
# slb3 = p2ro + the slice pass gathering 16 B per lane (b128, 3 items x 4
# dwords).  The -m gpu suite on the in-tree build (= p2ro) first.
# usage (on the GPU box): bash tools/r05/gpu_r05d.sh <tag>
set -e
tag=${1:-r05d}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
bash tools/ab_run.sh ${tag}_1500 "--no-9000 --no-box-state" p2pf p2ro slb3
bash tools/ab_run.sh ${tag}_9000 "--frame-len 9000 --no-9000 --no-box-state" p2pf p2ro slb3
