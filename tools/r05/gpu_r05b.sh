#!/bin/bash
# Round 5, call b: rx_part2 loading the next gathered item's key triples a
# phase early (pf4 / pf8: scatter rounds of 4 / 8 keys) against round 4
# (base) and call a's form (p2sub); GPU parity of the in-tree build (= pf4,
# knobs read at queue creation, no diagnostic variants) on the tests this
# touches, then the whole -m gpu suite.
# usage (on the GPU box): bash tools/r05/gpu_r05b.sh <tag>
set -e
tag=${1:-r05b}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
bash tools/ab_run.sh ${tag}_1500 "--no-9000 --no-box-state" base p2sub pf4 pf8
bash tools/ab_run.sh ${tag}_9000 "--frame-len 9000 --no-9000 --no-box-state" base p2sub pf4 pf8
