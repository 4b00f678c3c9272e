#!/bin/bash
# Round 5, call g: the fused decode's round flush writing two buckets per
# store instruction (lanes 0-31 / 32-63, one descriptor per pair, per-lane
# offsets) = fl2 (working tree) vs head (HEAD).  The -m gpu suite on the
# in-tree build (= fl2) first.
# usage (on the GPU box): bash tools/r05/gpu_r05g.sh <tag>
set -e
tag=${1:-r05g}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
bash tools/ab_run.sh ${tag}_1500 "--no-9000 --no-box-state" head fl2
bash tools/ab_run.sh ${tag}_9000 "--frame-len 9000 --no-9000 --no-box-state" head fl2
