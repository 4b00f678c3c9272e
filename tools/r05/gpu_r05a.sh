#!/bin/bash
# Round 5, call a: rx_part2 as a two-pass counting sort over per-lane-slot
# counters (p2sub = the working tree) against round 4's (base = HEAD).
#   the -m gpu suite on the in-tree build (= p2sub);
#   same-box A/B at 1500 B and 9000 B;
#   LDS counters of p2sub's default runs (one pass per size).
# usage (on the GPU box): bash tools/r05/gpu_r05a.sh <tag>
set -e
tag=${1:-r05a}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
bash tools/ab_run.sh ${tag}_1500 "--no-9000 --no-box-state" base p2sub
bash tools/ab_run.sh ${tag}_9000 "--frame-len 9000 --no-9000 --no-box-state" base p2sub
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in 1500 9000; do
    timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
        SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/pmc_lds_${tag}_$L -o run \
        --output-format csv -- python3 bench.py --frame-len $L --steps 3 --warmup 1 --no-cpu-baseline --no-9000 \
        --no-box-state > gpurun_out/pmc_lds_${tag}_$L.log 2>&1
done
