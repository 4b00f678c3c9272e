#!/bin/bash
# Round 4, call c: where the decode's and rx_part2's time goes.
#   membench mixes (read / 4:1 / copy / frame patterns) on this box;
#   A/B on one box (build/ab/*.so): base = round-3 stage (120 keys, tail in
#   LDS); it = checksum tail corrected in the window loop, 134-key stage
#   (W 20 / 16); it_lo = the same at W 16 / 12; nostore = it without piece
#   stores (timing only); lines = it with whole-line flushes at 1500 B too;
#   SQ/LDS counters of the default 1500 B and 9000 B runs (one pass each).
# usage (on the GPU box): bash tools/r04/gpu_r04c.sh <tag>
set -e
tag=${1:-r04c}
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/membench_mix.py > gpurun_out/membench_$tag.json 2> gpurun_out/membench_$tag.err
bash tools/ab_run.sh ${tag}_1500 "--no-9000 --no-box-state" base it it_lo nostore lines
bash tools/ab_run.sh ${tag}_9000 "--frame-len 9000 --no-9000 --no-box-state" base it it_lo
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in 1500 9000; do
    timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
        SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/pmc_lds_${tag}_$L -o run \
        --output-format csv -- python3 bench.py --frame-len $L --steps 3 --warmup 1 --no-cpu-baseline --no-9000 \
        --no-box-state > gpurun_out/pmc_lds_${tag}_$L.log 2>&1
done
