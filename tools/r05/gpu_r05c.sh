#!/bin/bash
# Round 5, call c: the -m gpu suite on HEAD (staging probe, raw drain,
# destroy-ordering test), the default bench line (with the probe's outcome),
# SURVEY 8(d)'s packed-stride 1500 B line (stride 1536), the counter list of
# this rocprofv3, one SQ pass over the default 1500 B run (wave-cycle
# split of the decode: parked / issue-stalled / active, SALU / VALU / LDS / VMEM).
# usage (on the GPU box): bash tools/r05/gpu_r05c.sh <tag>
set -e
tag=${1:-r05c}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
timeout -k 10 300 python3 bench.py --stride 1536 --no-9000 > gpurun_out/bench_${tag}_s1536.json \
    2> gpurun_out/bench_${tag}_s1536.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_$tag.txt 2>&1 || true
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU \
    SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d gpurun_out/pmc_sq_${tag}_1500 -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-9000 --no-box-state \
    > gpurun_out/pmc_sq_${tag}_1500.log 2>&1
# rx_part2 with contiguous item shares per block (piece starts staged once
# per bucket): p2ct = the working tree, p2pf = HEAD (the phase-early loads)
bash tools/ab_run.sh ${tag}_1500 "--no-9000 --no-box-state" p2pf p2ct
bash tools/ab_run.sh ${tag}_9000 "--frame-len 9000 --no-9000 --no-box-state" p2pf p2ct
