#!/bin/bash
# LDS-pressure PMC pass (kernel-trace only) on one bench configuration:
# LDS-array busy cycles, bank/address conflicts, LDS instructions and waits.
# usage (on the GPU box): bash tools/pmc_lds.sh <tag> <frame_len>
set -e
tag=${1:-run}; L=${2:-1500}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/pmclds_${tag}_$L
mkdir -p $d
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS \
    SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_ATOMIC_RETURN -d $d/p1 -o run --output-format csv -- \
    python3 bench.py --frame-len $L --steps 3 --warmup 1 --no-cpu-baseline > $d/p1.log 2>&1
python3 tools/pmc_summary.py $d > $d/summary.txt
