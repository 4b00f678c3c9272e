#!/bin/bash
# Stall-source PMC passes on one bench configuration (kernel-trace only).
# usage: bash tools/pmc_sq2.sh <tag> <frame_len> [bench args]
set -e
tag=${1:-run}; L=${2:-1500}; shift 2 || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/pmcsq2_${tag}_$L
mkdir -p $d
i=0
for grp in "SQ_WAIT_INST_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_SALU" \
           "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TC_STALL TD_TD_BUSY SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d $d/p$i -o run --output-format csv -- \
        python3 bench.py --frame-len $L --steps 3 --warmup 1 --no-cpu-baseline "$@" > $d/p$i.log 2>&1
done
