#!/bin/bash
# SQ-level PMC passes on one bench configuration (kernel-trace only), for
# issue/stall breakdowns.  usage: bash tools/pmc_sq.sh <tag> <frame_len>
set -e
tag=${1:-run}; L=${2:-1500}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/pmcsq_${tag}_$L
mkdir -p $d
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d $d/p$i -o run --output-format csv -- \
        python3 bench.py --frame-len $L --steps 3 --warmup 1 --no-cpu-baseline > $d/p$i.log 2>&1
done
