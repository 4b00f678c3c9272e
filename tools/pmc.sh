#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass, no tracing flags) over a
# short bench run.  usage (on the GPU box): bash tools/pmc.sh <tag> [bench args...]
set -e
tag=${1:-run}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_$tag
rocprofv3 -L > gpurun_out/pmc_$tag/counters_available.txt 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc_$tag/p$i -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/pmc_$tag/p$i.log 2>&1 || \
        echo "pass $i ($grp) failed rc=$?" >> gpurun_out/pmc_$tag/errors.txt
done
