#!/bin/bash
# Round 6 final evidence, call 1 of 2: PMC traffic of every bench line's
# roofline kernel regenerated from scratch on the final tree (calibrated
# FETCH_SIZE x 2 + WRITE_SIZE per dispatch, tools/pmc.sh: three passes
# each) -- the headline 1M x 1500 B, 1M x 9000 B and the by_config lines
# (configs[1] 256K x 1500 B parse + checksum over 4 rotated images,
# configs[2] 256K x 9000 B, the mixed 1500/9000 B batch) -- into
# gpurun_out/pmc_summary.json, plus the chain's LDS counters at both sizes.
# usage (on the GPU box): bash tools/r06/gpu_final_r06_pmc.sh <tag>
set -e
tag=${1:-r06z}
mkdir -p gpurun_out
rm -f gpurun_out/pmc_summary.json
bash tools/pmc.sh $tag 1500
bash tools/pmc.sh $tag 9000
FRAMES=262144 bash tools/pmc.sh ${tag}_cfg1 1500 --no-histo --no-records --rotate 4
FRAMES=262144 bash tools/pmc.sh ${tag}_cfg2 9000
bash tools/pmc.sh ${tag}_mixed 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in 1500 9000; do
    timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
        SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/pmc_lds_${tag}_$L -o run \
        --output-format csv -- python3 bench.py --frame-len $L --steps 3 --warmup 1 --no-cpu-baseline --no-9000 \
        --no-box-state > gpurun_out/pmc_lds_${tag}_$L.log 2>&1
done
