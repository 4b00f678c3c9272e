#!/bin/bash
# r06w: one PMC pass of the read requests by size (TCC_EA0_RDREQ_{,32B,64B,128B}_sum)
# over the headline bench, whose in-process membenches (stream_read: known
# bytes; frames_pattern) calibrate the byte formula.
set -e
tag=${1:-r06w}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_${tag}_1500
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d gpurun_out/pmc_${tag}_1500/p4 -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-9000 --no-configs --no-box-state \
    > gpurun_out/pmc_${tag}_1500/p4.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_1500 > gpurun_out/pmc_${tag}_1500/summary.txt
