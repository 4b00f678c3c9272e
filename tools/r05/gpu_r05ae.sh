#!/bin/bash
# Round 5, call ae: the 9000 B decode's slow state against address
# translation.  Two PMC passes (kernel trace only, no tracing domains) over a
# short 9000 B bench run whose warmup includes the staging probe (five piece
# buffers, each decoded twice): per dispatch, UTCL1 translation requests and
# misses and the TCP -> TCC read latency (pass 1), UTCL2 busy cycles and the
# TCC -> memory read requests (pass 2), next to each dispatch's duration.
# usage (on the GPU box): bash tools/r05/gpu_r05ae.sh <tag>
set -e
tag=${1:-r05ae}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/$tag
mkdir -p $d
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d $d/p$i -o run --output-format csv -- \
        python3 bench.py --frame-len 9000 --steps 4 --warmup 1 --no-cpu-baseline --no-9000 --no-box-state \
        > $d/p$i.json 2> $d/p$i.err
done
