#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass, kernel-trace only, no
# tracing domains) over a short bench run, then the per-kernel summary into
# gpurun_out/pmc_summary.json under bench.py's workload key.
# usage (on the GPU box): [FRAMES=n] bash tools/pmc.sh <tag> <frame_len> [bench args...]
# (frame_len 0 = the mixed 1500/9000 B workload; --no-9000: the 1500 B run alone,
# whose by_frame_len 9000 B pass would otherwise mix into the same kernel names)
set -e
tag=${1:-run}; L=${2:-1500}; shift 2 || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/pmc_${tag}_$L
mkdir -p $d
i=0
# (pass 4: read requests by size -- 4 TCC counters, the block's limit)
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp -d $d/p$i -o run --output-format csv -- \
        python3 bench.py --frame-len $L --frames ${FRAMES:-1048576} --steps 3 --warmup 1 --no-cpu-baseline --no-9000 "$@" > $d/p$i.log 2>&1
done
python3 tools/pmc_summary.py $d gpurun_out/pmc_summary.json "$L:csum:${FRAMES:-1048576}" > $d/summary.txt
