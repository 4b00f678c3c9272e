#!/bin/bash
# Instruction-mix / stall PMC passes over a short bench run (one frame size),
# plus the 4-B store WRITE_SIZE calibration (tools/calib_write.py).
# usage (on the GPU box): bash tools/pmc_detail.sh <tag> <frame_len> [bench args...]
tag=${1:-run}; L=${2:-1500}; shift 2 || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/pmcd_${tag}_$L
mkdir -p $d
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp -d $d/p$i -o run --output-format csv -- \
        python3 bench.py --frame-len $L --frames 1048576 --steps 3 --warmup 1 --no-cpu-baseline --no-9000 "$@" > $d/p$i.log 2>&1
    rc=$?
    echo "pass $i rc=$rc" >> $d/rc.txt
    if [ $rc -eq 137 ] || [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py $d > $d/summary.txt
c=gpurun_out/calib_${tag}
mkdir -p $c
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $c/p1 -o run --output-format csv -- python3 tools/calib_write.py > $c/calib.json 2> $c/calib.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $c/p2 -o run --output-format csv -- python3 tools/calib_write.py > $c/calib2.json 2> $c/calib2.err
python3 tools/pmc_summary.py $c > $c/summary.txt || true
