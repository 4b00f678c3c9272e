#!/bin/bash
# Round 5, call f: where the fused decode's round flushes cost time.
# Timing-only builds (wrong tables, never tested or shipped; built from the
# working tree with a local edit): d_ns = the flush
# without its piece stores; d_nf = no flush inside the rounds (counts reset,
# keys dropped; barriers kept); head = HEAD.  Interleaved bench runs at both
# sizes; then the SQ wave-cycle split of the 9000 B decode.
# usage (on the GPU box): bash tools/r05/gpu_r05f.sh <tag>
set -e
tag=${1:-r05f}
mkdir -p gpurun_out
bash tools/ab_run.sh ${tag}_1500 "--no-9000 --no-box-state" head d_ns d_nf
bash tools/ab_run.sh ${tag}_9000 "--frame-len 9000 --no-9000 --no-box-state" head d_ns d_nf
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU \
    SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d gpurun_out/pmc_sq_${tag}_9000 -o run --output-format csv -- \
    python3 bench.py --frame-len 9000 --steps 3 --warmup 1 --no-cpu-baseline --no-9000 --no-box-state \
    > gpurun_out/pmc_sq_${tag}_9000.log 2>&1
