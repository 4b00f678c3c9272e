#!/bin/bash
# part2 with ranks through LDS: A/B vs HEAD, then one SQ PMC pass per build (1500 B)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
DQDK_GPU_LIB=$PWD/build/ab/p2c.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fullsize.py -k "1500" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03n.log 2>&1
bash tools/ab_run.sh r03n "" base p2c
for n in base p2c; do
  d=gpurun_out/pmcn_$n
  mkdir -p $d
  DQDK_GPU_LIB=$PWD/build/ab/$n.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $d/p1 -o run --output-format csv -- python3 bench.py --frame-len 1500 --frames 1048576 --steps 3 --warmup 1 --no-cpu-baseline --no-9000 > $d/p1.log 2>&1
  python3 tools/pmc_summary.py $d > $d/summary.txt
done
