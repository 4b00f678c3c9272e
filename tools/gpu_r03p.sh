#!/bin/bash
# pipelined u32 slice gather: quick parity, then A/B of gather shapes vs HEAD
set -e
mkdir -p gpurun_out
DQDK_GPU_LIB=$PWD/build/ab/sl3.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "synthetic or peaked or staged or carries" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r03p.log 2>&1
bash tools/ab_run.sh r03p "" base sl3 sl3b sl3c
