#!/bin/bash
# u32 slice bins (1024-thread slice blocks, no heavy pass, budgeted hist_k),
# item-indexed part2 output, overflow regions in part1: GPU tests, then A/B vs HEAD
set -e
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pinned.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r03o_a.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_egress.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03o_b.log 2>&1
bash tools/ab_run.sh r03o "" base sl2
