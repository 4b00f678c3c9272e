#!/bin/bash
# lean part2 (prep folded in, fixup in part1): parity on the GPU, then A/B vs HEAD
set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pinned.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r03m_a.log 2>&1
bash tools/ab_run.sh r03m "" base p2v2
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_egress.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03m_b.log 2>&1
