#!/bin/bash
# key-triple pieces (decode writes 8 B per 3 keys, part2 gathers triples): GPU tests, A/B vs HEAD
set -e
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pinned.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r03v_a.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_egress.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03v_b.log 2>&1
bash tools/ab_run.sh r03v "" r3b tri
