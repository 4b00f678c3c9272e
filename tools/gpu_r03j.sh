#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03j.log 2>&1
bash tools/alloc_ab.sh r03j 3
