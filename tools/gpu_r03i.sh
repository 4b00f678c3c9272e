#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 240 --timeout-method thread -k "1M-9000-clean or 1M-1500-clean" > gpurun_out/pytest_r03i.log 2>&1
DQDK_GPU_ALLOC=vmm DQDK_GPU_IMAGE_ALLOC=vmm timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread >> gpurun_out/pytest_r03i.log 2>&1
bash tools/alloc_ab.sh r03i 2
