#!/bin/bash
set -e
mkdir -p gpurun_out
DQDK_GPU_LIB=$PWD/build/ab/pipe.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_pinned.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03l.log 2>&1
bash tools/ab_run.sh r03l "" base nopipe pipe pipe7
