#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_pinned.py tests/test_c_harness.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03k.log 2>&1
bash tools/ab_run.sh r03k "" base sk
bash tools/pmc_detail.sh r03k 1500
