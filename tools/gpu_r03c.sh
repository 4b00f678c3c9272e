#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_pinned.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03c.log 2>&1
bash tools/ab_run.sh r03c "" base pair pairdpp dpp pair2dpp
timeout -k 10 300 python3 tools/raw_overlap.py > gpurun_out/raw_overlap_r03c.json 2> gpurun_out/raw_overlap_r03c.err
