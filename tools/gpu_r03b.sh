#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_egress.py tests/test_c_harness.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_egress_r03b.log 2>&1
timeout -k 10 300 python3 tools/raw_overlap.py > gpurun_out/raw_overlap_r03b.json 2> gpurun_out/raw_overlap_r03b.err
bash tools/pmc_detail.sh r03b 1500
