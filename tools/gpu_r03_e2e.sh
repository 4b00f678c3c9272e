#!/bin/bash
# Round-3 end: the whole GPU suite, then the PCIe-inclusive rates (configs[4]).
set -e
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_r03.log 2>&1
bash tools/gpu_e2e.sh r03
timeout -k 10 300 python3 bench.py --e2e > gpurun_out/bench_e2e_r03.json 2> gpurun_out/bench_e2e_r03.err
