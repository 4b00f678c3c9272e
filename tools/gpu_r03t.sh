#!/bin/bash
# block-major fused pieces: GPU tests, A/B vs the previous commit (r3), placement probe
set -e
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pinned.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r03t_a.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03t_b.log 2>&1
bash tools/ab_run.sh r03t "" r3 bm
for n in r3 bm; do DQDK_GPU_LIB=$PWD/build/ab/$n.so timeout -k 10 300 python3 tools/placement.py --frame-len 9000 --max-gb 8 --step-gb 4 > gpurun_out/placement_r03t_$n.jsonl 2>/dev/null; done
