#!/bin/bash
set -e
mkdir -p gpurun_out/ab_r03f
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_fullsize.py tests/test_abi.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03f.log 2>&1
for r in 1 2; do
    DQDK_GPU_CONTIG=1 timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_r03f/contig_$r.json 2> gpurun_out/ab_r03f/contig_$r.err
    DQDK_GPU_CONTIG=0 timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_r03f/imgonly_$r.json 2> gpurun_out/ab_r03f/imgonly_$r.err
    DQDK_GPU_CONTIG=0 timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --umem-alloc torch > gpurun_out/ab_r03f/none_$r.json 2> gpurun_out/ab_r03f/none_$r.err
done
