#!/bin/bash
set -e
mkdir -p gpurun_out/ab_r03g
for r in 1 2; do
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_r03g/img_$r.json 2> gpurun_out/ab_r03g/img_$r.err
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --umem-alloc torch > gpurun_out/ab_r03g/torch_$r.json 2> gpurun_out/ab_r03g/torch_$r.err
    DQDK_GPU_CONTIG=1 timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --umem-alloc torch > gpurun_out/ab_r03g/intonly_$r.json 2> gpurun_out/ab_r03g/intonly_$r.err
done
