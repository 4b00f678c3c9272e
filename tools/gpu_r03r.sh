#!/bin/bash
# 9000 B decode placement probes: staging allocation kinds x image placement, bimodal torch/contig
set -e
mkdir -p gpurun_out
for k in plain contig; do
  DQDK_GPU_ALLOC=$k timeout -k 10 300 python3 tools/placement.py --frame-len 9000 --max-gb 2 --step-gb 1 > gpurun_out/placement_9000_$k.jsonl 2>/dev/null
done
bash tools/bimodal.sh r03r 2 > gpurun_out/bimodal_r03r.txt 2>&1
