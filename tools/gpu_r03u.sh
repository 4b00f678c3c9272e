#!/bin/bash
# overlap feasibility: 1 vs 2 queues on 2 streams, decode grid capped or not (1500 B and 9000 B)
set -e
mkdir -p gpurun_out
o=gpurun_out/overlap_r03u.jsonl
: > $o
for L in 1500 9000; do
  timeout -k 10 120 python3 tools/overlap.py --frame-len $L --queues 1 >> $o 2>/dev/null
  for c in 256 192 128; do
    DQDK_GPU_DECODE_CUS=$c timeout -k 10 120 python3 tools/overlap.py --frame-len $L --queues 2 | sed "s/}/, \"decode_cus\": $c}/" >> $o 2>/dev/null
  done
done
