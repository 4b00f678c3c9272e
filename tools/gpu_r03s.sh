#!/bin/bash
# default bench: UMEM images allocated largest first vs in measurement order
set -e
mkdir -p gpurun_out/ab_r03s
for r in 1 2; do
  for o in large-first given; do
    DQDK_BENCH_IMAGE_ORDER=$o timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_r03s/${o}_$r.json 2> gpurun_out/ab_r03s/${o}_$r.err
  done
done
