#!/bin/bash
# Decode timing diagnostics on --no-csum --no-histo (checksum/histogram results ignored).
set -e
tag=$1; shift
mkdir -p gpurun_out/diag_$tag
for r in 1 2; do
for n in "$@"; do
  for L in 1500 9000; do
      DQDK_GPU_LIB=$PWD/build/ab/$n.so timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 --warmup 2 --no-cpu-baseline --no-csum --no-histo \
        > gpurun_out/diag_$tag/${n}_${L}_$r.json 2> gpurun_out/diag_$tag/${n}_${L}_$r.err
  done
done
done
