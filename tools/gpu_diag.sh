#!/bin/bash
# Decode diagnostics: records on/off, histogram off, per A/B build.
set -e
tag=$1; shift
mkdir -p gpurun_out/diag_$tag
for n in "$@"; do
  for L in 1500 9000; do
    for mode in "full:" "nohisto:--no-histo" "norec:--no-histo --no-records"; do
      nm=${mode%%:*}; args=${mode#*:}
      DQDK_GPU_LIB=$PWD/build/ab/$n.so timeout -k 10 200 python3 bench.py --frame-len $L --steps 10 --warmup 2 --no-cpu-baseline $args \
        > gpurun_out/diag_$tag/${n}_${L}_$nm.json 2> gpurun_out/diag_$tag/${n}_${L}_$nm.err
    done
  done
done
