#!/bin/bash
# r06j: where r06i's decode slowdown (0.401 -> 0.449 ms at 1500 B with
# rx_part1's launch removed) comes from: p1launch = HEAD (rx_part1 launched);
# nop1b = segment sizes added one 128-B line per bucket (r06i: 568 words in
# 18 lines); nop1b_list = the same with the overflow keys listed
# (DQDK_GPU_OVF_LIST=1: rx_part1 groups them, no atomics at the decode's end);
# nop1c = nop1b without the segment-size atomics (timing only).  Same box,
# 1500 B and 9000 B, --steps 32, two rounds.
set -e
tag=${1:-r06j}
d=gpurun_out/ab_p1b_$tag
mkdir -p $d
run() {  # name lib [env]
    env $3 DQDK_GPU_LIB=$PWD/build/ab/$2.so timeout -k 10 300 python3 bench.py --steps 32 --warmup 2 --no-cpu-baseline \
        --no-configs --no-box-state > $d/$1_$r.json 2> $d/$1_$r.err
}
for r in 1 2; do
    run p1launch p1launch
    run nop1b nop1b
    run nop1b_list nop1b DQDK_GPU_OVF_LIST=1
    run nop1c nop1c
done
