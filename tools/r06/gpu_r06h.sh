#!/bin/bash
# r06h: per-batch overheads inside the timed region.  (a) Slot scratch zeroed
# at queue creation (zeroed.so) vs clean_slot's four memset launches on each
# slot's first use (memset.so: 21 of the 32 timed batches at 1500 B paid
# them); (b) the bench's own events: default (a torch event per step + HIP
# events around every decode) / no per-step events / neither (decode timed in
# the breakdown pass).  Same box, 1500 B only, --steps 32, three rounds.
set -e
tag=${1:-r06h}
d=gpurun_out/ab_ev_$tag
mkdir -p $d
for r in 1 2 3; do
    DQDK_GPU_LIB=$PWD/build/ab/memset.so timeout -k 10 200 python3 bench.py --steps 32 --warmup 2 --no-cpu-baseline \
        --no-9000 --no-configs --no-box-state > $d/memset_$r.json 2> $d/memset_$r.err
    for v in "1 1" "0 1" "0 0"; do
        set -- $v
        DQDK_GPU_LIB=$PWD/build/ab/zeroed.so timeout -k 10 200 python3 bench.py --steps 32 --warmup 2 --no-cpu-baseline \
            --no-9000 --no-configs --no-box-state --step-events $1 --decode-events $2 > $d/s$1d$2_$r.json 2> $d/s$1d$2_$r.err
    done
done
