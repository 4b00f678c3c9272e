#!/bin/bash
# r06h: what the bench's own events cost inside the timed region (the gaps
# between a batch's rx_part2 and the next decode measured ~10 us under
# rocprof): default (a torch event per step + HIP events around every
# decode) / no per-step events / neither (decode timed in the breakdown pass
# instead), same box, 1500 B only, --steps 32, three rounds.
set -e
tag=${1:-r06h}
d=gpurun_out/ab_ev_$tag
mkdir -p $d
for r in 1 2 3; do
    for v in "1 1" "0 1" "0 0"; do
        set -- $v
        timeout -k 10 200 python3 bench.py --steps 32 --warmup 2 --no-cpu-baseline --no-9000 --no-configs --no-box-state \
            --step-events $1 --decode-events $2 > $d/s$1d$2_$r.json 2> $d/s$1d$2_$r.err
    done
done
