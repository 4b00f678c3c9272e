#!/bin/bash
# r06d: rx_part2 item size (the slice pass is a gather of
# runs whose length is item / 64 per span): 15 (shipped) / 18 keys per thread
# (2 blocks per CU, 79.5 KB LDS) / 30 keys per thread (1 block per CU, slice
# gather 4 dwords per lane), same box, 1500 B and 9000 B, two rounds.
set -e
tag=${1:-r06d}
bash tools/ab_run.sh p2_$tag "--no-configs --no-box-state" p2k15 p2k18 p2k30
