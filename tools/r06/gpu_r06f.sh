#!/bin/bash
# r06f: rx_part2 with packed u16 slice counters (two per LDS word: 16 KB less
# LDS), which leaves room for larger items at two blocks per CU: 18 keys per
# thread (shipped since r06d) / 18 packed / 21 packed / 24 packed, same box,
# 1500 B and 9000 B, two interleaved rounds.
set -e
tag=${1:-r06f}
bash tools/ab_run.sh p2p_$tag "--no-configs --no-box-state" k18 k18p k21p k24p
