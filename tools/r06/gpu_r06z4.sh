#!/bin/bash
# r06z4: rx_part2's scatter group (returning LDS adds issued before their
# stores) with 18-key items: 4 (shipped) vs 3 / 6 / 9, at 1500 and 9000 B.
set -e
tag=${1:-r06z4}
mkdir -p gpurun_out
bash tools/ab_run.sh sg_$tag "--no-9000 --no-configs --no-box-state" base sg3 sg6 sg9
bash tools/ab_run.sh sg9k_$tag "--frame-len 9000 --no-configs --no-box-state" base sg6 sg9
