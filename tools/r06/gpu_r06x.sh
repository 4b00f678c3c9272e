#!/bin/bash
# r06x: PMC traffic of every bench line's roofline kernel regenerated on the
# final tree with tools/pmc.sh's four passes (FETCH_SIZE, WRITE_SIZE, SQ,
# read requests by size) -- headline 1M x 1500 B, 1M x 9000 B, configs[1]
# (4 rotated images), configs[2], the mixed batch -- into
# gpurun_out/pmc_summary.json.
set -e
tag=${1:-r06x}
mkdir -p gpurun_out
rm -f gpurun_out/pmc_summary.json
bash tools/pmc.sh $tag 1500 --no-configs --no-box-state
bash tools/pmc.sh $tag 9000 --no-configs --no-box-state
FRAMES=262144 bash tools/pmc.sh ${tag}_cfg1 1500 --no-histo --no-records --rotate 4 --no-configs --no-box-state
FRAMES=262144 bash tools/pmc.sh ${tag}_cfg2 9000 --no-configs --no-box-state
bash tools/pmc.sh ${tag}_mixed 0 --no-configs --no-box-state
