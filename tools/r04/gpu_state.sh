#!/bin/bash
# One box's 9000 B speed state and identity: a short 9000 B bench line with
# box_state (HBM vendor, VBIOS, clocks, partitions) and the decode's
# fraction of the same-process stream read.
# usage (on the GPU box): bash tools/r04/gpu_state.sh <tag>
set -e
tag=${1:-state}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --frame-len 9000 --no-9000 --no-cpu-baseline --steps 8 --warmup 2 \
    > gpurun_out/state_$tag.json 2> gpurun_out/state_$tag.err
python3 - gpurun_out/state_$tag.json <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
bs = b.get("box_state", {})
print(json.dumps({"decode_ms": b["kernels"]["rx_decode"]["avg_ms"], "frac_stream": b["roofline"].get("frac_of_measured_stream"),
                  **{k: bs.get(k) for k in ("bdf", "mem_info_vram_vendor", "vbios_version", "product_name",
                                             "current_link_speed", "sclk_current", "mclk_current")}}))
PY
