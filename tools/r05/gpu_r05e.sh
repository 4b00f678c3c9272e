#!/bin/bash
# Round 5, call e: DESIGN.md section 7 on HEAD -- the PCIe-inclusive pipeline
# rates (tools/gpu_e2e.sh), bench.py --e2e (unpaced / paced at 100 Gbit/s),
# and the drop-in latency sweep with 1 and 3 workers (tools/dropin_latency.py).
# usage (on the GPU box): bash tools/r05/gpu_r05e.sh <tag>
set -e
tag=${1:-r05e}
mkdir -p gpurun_out
bash tools/gpu_e2e.sh $tag
timeout -k 10 300 python3 bench.py --e2e --steps 48 --no-cpu-baseline > gpurun_out/bench_e2e_$tag.json \
    2> gpurun_out/bench_e2e_$tag.err
timeout -k 10 900 python3 -u tools/dropin_latency.py --out gpurun_out/dropin_$tag.jsonl > gpurun_out/dropin_$tag.log 2>&1
