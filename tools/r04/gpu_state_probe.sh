#!/bin/bash
# Round 4: the per-process speed state -- tools/state_probe.py in three
# processes on one box (each: 3 contiguous images + 1 torch image x 2 queues).
# usage (on the GPU box): bash tools/r04/gpu_state_probe.sh <tag>
set -e
tag=${1:-probe}
mkdir -p gpurun_out
for i in 1 2 3; do
    timeout -k 10 300 python3 tools/state_probe.py >> gpurun_out/state_probe_$tag.jsonl 2>> gpurun_out/state_probe_$tag.err
done
