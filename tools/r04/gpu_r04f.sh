#!/bin/bash
# Round 4, call f: the new small-batch / plugin tests, the drop-in latency
# sweep with rx_small, then call c's decode A/B, membench mixes and LDS PMC.
# usage (on the GPU box): bash tools/r04/gpu_r04f.sh <tag>
set -e
tag=${1:-r04f}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plugin.py tests/test_c_harness.py \
    -m gpu -x -q -k "small or plugin or harness" --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
timeout -k 10 600 python3 -u tools/dropin_latency.py --quick --out gpurun_out/dropin_$tag.jsonl > gpurun_out/dropin_$tag.log 2>&1
bash tools/r04/gpu_r04c.sh $tag
