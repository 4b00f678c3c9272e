#!/bin/bash
# r06u: the latency harness gives each worker its own UMEM, as the reference
# does (src/dqdk.c:562): its -m gpu tests, then the drop-in latency sweep.
set -e
tag=${1:-r06u}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_c_harness.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_harness_$tag.log 2>&1
timeout -k 10 700 python3 -u tools/dropin_latency.py --out gpurun_out/dropin_$tag.jsonl > gpurun_out/dropin_$tag.log 2>&1
