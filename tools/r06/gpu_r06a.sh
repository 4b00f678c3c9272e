#!/bin/bash
# r06a: the host-reuse ordering of VERDICT r5 item 1 alone, then the whole
# -m gpu suite once (per-test device check in tests/conftest.py), then the
# default bench line.  Stops at the first failure.
set -e
tag=${1:-r06a}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_host_reuse.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_reuse_$tag.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
# the decode's ceiling: shipped vs the ceiling variants
# (tools/ab_build.sh base wt; EXTRA_FLAGS=-DDQDK_CEIL=1|2 ... ceil1|ceil2 wt)
bash tools/ab_run.sh ceil_$tag "--no-9000 --no-configs --no-box-state" base ceil1 ceil2
