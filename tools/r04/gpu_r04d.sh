#!/bin/bash
# Round 4, call d: the test sequence that ended in an illegal-address error in
# call b (bench rehearsal -> egress -> parity golden), with kernels and copies
# serialized so an error is reported by the launch that caused it; then the
# rest of the -m gpu suite, the drop-in latency sweep and the bench line.
# usage (on the GPU box): bash tools/r04/gpu_r04d.sh <tag>
set -e
tag=${1:-r04d}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_bench_launch.py \
    tests/test_gpu_egress.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_serial_$tag.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    --deselect tests/test_bench_launch.py --deselect tests/test_gpu_egress.py --deselect tests/test_gpu_parity.py \
    --deselect tests/test_gpu_fullsize.py --deselect tests/test_gpu_configs.py > gpurun_out/pytest_gpu_$tag.log 2>&1
timeout -k 10 600 python3 -u tools/dropin_latency.py --out gpurun_out/dropin_$tag.jsonl > gpurun_out/dropin_$tag.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
