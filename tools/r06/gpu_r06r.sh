#!/bin/bash
# r06r: phase A reading a frame's second 64 B only when its headers reach
# them (-DDQDK_HDR64=1): same-box A/B of the headline (base = HEAD, hdr0 =
# the new load form with the option off, hdr64) and of configs[1]'s
# records-path decode, then the parity suites on the hdr64 library.
set -e
tag=${1:-r06r}
mkdir -p gpurun_out
bash tools/ab_run.sh hdr_$tag "--no-9000 --no-configs --no-box-state" base hdr0 hdr64
bash tools/ab_run.sh hdrc1_$tag "--frames 262144 --no-histo --no-records --rotate 4 --no-9000 --no-configs --no-box-state" \
    base hdr64
DQDK_GPU_LIB=$PWD/build/ab/hdr64.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_configs.py tests/test_gpu_fused_head.py tests/test_gpu_pinned.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_hdr64_$tag.log 2>&1
