#!/bin/bash
# GPU tests with every kernel launch and every copy serialised, so that a GPU
# fault is reported by the operation that caused it.
# HIP's runtime reads AMD_SERIALIZE_KERNEL / AMD_SERIALIZE_COPY itself (3 =
# wait before and after each launch / copy); torch also parses
# AMD_SERIALIZE_KERNEL, as a boolean, and warns "valid values are 0 or 1" for
# 3 -- that warning is torch's, HIP still serialises.  HIP_LAUNCH_BLOCKING=1
# makes torch's own launches synchronous too.
# usage (GPU box): bash tools/serial_pytest.sh <tag> [pytest args...]
set -e
tag=${1:-serial}; shift || true
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 HIP_LAUNCH_BLOCKING=1 timeout -k 10 900 \
    python3 -u -m pytest -m gpu -x -v --timeout 240 --timeout-method thread "${@:-tests}" \
    > gpurun_out/pytest_serial_$tag.log 2>&1
