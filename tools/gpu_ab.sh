#!/bin/bash
# One GPU call of an A/B experiment: GPU parity tests of the candidate build
# (the last one named), then tools/ab_run.sh over every named build.
# usage (GPU box): bash tools/gpu_ab.sh <tag> "<pytest -k expression | all | none>" "<bench args>" build...
# (builds: build/ab/<name>.so from tools/ab_build.sh)
set -e
tag=$1; k=$2; bargs=$3; shift 3
cand=${@: -1}
mkdir -p gpurun_out
if [ "$k" = all ]; then
    DQDK_GPU_LIB=$PWD/build/ab/$cand.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 \
        --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
elif [ "$k" != none ]; then
    DQDK_GPU_LIB=$PWD/build/ab/$cand.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py \
        tests/test_gpu_fullsize.py -k "$k" -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
fi
bash tools/ab_run.sh $tag "$bargs" "$@"
