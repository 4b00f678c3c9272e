#!/bin/bash
# Same-box PMC comparison of build/ab/<lib>.so builds (A/B diagnostics).
# usage (on the GPU box): bash tools/pmc_ab.sh <tag> <lib> "<counter group>" [bench args]
set -e
tag=$1; lib=$2; grp=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/pmcab_$tag; mkdir -p $d
DQDK_GPU_LIB=$PWD/build/ab/$lib.so timeout -k 10 200 rocprofv3 --pmc $grp -d $d -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-9000 "$@" > $d/run.log 2>&1
