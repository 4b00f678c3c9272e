#!/bin/bash
# Same-box A/B of build/ab/*.so variants at both frame sizes.
# usage: bash tools/gpu_ab.sh <tag> name1 name2 ...
set -e
tag=$1; shift
bash tools/ab_run.sh ${tag}_1500 "" "$@"
bash tools/ab_run.sh ${tag}_9000 "--frame-len 9000" "$@"
