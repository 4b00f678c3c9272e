#!/bin/bash
# Round 6, final tree (r06o's library, whose -m gpu suite passed): smoke(),
# the default bench line, rocprofv3 kernel stats of the bench command at
# both sizes.
# usage (on the GPU box): bash tools/r06/gpu_r06p.sh <tag>
set -e
tag=${1:-r06p}
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.txt 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
bash tools/prof.sh $tag
