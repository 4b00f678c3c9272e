#!/bin/bash
# Round 5's final evidence on one box, from the final tree: the -m gpu suite,
# smoke(), PMC traffic of the decode regenerated from scratch (both sizes,
# calibrated FETCH_SIZE x 2 + WRITE_SIZE: tools/pmc.sh), LDS counters of the
# chain (rx_part2's bank-conflict share), the default bench line reading that
# traffic, rocprofv3 kernel stats of the bench command at both sizes.
# usage (on the GPU box): bash tools/r05/gpu_final_r05.sh <tag>
set -e
tag=${1:-r05z}
mkdir -p gpurun_out
rm -f gpurun_out/pmc_summary.json
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.txt 2>&1
bash tools/pmc.sh $tag 1500
bash tools/pmc.sh $tag 9000
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in 1500 9000; do
    timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
        SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/pmc_lds_${tag}_$L -o run \
        --output-format csv -- python3 bench.py --frame-len $L --steps 3 --warmup 1 --no-cpu-baseline --no-9000 \
        --no-box-state > gpurun_out/pmc_lds_${tag}_$L.log 2>&1
done
timeout -k 10 400 python3 bench.py --pmc gpurun_out/pmc_summary.json > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
bash tools/prof.sh $tag
