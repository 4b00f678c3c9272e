#!/bin/bash
# r06l: on the final tree, (a) the N-GPU line as the driver launches it
# (torchrun, 2 ranks sharing the one GPU over gloo: a rehearsal, not a
# scaling point) -- every rank's report and the aggregate roofline; (b)
# DESIGN.md section 7 refreshed: PCIe-inclusive pipeline rates, bench.py
# --e2e, the drop-in latency sweep.
set -e
tag=${1:-r06l}
mkdir -p gpurun_out
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --share-gpu --no-configs > gpurun_out/bench_2rank_$tag.json \
    2> gpurun_out/bench_2rank_$tag.err
bash tools/r05/gpu_r05e.sh $tag
