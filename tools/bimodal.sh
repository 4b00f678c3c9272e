#!/bin/bash
# 9000 B decode bimodality probe: separate processes, torch-allocated vs
# contiguous (hipDeviceMallocContiguous) UMEM images, interleaved.
# usage (GPU box): bash tools/bimodal.sh <tag> [rounds]
tag=${1:-bm}; rounds=${2:-4}
d=gpurun_out/bimodal_$tag
mkdir -p $d
for r in $(seq 1 $rounds); do
    for a in torch contig; do
        timeout -k 10 200 python3 bench.py --frame-len 9000 --steps 10 --warmup 2 --no-cpu-baseline --umem-alloc $a \
            > $d/${a}_$r.json 2> $d/${a}_$r.err || exit $?
    done
done
python3 - "$d" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    x = json.loads(open(f).read().strip().splitlines()[-1])
    r = x["roofline"]
    print(f.split("/")[-1], x["value"], x["kernels"]["rx_decode"]["avg_ms"], r["umem_image"]["va"], r["umem_image"]["va_mod_2MiB"],
          r["measured_stream_read_GB_s"])
PY
