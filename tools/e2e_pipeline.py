#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) receive rates for DESIGN.md §7 (tools/gpu_e2e.sh).

The pinned H2D -> kernels -> D2H pipeline is dqdk_amd.pipeline.E2EPipeline
(the same one `bench.py --e2e` runs for BASELINE configs[4]); this script
adds the variants DESIGN.md compares (whole-image vs frames-only H2D,
records D2H) and the zero-copy host drop-in (dqdk_gpu_rx_batch on mapped
UMEM).  Prints one JSON object.  Never the bench.py `value`.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=1 << 18, help="frames per batch")
    p.add_argument("--batches", type=int, default=48)
    p.add_argument("--depth", type=int, default=3)
    p.add_argument("--frame-len", type=int, default=1500)
    p.add_argument("--stride", type=int, default=0)
    p.add_argument("--records", action="store_true", help="also copy decoded records back")
    p.add_argument("--no-csum", action="store_true")
    p.add_argument("--copy", choices=["image", "frames"], default="frames")
    p.add_argument("--no-zero-copy", action="store_true")
    args = p.parse_args()

    import dqdk_amd as D
    from dqdk_amd.pipeline import E2EPipeline
    L = args.frame_len
    stride = args.stride or (4096 if L <= 4096 else 9216)
    n = args.frames
    cfg = D.RxConfig(payloadsz=L - 42, mode=D.MODE_ENERGYHISTO, flags=0 if args.no_csum else D.F_CSUM)
    pl = E2EPipeline(0, cfg, n, L, stride, depth=args.depth, images=4, records=args.records, copy=args.copy)
    pl.run(args.depth)  # warm-up
    r = pl.run(args.batches)
    pl.close()
    out = {"pipeline": f"pinned H2D ({args.copy}) -> rx -> D2H, depth {args.depth}, {n} frames/batch",
           "frame_len": L, "stride": stride, "batches": args.batches, "records_d2h": args.records,
           "csum": not args.no_csum, "Mpkt_s": round(r["Mpkt_s"], 3), "frame_GB_s": round(r["frame_GB_s"], 2),
           "pcie_h2d_GB_s": round(r["pcie_h2d_GB_s"], 2), "pcie_d2h_GB_s": round(r["pcie_d2h_GB_s"], 2),
           "batch_latency_ms": {k: round(v, 3) for k, v in r["batch_latency_ms"].items()}}
    if not args.no_zero_copy:
        # zero-copy host drop-in: the kernels read the registered (mapped) UMEM over PCIe
        umem, desc = D.synth_umem(n, L, stride, queue=0, threads=16)
        with D.RxQueue(0, cfg, n) as q:
            q.register_umem(umem)
            q.process_batch(umem, desc)
            t0 = time.perf_counter()
            nz = 8
            for _ in range(nz):
                res, _ = q.process_batch(umem, desc)
            sz = time.perf_counter() - t0
            assert (res["status"] == D.RX_OK).all()
            q.unregister_umem(umem)
        out["zero_copy_dropin_Mpkt_s"] = round(n * nz / sz / 1e6, 3)
        out["zero_copy_dropin_frame_GB_s"] = round(n * nz * L / sz / 1e9, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
