#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) receive pipeline, SURVEY §8(d) "End-to-end".

Host UMEM batches (pinned, as an AF_XDP UMEM registered with the GPU would
be) stream through the GPU path with three HIP streams:

    h2d stream : frames + descriptors of batch b -> device slot b % depth
    rx stream  : dqdk_gpu_rx_batch_device on that slot (decode, counters,
                 histogram into the queue's HBM table)
    d2h stream : per-frame results (8 B) [+ decoded records, 4 B/event]
                 of batch b back to pinned host buffers

so copies in both directions overlap the kernels of neighbouring batches.
Reports packets/s and PCIe GB/s over the whole run, plus the zero-copy
host drop-in (dqdk_gpu_rx_batch on mapped UMEM) for comparison.  Prints one
JSON object; DESIGN.md quotes it.  Not the bench.py metric (that one is
device-resident by definition).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=1 << 18, help="frames per batch")
    p.add_argument("--batches", type=int, default=48)
    p.add_argument("--images", type=int, default=4, help="distinct host batch images cycled through")
    p.add_argument("--depth", type=int, default=3)
    p.add_argument("--frame-len", type=int, default=1500)
    p.add_argument("--stride", type=int, default=0)
    p.add_argument("--records", action="store_true", help="also copy decoded records back")
    p.add_argument("--no-csum", action="store_true")
    p.add_argument("--copy", choices=["image", "frames"], default="frames",
                   help="H2D the whole UMEM image, or only the first frame_len bytes of each chunk "
                        "(one strided hipMemcpy2DAsync; UMEM layout and descriptors unchanged)")
    p.add_argument("--no-zero-copy", action="store_true")
    args = p.parse_args()

    import torch

    import dqdk_amd as D
    dev = torch.device("cuda", 0)
    L = args.frame_len
    stride = args.stride or (4096 if L <= 4096 else 9216)
    n = args.frames
    cfg = D.RxConfig(payloadsz=L - 42, mode=D.MODE_ENERGYHISTO, flags=0 if args.no_csum else D.F_CSUM)
    E = cfg.events

    # host side: pinned batch images (frames at addr = slot*stride within the batch)
    imgs, descs = [], []
    for i in range(args.images):
        u, d = D.synth_umem(n, L, stride, queue=i, threads=16)
        t = torch.from_numpy(u).pin_memory()
        imgs.append(t)
        descs.append(torch.from_numpy(d.view(np.uint8)).pin_memory())
    umem_bytes = imgs[0].numel()

    # strided copy: rows of `width` bytes at pitch `stride` (frames sit at addr = i * stride)
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy2DAsync.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t,
                                     C.c_int, C.c_void_p]
    width = (L + 63) // 64 * 64
    assert width <= stride

    def h2d_frames(dst, src, stream):
        rc = hip.hipMemcpy2DAsync(dst.data_ptr(), stride, src.data_ptr(), stride, width, n, 1, stream.cuda_stream)
        assert rc == 0, f"hipMemcpy2DAsync failed: {rc}"

    q = D.RxQueue(0, cfg, n)
    s_h2d, s_rx, s_d2h = (torch.cuda.Stream(dev) for _ in range(3))
    q.set_stream(s_rx.cuda_stream)
    slots = []
    for _ in range(args.depth):
        slots.append({
            "umem": torch.empty(umem_bytes, dtype=torch.uint8, device=dev),
            "desc": torch.empty(n * 16, dtype=torch.uint8, device=dev),
            "res": torch.empty(n * 8, dtype=torch.uint8, device=dev),
            "keys": torch.empty(max(n * E, 1), dtype=torch.int32, device=dev),
            "h_res": torch.empty(n * 8, dtype=torch.uint8).pin_memory(),
            "h_keys": torch.empty(max(n * E, 1), dtype=torch.int32).pin_memory() if args.records else None,
            "copied": torch.cuda.Event(), "done": torch.cuda.Event(), "out": torch.cuda.Event(),
            "used": False,
        })

    def run(nb):
        for b in range(nb):
            sl = slots[b % args.depth]
            img = b % args.images
            with torch.cuda.stream(s_h2d):
                if sl["used"]:
                    s_h2d.wait_event(sl["done"])  # kernels of batch b-depth finished reading the slot
                if args.copy == "image":
                    sl["umem"].copy_(imgs[img], non_blocking=True)
                else:
                    h2d_frames(sl["umem"], imgs[img], s_h2d)
                sl["desc"].copy_(descs[img], non_blocking=True)
                sl["copied"].record(s_h2d)
            s_rx.wait_event(sl["copied"])
            if sl["used"]:
                s_rx.wait_event(sl["out"])  # results of batch b-depth copied out
            q.process_device(sl["umem"].data_ptr(), umem_bytes, sl["desc"].data_ptr(), n, sl["res"].data_ptr(),
                             sl["keys"].data_ptr())
            sl["done"].record(s_rx)
            with torch.cuda.stream(s_d2h):
                s_d2h.wait_event(sl["done"])
                sl["h_res"].copy_(sl["res"], non_blocking=True)
                if args.records:
                    sl["h_keys"].copy_(sl["keys"], non_blocking=True)
                sl["out"].record(s_d2h)
            sl["used"] = True
        torch.cuda.synchronize(dev)

    run(args.depth)  # warm-up
    q.reset_counters()
    t0 = time.perf_counter()
    run(args.batches)
    sec = time.perf_counter() - t0
    cnt = q.counters()
    assert cnt["rcvd_pkts"] == n * args.batches, cnt
    for sl in slots:
        r = sl["h_res"].numpy().view(D.RESULT_DTYPE)
        assert (r["status"] == D.RX_OK).all()

    pk = n * args.batches
    h2d = ((umem_bytes if args.copy == "image" else n * width) + n * 16) * args.batches
    d2h = (n * 8 + (n * E * 4 if args.records else 0)) * args.batches
    out = {
        "pipeline": f"pinned H2D ({args.copy}) -> rx -> D2H, depth {args.depth}, {n} frames/batch",
        "frame_len": L, "stride": stride, "batches": args.batches, "records_d2h": args.records,
        "csum": not args.no_csum,
        "Mpkt_s": round(pk / sec / 1e6, 3),
        "frame_GB_s": round(pk * L / sec / 1e9, 2),
        "pcie_h2d_GB_s": round(h2d / sec / 1e9, 2),
        "pcie_d2h_GB_s": round(d2h / sec / 1e9, 2),
    }

    if args.no_zero_copy:
        q.close()
        print(json.dumps(out), flush=True)
        return
    # zero-copy host drop-in (dqdk_gpu_rx_batch): kernels read the mapped UMEM over PCIe
    # a fresh (pageable) image: hipHostRegister refuses memory torch has already pinned
    del imgs, slots
    umem_np, desc_np = D.synth_umem(n, L, stride, queue=0, threads=16)
    q.use_own_stream()
    q.register_umem(umem_np)
    q.process_batch(umem_np, desc_np)
    t0 = time.perf_counter()
    nz = 8
    for _ in range(nz):
        res, _ = q.process_batch(umem_np, desc_np)
    sz = time.perf_counter() - t0
    assert (res["status"] == D.RX_OK).all()
    out["zero_copy_dropin_Mpkt_s"] = round(n * nz / sz / 1e6, 3)
    out["zero_copy_dropin_frame_GB_s"] = round(n * nz * L / sz / 1e9, 2)
    q.unregister_umem(umem_np)
    q.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
