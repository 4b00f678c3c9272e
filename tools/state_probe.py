#!/usr/bin/env python3
"""Where the per-process 9000 B speed state lives: in one
process, several device UMEM images holding the same frames (each its own
contiguous allocation, plus one from torch's allocator) decoded by several
queues (each with its own staging allocations), every (image, queue) pair
timed interleaved.  If the decode time follows the image or the queue within
one process, the state is the placement of that allocation; if every pair
runs alike and only processes differ, it is process-wide.  Prints one JSON
line.

usage: python tools/state_probe.py [--frames 1048576] [--frame-len 9000] [--images 3] [--queues 2] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import bench  # noqa: E402  (its synthetic-UMEM helpers)
import dqdk_amd as D  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--frame-len", type=int, default=9000)
    ap.add_argument("--images", type=int, default=3)
    ap.add_argument("--queues", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=6)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    L, n = args.frame_len, args.frames
    stride = 4096 if L <= 4096 else 9216
    size = bench.umem_size(D, n, L, stride, 0)
    bufs = [D.DeviceBuffer(0, size) for _ in range(args.images)]  # images first, as bench.py does
    d0, d_desc, desc, _, _ = bench.synth_to_device(D, torch, dev, n, L, stride, 0, image=bufs[0])
    imgs = [("contig0", bufs[0], d0)]
    for k in range(1, args.images):
        t = bufs[k].tensor[:size]
        t.copy_(d0)
        imgs.append((f"contig{k}", bufs[k], t))
    tt = torch.empty(size, dtype=torch.uint8, device=dev)
    tt.copy_(d0)
    imgs.append(("torch", None, tt))
    cfg = D.RxConfig(payloadsz=L - 42, flags=D.F_CSUM)
    stream = torch.cuda.current_stream(dev)
    queues = []
    for _ in range(args.queues):
        q = D.RxQueue(0, cfg, n)
        q.set_stream(stream.cuda_stream)
        queues.append(q)
    d_res = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
    times = {}
    for rep in range(args.reps):
        for qi, q in enumerate(queues):
            for name, _, t in imgs:
                for _ in range(2):  # warm
                    q.process_device(t.data_ptr(), size, d_desc.data_ptr(), n, d_res.data_ptr(), None)
                torch.cuda.synchronize(dev)
                q.read_timing()
                q.timing_stages(["rx_decode"])
                q.enable_timing(True)
                for _ in range(args.steps):
                    q.process_device(t.data_ptr(), size, d_desc.data_ptr(), n, d_res.data_ptr(), None)
                torch.cuda.synchronize(dev)
                q.enable_timing(False)
                s = q.read_timing()["rx_decode"]
                times.setdefault(f"q{qi}/{name}", []).append(round(s["ms"] / s["launches"], 4))
    # the same image and queue, the fused pieces moved inside their allocation
    import os
    shifts = {}
    q = queues[0]
    name, _, t = imgs[0]
    for rep in range(args.reps):
        for kib in (0, 64, 256, 1024, 2048, 4096, 8192, 16384):
            os.environ["DQDK_GPU_PIECE_SHIFT"] = str(kib)
            for _ in range(2):
                q.process_device(t.data_ptr(), size, d_desc.data_ptr(), n, d_res.data_ptr(), None)
            torch.cuda.synchronize(dev)
            q.read_timing()
            q.timing_stages(["rx_decode"])
            q.enable_timing(True)
            for _ in range(args.steps):
                q.process_device(t.data_ptr(), size, d_desc.data_ptr(), n, d_res.data_ptr(), None)
            torch.cuda.synchronize(dev)
            q.enable_timing(False)
            s = q.read_timing()["rx_decode"]
            shifts.setdefault(f"q0/{name}/shift{kib}K", []).append(round(s["ms"] / s["launches"], 4))
    os.environ.pop("DQDK_GPU_PIECE_SHIFT", None)
    # cheap per-image probes: do they separate the images the decode runs slow on?
    import ctypes as C
    from dqdk_amd import _lib as LB
    ms = C.c_double()
    fb = (L + 15) // 16 * 16
    keys = torch.empty(n * ((L - 42) // 16), dtype=torch.int32, device=dev)
    probes = {}
    for name, _, t in imgs:
        LB.check(LB.lib().dqdk_gpu_membench_read(t.data_ptr(), size, stream.cuda_stream, 3, C.byref(ms)), "read")
        rd = size / (ms.value * 1e-3) / 1e9
        LB.check(LB.lib().dqdk_gpu_membench_frames(t.data_ptr(), stride, fb, n, None, 0, 0, stream.cuda_stream, 3,
                                                   C.byref(ms)), "frames")
        fr = n * fb / (ms.value * 1e-3) / 1e9
        LB.check(LB.lib().dqdk_gpu_membench_frames(t.data_ptr(), stride, fb, n, keys.data_ptr(), 4 * ((L - 42) // 16), 0,
                                                   stream.cuda_stream, 3, C.byref(ms)), "frames+w")
        fw = n * (fb + 4 * ((L - 42) // 16)) / (ms.value * 1e-3) / 1e9
        n4 = min(size // 4096, keys.numel() * 4 // (4 * 91))
        LB.check(LB.lib().dqdk_gpu_membench_frames(t.data_ptr(), 4096, 1504, n4, keys.data_ptr(), 4 * 91, 0,
                                                   stream.cuda_stream, 3, C.byref(ms)), "frames4k+w")
        f4 = n4 * (1504 + 4 * 91) / (ms.value * 1e-3) / 1e9
        probes[name] = {"stream_read_GB_s": round(rd, 1), "frames_read_GB_s": round(fr, 1), "frames_rw_GB_s": round(fw, 1),
                        "frames4k_rw_GB_s": round(f4, 1)}
    pr = torch.cuda.get_device_properties(0)
    out = {"bdf": "%04x:%02x:%02x.0" % (getattr(pr, "pci_domain_id", 0), pr.pci_bus_id, pr.pci_device_id),
           "frame_len": L, "frames": n, "decode_ms": times, "piece_shift_ms": shifts, "probes": probes,
           "va_mod_2MiB": {name: (t.data_ptr() % (2 << 20)) for name, _, t in imgs}}
    print(json.dumps(out), flush=True)
    for q in queues:
        q.close()
    for b in bufs:
        b.close()


if __name__ == "__main__":
    main()
