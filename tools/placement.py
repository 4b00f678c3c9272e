#!/usr/bin/env python3
"""Decode time vs the UMEM image's position inside one contiguous device
arena (the 9000 B decode is 2.27 or 2.45 ms depending on where the image
lands).  The arena holds n + extra synthetic frames at the
UMEM stride; an image at offset k * stride is frames k .. k + n of it, so
every placement decodes the same kind of frames.

usage (GPU box): python3 tools/placement.py [--frame-len 9000] [--max-gb 8] [--step-gb 0.5]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frame-len", type=int, default=9000)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--max-gb", type=float, default=8.0)
    ap.add_argument("--step-gb", type=float, default=0.5)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import torch

    import dqdk_amd as D

    L, n = a.frame_len, a.frames
    stride = 4096 if L <= 4096 else 9216
    extra = int(a.max_gb * (1 << 30)) // stride + 1
    tot = n + extra
    dev = torch.device("cuda", 0)
    arena = D.DeviceBuffer(0, tot * stride)
    t = arena.tensor
    chunk = 1 << 16
    desc0 = None
    t0 = time.time()
    for f0 in range(0, tot, chunk):
        m = min(chunk, tot - f0)
        u, d = D.synth_umem(m, L, stride, first=f0, threads=16)
        t[f0 * stride:f0 * stride + u.size].copy_(torch.from_numpy(u))
        if f0 == 0:
            desc0 = d
    # descriptors of frames 0 .. n at the stride (frame content is position-independent in the arena)
    desc = np.zeros(n, dtype=desc0.dtype)
    desc["addr"] = np.arange(n, dtype=np.uint64) * stride
    desc["len"] = L
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    cfg = D.RxConfig(payloadsz=L - 42, flags=D.F_CSUM)
    d_res = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
    q = D.RxQueue(0, cfg, n)
    q.timing_stages(["rx_decode"])
    q.enable_timing(True)
    print(json.dumps({"arena_va": hex(arena.ptr), "contiguous": arena.contiguous, "synth_s": round(time.time() - t0, 1)}),
          flush=True)
    offs = np.arange(0, a.max_gb + 1e-9, a.step_gb)
    for rnd in range(2):
        for og in offs:
            k = int(og * (1 << 30)) // stride
            base = arena.ptr + k * stride
            for _ in range(2):
                q.process_device(base, n * stride, d_desc.data_ptr(), n, d_res.data_ptr(), None)
            torch.cuda.synchronize(dev)
            q.read_timing()
            for _ in range(a.iters):
                q.process_device(base, n * stride, d_desc.data_ptr(), n, d_res.data_ptr(), None)
            tm = q.read_timing()["rx_decode"]
            print(json.dumps({"round": rnd, "off_gb": round(float(og), 3), "va": hex(base),
                              "decode_ms": round(tm["ms"] / max(tm["launches"], 1), 4)}), flush=True)
    q.close()
    arena.close()


if __name__ == "__main__":
    main()
