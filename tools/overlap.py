#!/usr/bin/env python3
"""Feasibility probe: does a batch's histogram chain overlap the next batch's
decode?  Two queues on two streams take alternate batches of the same
device-resident workload (each its own table and staging) vs one queue;
DQDK_GPU_DECODE_CUS caps the fused decode's persistent grid, leaving CUs to
the other stream's kernels.  Prints Mpkt/s per mode.

usage (GPU box): python3 tools/overlap.py [--frame-len 1500] [--steps 20]
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
    ap.add_argument("--frame-len", type=int, default=1500)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--queues", type=int, default=2)
    a = ap.parse_args()
    import torch

    import dqdk_amd as D

    L, n = a.frame_len, a.frames
    stride = 4096 if L <= 4096 else 9216
    dev = torch.device("cuda", 0)
    img = D.DeviceBuffer(0, n * stride)
    t = img.tensor
    descs = []
    for f0 in range(0, n, 1 << 16):
        m = min(1 << 16, n - f0)
        u, d = D.synth_umem(m, L, stride, first=f0, threads=16)
        t[f0 * stride:f0 * stride + u.size].copy_(torch.from_numpy(u))
        d = d.copy()
        d["addr"] += f0 * stride
        descs.append(d)
    desc = np.concatenate(descs)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    cfg = D.RxConfig(payloadsz=L - 42, flags=D.F_CSUM)
    nq = a.queues
    qs = [D.RxQueue(0, cfg, n) for _ in range(nq)]
    ss = [torch.cuda.Stream(dev) for _ in range(nq)]
    res = [torch.zeros(n * 8, dtype=torch.uint8, device=dev) for _ in range(nq)]
    for q, s in zip(qs, ss):
        q.set_stream(s.cuda_stream)

    def run(k):
        for i in range(k):
            j = i % nq
            qs[j].process_device(img.ptr, n * stride, d_desc.data_ptr(), n, res[j].data_ptr(), None)
        for q in qs:
            q.flush_histogram()

    run(2 * nq)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(a.steps)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    print(json.dumps({"frame_len": L, "queues": nq, "steps": a.steps, "ms_per_step": round(dt / a.steps * 1e3, 4),
                      "Mpkt_s": round(n * a.steps / dt / 1e6, 1)}), flush=True)
    for q in qs:
        q.close()
    img.close()


if __name__ == "__main__":
    main()
