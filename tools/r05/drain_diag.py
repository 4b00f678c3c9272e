#!/usr/bin/env python3
"""Round 5, call af: is the 9000 B decode's slow state the decode itself on
its buffers, or the decode overlapping what runs before it?  One process, one
1M x 9000 B image at a time (bench.py's synthetic frames, physically
contiguous; two images in turn), three queues per image with the staging
probe off (each keeps its first piece
buffer: the allocator's placement, slow or fast).  Per queue, the decode's
event-timed ms over 12 batches back to back ("chain", as in the bench), then
12 batches each after a host-side drain of the device ("drained"), then 12
with a 5 ms idle gap after the drain ("idle"), the three twice in turn.
usage (on the GPU box): python3 tools/r05/drain_diag.py > gpurun_out/r05af.json
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import dqdk_amd as D  # noqa: E402

os.environ["DQDK_GPU_STAGING_PROBE"] = "0"
dev = torch.device("cuda:0")
n, L, stride = 1 << 20, 9000, 9216
cfg = D.RxConfig(payloadsz=L - 42, flags=D.F_CSUM)
d_res = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
out = {"what": __doc__.split("\n\n")[0], "queues": []}
owner = None
for qi in range(6):
    if qi % 3 == 0:
        d_umem = d_desc = None
        if owner is not None:
            owner.close()
        torch.cuda.synchronize(dev)
        d_umem, d_desc, desc, _, owner = bench.synth_to_device(D, torch, dev, n, L, stride, queue=qi // 3,
                                                               alloc="contig")
        bench.progress(f"image {qi // 3} resident")
    q = D.RxQueue(0, cfg, n)
    stream = torch.cuda.current_stream(dev)
    q.set_stream(stream.cuda_stream)

    def step():
        q.process_device(d_umem.data_ptr(), d_umem.numel(), d_desc.data_ptr(), n, d_res.data_ptr(), None)

    for _ in range(3):
        step()
    q.flush_histogram()
    torch.cuda.synchronize(dev)
    q.timing_stages(["rx_decode"])
    rec = {}
    for rnd in range(2):
        for mode in ("chain", "drained", "idle"):
            q.read_timing()
            q.enable_timing(True)
            for _ in range(12):
                if mode != "chain":
                    torch.cuda.synchronize(dev)
                    if mode == "idle":
                        time.sleep(0.005)
                step()
            torch.cuda.synchronize(dev)
            q.enable_timing(False)
            t = q.read_timing()["rx_decode"]
            rec.setdefault(mode, []).append(round(t["ms"] / t["launches"], 4))
            bench.progress(f"queue {qi} round {rnd} {mode}: {rec[mode][-1]} ms")
    q.flush_histogram()
    torch.cuda.synchronize(dev)
    rec["image"] = qi // 3
    out["queues"].append(rec)
    q.close()
print(json.dumps(out))
