"""End-to-end (PCIe-inclusive) receive pipeline for one queue on one GPU.

SURVEY §8(d) "End-to-end" / BASELINE configs[4]: the path starts in host
memory (AF_XDP UMEM hugepages, src/dqdk-mem.c:12-28) and ends there (decoded
results; optionally the decoded records).  Host UMEM batches (pinned, as a
registered AF_XDP UMEM would be) stream through the GPU with three HIP
streams so copies in both directions overlap the kernels of neighbouring
batches:

    h2d stream : frames + descriptors of batch b -> device slot b % depth
    rx stream  : dqdk_gpu_rx_batch_device on that slot (decode, counters,
                 histogram into the queue's HBM table)
    d2h stream : per-frame results (8 B) [+ decoded records, 4 B/event]
                 of batch b back to pinned host buffers

Replay can be paced to an offered load (e.g. 100 Gbit/s over all queues):
batch b is released at b * batch_bytes / rate, and its latency is measured
from release to its results landing in host memory.  These rates include
PCIe and are never bench.py's device-resident `value`.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np
import torch

from . import rx as R
from . import _lib as L

_hip = None


def _hip_lib():
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipMemcpy2DAsync.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t,
                                          C.c_int, C.c_void_p]
    return _hip


class E2EPipeline:
    """depth device slots cycling over `images` pinned host batch images."""

    def __init__(self, device: int, cfg: R.RxConfig, n: int, frame_len: int, stride: int, queue: int = 0,
                 depth: int = 3, images: int = 2, records: bool = False, copy: str = "frames",
                 faulty: bool = False):
        """records=False hands the decode no record buffer: a histogram batch
        then takes the default (fused) decode, as bench.py's device-resident
        line does; records=True writes frame-order records and copies them
        back (the unfused path)."""
        assert copy in ("frames", "image")
        self.dev = torch.device("cuda", device)
        self.n, self.L, self.stride, self.depth, self.records, self.copy = n, frame_len, stride, depth, records, copy
        self.cfg = cfg
        E = cfg.events
        self.imgs, self.descs = [], []
        for i in range(images):
            u, d = R.synth_umem(n, frame_len, stride, queue=queue, first=i * n, threads=16, faulty=faulty)
            d = d.copy()  # addresses are relative to the image
            self.imgs.append(torch.from_numpy(u).pin_memory())
            self.descs.append(torch.from_numpy(d.view(np.uint8)).pin_memory())
            self.frame_bytes = int(d["len"].astype(np.int64).sum())
        self.umem_bytes = self.imgs[0].numel()
        # only the first roundup(L, 64) bytes of each UMEM chunk cross the link
        # (mixed sizes: the largest frame); layout and descriptors unchanged
        self.width = min(stride, (max(frame_len, 9000 if frame_len == 0 else frame_len) + 63) // 64 * 64)
        self.q = R.RxQueue(device, cfg, n)
        self.s_h2d, self.s_rx, self.s_d2h = (torch.cuda.Stream(self.dev) for _ in range(3))
        self.q.set_stream(self.s_rx.cuda_stream)
        self.slots = []
        self.bufs = []  # the slots' UMEM images: library device allocations (contiguous where possible)
        for _ in range(depth):
            self.bufs.append(R.DeviceBuffer(device, self.umem_bytes))
            self.slots.append({
                "umem": self.bufs[-1].tensor,
                "desc": torch.empty(n * 16, dtype=torch.uint8, device=self.dev),
                "res": torch.empty(n * 8, dtype=torch.uint8, device=self.dev),
                "keys": torch.empty(max(n * E, 1), dtype=torch.int32, device=self.dev) if records else None,
                "h_res": torch.empty(n * 8, dtype=torch.uint8).pin_memory(),
                "h_keys": torch.empty(max(n * E, 1), dtype=torch.int32).pin_memory() if records else None,
                "copied": torch.cuda.Event(), "done": torch.cuda.Event(), "out": torch.cuda.Event(),
                "used": False,
            })

    def _h2d(self, sl, img):
        if self.copy == "image":
            sl["umem"].copy_(self.imgs[img], non_blocking=True)
        else:
            rc = _hip_lib().hipMemcpy2DAsync(sl["umem"].data_ptr(), self.stride, self.imgs[img].data_ptr(), self.stride,
                                             self.width, self.n, 1, self.s_h2d.cuda_stream)
            if rc != 0:
                raise RuntimeError(f"hipMemcpy2DAsync failed: {rc}")
        sl["desc"].copy_(self.descs[img], non_blocking=True)

    def image(self, k: int):
        """Host UMEM image k and its descriptors (batch b replays image b % images)."""
        return self.imgs[k].numpy(), self.descs[k].numpy().view(L.DESC_DTYPE)

    def run(self, nbatches: int, offered_bytes_per_s: float | None = None, on_result=None) -> dict:
        """Replay nbatches batches; paced when offered_bytes_per_s is given.
        Returns rates over the run and per-batch latency (release -> results in host memory).
        on_result(b, results[, records]) is called as each batch's D2H completes (host
        copies of the pinned buffers, before the slot is reused)."""
        period = self.frame_bytes / offered_bytes_per_s if offered_bytes_per_s else 0.0
        torch.cuda.synchronize(self.dev)
        for sl in self.slots:  # the previous run has drained every slot
            sl["used"] = False
        lat = []
        pending = []  # [release time, its results-in-host-memory event], in batch order

        def poll(block=False):
            # a batch's latency ends when its D2H event completes (polled from the host)
            while pending and (block or pending[0][1].query()):
                if block:
                    pending[0][1].synchronize()
                rel, _, b, sl = pending.pop(0)
                lat.append(time.perf_counter() - rel)
                if on_result is not None:
                    r = sl["h_res"].numpy().view(L.RESULT_DTYPE).copy()
                    on_result(b, r, sl["h_keys"].numpy().view(np.uint32).copy() if self.records else None)
                block = False

        t0 = time.perf_counter()
        for b in range(nbatches):
            if period:
                while time.perf_counter() < t0 + b * period:
                    poll()
            release = time.perf_counter()
            sl = self.slots[b % self.depth]
            img = b % len(self.imgs)
            if sl["used"]:
                # slot reuse: batch b - depth's results have reached host memory
                while len(pending) >= self.depth:
                    poll(block=True)
            with torch.cuda.stream(self.s_h2d):
                self._h2d(sl, img)
                sl["copied"].record(self.s_h2d)
            self.s_rx.wait_event(sl["copied"])
            self.q.process_device(sl["umem"].data_ptr(), self.umem_bytes, sl["desc"].data_ptr(), self.n,
                                  sl["res"].data_ptr(), sl["keys"].data_ptr() if self.records else None)
            sl["done"].record(self.s_rx)
            with torch.cuda.stream(self.s_d2h):
                self.s_d2h.wait_event(sl["done"])
                sl["h_res"].copy_(sl["res"], non_blocking=True)
                if self.records:
                    sl["h_keys"].copy_(sl["keys"], non_blocking=True)
                out = torch.cuda.Event()
                out.record(self.s_d2h)
            sl["used"] = True
            pending.append([release, out, b, sl])
            poll()
        while pending:
            poll(block=True)
        self.q.flush_histogram()
        torch.cuda.synchronize(self.dev)
        sec = time.perf_counter() - t0
        pk = self.n * nbatches
        h2d = ((self.umem_bytes if self.copy == "image" else self.n * self.width) + self.n * 16) * nbatches
        d2h = (self.n * 8 + (self.n * self.cfg.events * 4 if self.records else 0)) * nbatches
        lat_ms = np.array(lat) * 1e3
        return {"sec": sec, "packets": pk, "Mpkt_s": pk / sec / 1e6, "frame_GB_s": self.frame_bytes * nbatches / sec / 1e9,
                "pcie_h2d_GB_s": h2d / sec / 1e9, "pcie_d2h_GB_s": d2h / sec / 1e9,
                "batch_latency_ms": {"p50": float(np.percentile(lat_ms, 50)), "p99": float(np.percentile(lat_ms, 99)),
                                     "max": float(lat_ms.max())}}

    def close(self):
        self.q.close()
        torch.cuda.synchronize(self.dev)
        for sl in self.slots:
            sl["umem"] = None
        for b in self.bufs:
            b.close()
