"""Measured memory bounds on this GPU for the decode's traffic shapes
(membench.hip via the C ABI), one JSON line:

  stream_read      contiguous 16-B loads over a 4 GiB buffer
  mix41            4:1 read:write, contiguous (the decode's ~5.5:1 at 1500 B)
  copy11           1:1 copy
  frames_pattern   1M frames at stride 4096 / 9216, one wave per frame, the
                   frame bytes read and 4 B per event written (the per-frame
                   loop's shape without arithmetic)
  frames_flat      the same bytes, flat grid-stride walk (max loads in flight)

usage: python tools/membench_mix.py [--iters 5]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from dqdk_amd import _lib as L


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    lib = L.lib()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    ms = C.c_double()
    out = {}
    big = 4 << 30
    buf = torch.empty(big, dtype=torch.uint8, device=dev)
    L.check(lib.dqdk_gpu_membench_read(buf.data_ptr(), big, s, args.iters, C.byref(ms)), "read")
    out["stream_read_GB_s"] = round(big / (ms.value * 1e-3) / 1e9, 1)
    dst = torch.empty(big, dtype=torch.uint8, device=dev)
    n, stride = big // 4096, 4096
    # flat = 3: n * stride bytes read contiguously, a quarter of that written
    L.check(lib.dqdk_gpu_membench_frames(buf.data_ptr(), stride, 0, n, dst.data_ptr(), 0, 3, s, args.iters,
                                         C.byref(ms)), "mix41")
    out["mix41_GB_s"] = round(big * 1.25 / (ms.value * 1e-3) / 1e9, 1)
    L.check(lib.dqdk_gpu_membench_frames(buf.data_ptr(), stride, 0, n // 2, dst.data_ptr(), 0, 4, s, args.iters,
                                         C.byref(ms)), "copy11")
    out["copy11_GB_s"] = round(big / 2 * 2 / (ms.value * 1e-3) / 1e9, 1)
    del dst
    keys = torch.empty((1 << 20) * 91, dtype=torch.int32, device=dev)
    for L_, stride_, E in ((1500, 4096, 91), (9000, 9216, 559)):
        nf = 1 << 20
        fb = (L_ + 15) // 16 * 16
        if nf * stride_ > big:
            buf = torch.empty(nf * stride_, dtype=torch.uint8, device=dev)
        if E * nf > keys.numel():
            keys = torch.empty(nf * E, dtype=torch.int32, device=dev)
        L.check(lib.dqdk_gpu_membench_frames(buf.data_ptr(), stride_, fb, nf, keys.data_ptr(), 4 * E, 0, s, args.iters,
                                             C.byref(ms)), "frames pattern")
        out[f"frames_pattern_{L_}_GB_s"] = round(nf * (fb + 4 * E) / (ms.value * 1e-3) / 1e9, 1)
        L.check(lib.dqdk_gpu_membench_frames(buf.data_ptr(), stride_, fb, nf, keys.data_ptr(), 4 * E, 1, s, args.iters,
                                             C.byref(ms)), "frames flat")
        out[f"frames_flat_{L_}_GB_s"] = round(nf * (fb + 4 * E) / (ms.value * 1e-3) / 1e9, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
