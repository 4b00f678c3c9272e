#!/usr/bin/env python3
"""Calibrate rocprofv3 WRITE_SIZE for 4-B-per-lane stores (MI355X_MICROARCH.md:
WRITE_SIZE is exact only for 16-B-per-lane streaming stores).  Runs the
membench store kernels with known byte counts; run it under
`rocprofv3 --pmc WRITE_SIZE` and compare per-dispatch WRITE_SIZE with the
bytes printed here (tools/pmc_summary.py does the division).
Modes: aligned 256-B dword runs, and unaligned runs of 60 / 30 dwords
(the fused decode's piece flush)."""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from dqdk_amd import _lib as L  # noqa: E402


def main():
    n = 1 << 22  # wave instructions
    out = torch.empty(n * 256 + (1 << 20), dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    ms = C.c_double()
    res = {}
    for name, obytes in (("aligned_256B", 0), ("run60", 240), ("run30", 120)):
        L.check(L.lib().dqdk_gpu_membench_frames(None, 0, 0, n, out.data_ptr(), obytes, 5, s, 2, C.byref(ms)),
                "membench store")
        per = obytes if obytes else 256
        res[name] = {"bytes_per_dispatch": n * per, "ms": round(ms.value, 4),
                     "GB_s": round(n * per / (ms.value * 1e-3) / 1e9, 1), "dispatches": 3}
    torch.cuda.synchronize()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
