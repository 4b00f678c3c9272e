#!/usr/bin/env python3
"""Host drop-in raw egress rate (dqdk_gpu_rx_batch with a raw fd): the serial
form (gather -> D2H -> write() inside each call, the default) against the
deferred side-stream form (set_raw_fd(fd, deferred=True): D2H on a side
stream, write() of batch b during batch b+1's call).  Waveform mode (the raw-storing mode, src/tristan.c:318-324),
1500 B frames, registered host UMEM, the file in /tmp.  Prints one JSON line."""
import json
import os
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import dqdk_amd as D  # noqa: E402


def rate(sync: bool, n: int, batches: int, mode: int, sink: str = "file") -> dict:
    cfg = D.RxConfig(payloadsz=1458, mode=mode, flags=D.F_CSUM)
    imgs = [D.synth_umem(n, 1500, 4096, queue=k, threads=16) for k in range(2)]
    if sink == "null":
        fd, path = os.open("/dev/null", os.O_WRONLY), None
    else:
        fd, path = tempfile.mkstemp(dir="/tmp")
    try:
        with D.RxQueue(0, cfg, n) as q:
            for u, _ in imgs:
                q.register_umem(u)
            q.set_raw_fd(fd, deferred=not sync)
            q.process_batch(*imgs[0])
            q.sync()
            t0 = time.perf_counter()
            for b in range(batches):
                q.process_batch(*imgs[b % 2])
            q.sync()
            sec = time.perf_counter() - t0
            q.set_raw_fd(-1)
        size = os.path.getsize(path) if path else None
    finally:
        os.close(fd)
        if path:
            os.unlink(path)
    assert size in (None, (batches + 1) * n * 1458), size
    return {"Mpkt_s": round(n * batches / sec / 1e6, 3), "raw_GB_s": round(n * 1458 * batches / sec / 1e9, 3)}


def main():
    n, batches = 1 << 16, 24
    out = {"frames_per_batch": n, "batches": batches, "frame_len": 1500}
    # no raw fd: the host drop-in alone (zero-copy reads of the registered UMEM)
    imgs = [D.synth_umem(n, 1500, 4096, queue=k, threads=16) for k in range(2)]
    with D.RxQueue(0, D.RxConfig(payloadsz=1458, mode=D.MODE_WAVEFORM, flags=D.F_CSUM), n) as q:
        q.process_batch(*imgs[0])
        t0 = time.perf_counter()
        for b in range(batches):
            q.process_batch(*imgs[b % 2])
        out["no_raw_Mpkt_s"] = round(n * batches / (time.perf_counter() - t0) / 1e6, 3)
    for mode_name, mode in (("waveform", D.MODE_WAVEFORM), ("listmode", D.MODE_LISTMODE)):
        for sink in ("file", "null"):
            out[f"{mode_name}_{sink}"] = {"serial": rate(True, n, batches, mode, sink),
                                          "side_stream": rate(False, n, batches, mode, sink)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
