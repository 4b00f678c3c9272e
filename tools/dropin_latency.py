"""Per-call latency and rate of the two drop-in forms at DQDK's batch sizes.

Runs build/fetch_xsk_harness (tests/c/) over synthetic frames in mlock'ed host
UMEM (one per worker, as src/dqdk.c:562 allocates them), for
  proc = batch  INTEGRATION.md's fetch_xsk patch (dqdk_gpu_rx_batch, UMEM
                registered once: the GPU reads the frames over PCIe)
  proc = fp     the unpatched fetch_xsk / process_frame / get_udp_payload with
                dqdk_gpu_frame_processor registered as the worker's
                dqdk_frame_processor_t (src/tristan.c:589-590)
at -b 64 (the default, src/tristan.c:393) and 2048 (production,
tristan-daq.sh:12), with 1 and 3 workers (Q=3, tristan-daq.sh:14), at
1500 B frames (payloadsz 1458) and the production 3434 B frames
(-s 3392, tristan-daq.sh:84).  The need it is compared with: 3.55 Mpkt/s
over Q=3 (tristan-simple.sh:76), i.e. 1.18 Mpkt/s per queue.

One JSON line per configuration to stdout (and --out): wall-clock Mpkt/s of
the receive loop (all workers), the same including the drain at fini (the
plugin decodes asynchronously), and the p50 / p99 / max duration of one
fetch_xsk call.
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HARNESS = ROOT / "build" / "fetch_xsk_harness"
NEED_PER_QUEUE = 3.55e6 / 3


def run(proc: str, batch: int, workers: int, flen: int, psz: int, frames: int, nimg: int, slot: int,
        timeout: int) -> dict:
    repeat = max(1, frames // nimg)
    ring = 4096 if batch <= 2048 else 2 * batch
    cmd = [str(HARNESS), f"synth:{nimg}:{flen}:4096", "-", str(batch), str(ring), "0", str(repeat), str(psz), "3",
           "0", "-", proc, str(workers), str(slot)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    if p.returncode != 0:
        raise RuntimeError(f"{cmd}: rc {p.returncode}: {p.stderr[-2000:]}")
    out = {k: int(v) for k, v in (l.split() for l in p.stdout.splitlines() if l.strip())}
    loop_s = out["loop_ns"] / 1e9
    done_s = (out["loop_ns"] + out["fini_ns"]) / 1e9
    return {
        "proc": proc, "batch": batch, "workers": workers, "umems": out["umem_count"], "frame_len": flen, "payloadsz": psz,
        "slot_payloads": slot if proc == "fp" else None,
        "frames": out["rcvd_frames"], "events": out["total_events"],
        "mpkts_loop": out["rcvd_frames"] / loop_s / 1e6,
        "mpkts_incl_drain": out["rcvd_frames"] / done_s / 1e6,
        "mpkts_per_worker": out["rcvd_frames"] / loop_s / 1e6 / workers,
        "need_per_queue_mpkts": NEED_PER_QUEUE / 1e6,
        "fetch_p50_us": out["fetch_p50_ns"] / 1e3, "fetch_p99_us": out["fetch_p99_ns"] / 1e3,
        "fetch_max_us": out["fetch_max_ns"] / 1e3,
        "per_frame_us": loop_s * workers / out["rcvd_frames"] * 1e6,
        "drain_ms": out["fini_ns"] / 1e6,
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    rows = []
    sizes = [(1500, 1458), (3434, 3392)]
    for flen, psz in sizes:
        for proc in ("fp", "batch"):
            for batch in (64, 2048):
                for workers in (1, 3):
                    if args.quick and (workers == 3 or flen == 3434):
                        continue
                    # enough frames for ~1 s of the slower forms
                    frames = (1 << 21) if proc == "fp" or batch == 2048 else (1 << 18)
                    r = run(proc, batch, workers, flen, psz, frames, 65536, 8192, 300)
                    rows.append(r)
                    line = json.dumps(r)
                    print(line, flush=True)
    if args.out:
        Path(args.out).write_text("".join(json.dumps(r) + "\n" for r in rows))
    return 0


if __name__ == "__main__":
    sys.exit(main())
