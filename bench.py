#!/usr/bin/env python3
"""bench.py -- device-resident DQDK receive path on MI355X.

One "step" = one batch through the whole hot path on the GPU: Eth/IPv4/UDP
parse + IPv4/UDP checksum verify (get_udp_payload + the checksum config,
src/dqdk.c:185-207, src/tcpip/*) + TRISTAN energy-histo decode of every
event into the queue's 2.38 GB histogram (tristan_process /
histogram_event, src/tristan.c:233-330) + the fetch_xsk counters
(src/dqdk.c:252-322).  Frames are resident in HBM before the timed region.

Default workload (BASELINE.json configs[1] frame size with the metric's full
parse + decode path, north-star batch size): 1,048,576 x 1500 B synthetic
UDP frames at the UMEM-faithful 4096 B stride, payloadsz 1458 (E = 91).
`--frame-len 9000 --stride 9216` gives the jumbo-frame config (configs[2]).

Multi-GPU (`torchrun --nproc-per-node N bench.py --gpus N`): one RX queue per
GPU, each rank its own frames and histogram, no collective in the data path
(SURVEY §8(e)); barrier + max-over-ranks timing; value = all ranks' packets
/ max time ("scaling": "weak").

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--frames", type=int, default=1 << 20)
    p.add_argument("--frame-len", type=int, default=1500)
    p.add_argument("--stride", type=int, default=0, help="UMEM slot bytes (default 4096, or 9216 for > 4096 B)")
    p.add_argument("--payloadsz", type=int, default=0, help="-s; default frame_len - 42")
    p.add_argument("--mode", default="energy-histo")
    p.add_argument("--no-csum", action="store_true", help="shipped path: checksum audit commented out")
    p.add_argument("--no-histo", action="store_true", help="decode only (no histogram accumulation)")
    p.add_argument("--cpu-baseline-sec", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--pmc", default=str(ROOT / "profiles" / "pmc_summary.json"),
                   help="rocprofv3 PMC summary used for roofline.traffic")
    return p.parse_args()


def main():
    args = parse_args()
    import torch
    import torch.distributed as dist

    import dqdk_amd as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    L = args.frame_len
    stride = args.stride or (4096 if L <= 4096 else 9216)
    payloadsz = args.payloadsz or max(L - 42, 0)
    n = args.frames
    flags = (0 if args.no_csum else D.F_CSUM) | (D.F_NO_HISTO if args.no_histo else 0)
    mode = D.MODES[args.mode]
    cfg = D.RxConfig(payloadsz=payloadsz, mode=mode, flags=flags)
    E = cfg.events
    histo = D.histo_enabled(mode, flags)

    # ---- input: queue `rank` of the synthetic UMEM replay, resident in HBM ----
    umem, desc = D.synth_umem(n, L, stride, queue=rank, threads=16)
    d_umem = torch.from_numpy(umem).to(dev)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    d_res = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
    d_keys = torch.zeros(max(n * E, 1), dtype=torch.int32, device=dev)
    umem_bytes = umem.nbytes
    q = D.RxQueue(local, cfg, n)
    stream = torch.cuda.current_stream(dev)
    q.set_stream(stream.cuda_stream)

    def step():
        q.process_device(d_umem.data_ptr(), umem_bytes, d_desc.data_ptr(), n, d_res.data_ptr(), d_keys.data_ptr())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    q.read_timing()  # discard
    q.enable_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    q.enable_timing(False)
    stages = q.read_timing()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # correctness guard on the measured batch (cheap, outside the timed region)
    cnt = q.counters()
    expect_pkts = n * (args.warmup + args.steps)
    assert cnt["rcvd_pkts"] == expect_pkts, cnt
    res = d_res.cpu().numpy().view(D.RESULT_DTYPE)
    assert (res["status"] == D.RX_OK).all(), np.bincount(res["status"])

    total_pkts = n * args.steps * world
    mpkts = total_pkts / elapsed / 1e6
    frame_gbs = total_pkts * L / elapsed / 1e9

    # ---- roofline of the dominant kernel (HIP events on the queue stream) ----
    alg = {
        # per-frame algorithmic bytes: desc + frame + result (+ 4-B record per event)
        "rx_decode": 16 + L + 8 + 4 * E,
        # keys read + one u32 read-modify-write per event, plus the 8-B result read
        "histogram": 8 + 12 * E,
        "counters": 2 * 8,
    }
    st = {}
    for name, s in stages.items():
        if s["launches"]:
            avg_ms = s["ms"] / s["launches"]
            gbs = alg[name] * n / (avg_ms * 1e-3) / 1e9
            st[name] = {"avg_ms": round(avg_ms, 4), "alg_bytes_per_frame": alg[name], "GB_s": round(gbs, 1),
                        "frac_hbm": round(gbs / HBM_PEAK_GBS, 4)}
    if "histogram" in st:
        st["histogram"]["Gupdates_s"] = round(n * E / (st["histogram"]["avg_ms"] * 1e-3) / 1e9, 2)
    dom = max(st, key=lambda k: st[k]["avg_ms"]) if st else "rx_decode"
    traffic = None
    try:
        pmc = json.loads(Path(args.pmc).read_text())
        w = pmc.get(f"{L}:{'csum' if not args.no_csum else 'nocsum'}:{n}", {})
        traffic = w.get(dom, {}).get("hbm_bytes_per_launch")
    except Exception:
        pass
    roofline = {"bound": "hbm", "kernel": dom,
                "achieved": st.get(dom, {}).get("GB_s"), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": st.get(dom, {}).get("frac_hbm"), "traffic": traffic}

    # ---- CPU baseline: the oracle (C restatement) on rank 0 at N=1 ----------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(umem, desc, cfg, histo, args.cpu_baseline_sec)

    if rank == 0:
        line = {
            "metric": "Mpkt/s & GB/s device-resident UDP/IP parse+TRISTAN decode, 1500B & 9000B",
            "value": round(mpkts, 3),
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded splitmix64 TRISTAN-over-UDP frames, SURVEY §8(d))",
            "config": {"workload": f"{n} x {L} B UDP frames (stride {stride}) parse+"
                                   f"{'' if args.no_csum else 'ip/udp checksum+'}TRISTAN {args.mode} decode"
                                   f"{'+histogram' if histo else ''}, device-resident",
                       "frames_per_batch": n, "frame_len": L, "stride": stride, "payloadsz": payloadsz,
                       "events_per_frame": E, "csum": not args.no_csum, "histogram": histo,
                       "parallelism": f"queue-per-gpu x{world}"},
            "frame_GB_s": round(frame_gbs, 2),
            "stages": st,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    q.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(umem, desc, cfg, histo, budget_sec):
    """Oracle (C restatement of src/tcpip + get_udp_payload + tristan_process)
    on one host core: the reference's one worker pthread per queue.  Bounded
    sample: the workload's first 65,536 frames, repeated until ~budget_sec."""
    import os as _os

    from oracle import oracle as O
    sample = min(len(desc), 65536)
    sub = desc[:sample]
    hist = np.zeros(O.HISTO_ENTRIES, dtype=np.uint32) if histo else None
    if hist is not None:
        hist[:] = 0  # pre-fault the 2.38 GB table (the reference uses hugepages, tristan.c:136-139)
    passes, sec = 0, 0.0
    while sec < budget_sec and passes < 1000:
        s, _ = O.rx_batch_threads(umem, sub, cfg.payloadsz, cfg.mode, cfg.flags, hist, threads=1)
        sec += s
        passes += 1
    rate = sample * passes / sec / 1e6
    return {"value": round(rate, 4), "unit": "Mpkt/s", "cores": 1, "kind": "port",
            "sample": f"first {sample} frames of the workload x {passes} passes ({sec:.1f} s), "
                      f"1 thread, histogram {'on (2.38 GB table)' if histo else 'off'}, "
                      f"host {_os.cpu_count()} cpus"}


if __name__ == "__main__":
    main()
