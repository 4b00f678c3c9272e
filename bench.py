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
`--frame-len 9000 --stride 9216` gives the jumbo-frame config (configs[2]);
`--frames 262144 --no-histo --no-records` is configs[1]'s parse + checksum
only; `--frame-len 0` the mixed config (configs[3]): each frame 1500 or 9000 B by a
seeded coin flip (synth.c), stride 9216, payloadsz 1458 (the reference's E
comes from the configured payload size, not the frame, tristan.c:311).

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
    p.add_argument("--frame-len", type=int, default=1500, help="0 = mixed 1500/9000 B (configs[3])")
    p.add_argument("--stride", type=int, default=0, help="UMEM slot bytes (default 4096, or 9216 for > 4096 B)")
    p.add_argument("--payloadsz", type=int, default=0, help="-s; default frame_len - 42")
    p.add_argument("--mode", default="energy-histo")
    p.add_argument("--no-csum", action="store_true", help="shipped path: checksum audit commented out")
    p.add_argument("--no-histo", action="store_true", help="decode only (no histogram accumulation)")
    p.add_argument("--histo-eager", action="store_true", help="slice pass after every batch (no staging)")
    p.add_argument("--no-records", action="store_true",
                   help="diagnostic: with --no-histo, pass no record buffer (decode writes nothing)")
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
    mixed = L == 0
    stride = args.stride or (4096 if 0 < L <= 4096 else 9216)
    payloadsz = args.payloadsz or (1458 if mixed else max(L - 42, 0))
    n = args.frames
    flags = (0 if args.no_csum else D.F_CSUM) | (D.F_NO_HISTO if args.no_histo else 0) | \
        (D.F_HISTO_EAGER if args.histo_eager else 0)
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
    frame_bytes = int(desc["len"].astype(np.int64).sum())  # per batch (n * L unless mixed)
    Lm = frame_bytes / n  # mean frame length
    q = D.RxQueue(local, cfg, n)
    stream = torch.cuda.current_stream(dev)
    q.set_stream(stream.cuda_stream)

    def step():
        q.process_device(d_umem.data_ptr(), umem_bytes, d_desc.data_ptr(), n, d_res.data_ptr(),
                         None if args.no_records else d_keys.data_ptr())

    for _ in range(args.warmup):
        step()
    q.flush_histogram()  # no warmup batch left staged for the timed region's slice passes
    torch.cuda.synchronize(dev)
    q.read_timing()  # discard
    # only rx_decode is bracketed by HIP events inside the timed region (the
    # roofline kernel); the other kernels are timed in a separate pass below,
    # so the timed steps carry no event packets between the other launches
    q.timing_stages(["rx_decode"])
    q.enable_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i in range(args.steps):
        step()
        evs[i + 1].record(stream)  # per-step GPU time for the median (no host sync inside)
    # the histogram's slice pass runs once per few staged batches: the pending
    # one runs inside the timed region, so every timed batch is in the table
    q.flush_histogram()
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

    # per-kernel breakdown: an extra pass (outside the timed region) with every
    # launch bracketed; rx_decode keeps its timed-region figure
    bd_steps = min(args.steps, 10)
    q.timing_stages(None)
    q.enable_timing(True)
    for _ in range(bd_steps):
        step()
    q.flush_histogram()
    torch.cuda.synchronize(dev)
    q.enable_timing(False)
    for name, s in q.read_timing().items():
        if name != "rx_decode":
            stages[name] = dict(s, batches=bd_steps)
    stages["rx_decode"]["batches"] = args.steps
    hist_k = q.histogram_batches_per_pass()  # partitioned batches per slice pass

    step_ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
    step_median_ms = step_ms[len(step_ms) // 2]
    total_pkts = n * args.steps * world
    mpkts = total_pkts / elapsed / 1e6
    frame_gbs = total_pkts * Lm / elapsed / 1e9

    # ---- per-kernel algorithmic bytes per launch ------------
    K = n * E  # decoded records per batch
    keys_written = histo or not args.no_records
    items = K // (1 << 14) + 284 + 1  # part2 work items (16K-key chunks of the 284 buckets)
    runs = items * 129 * 2  # u16 slice-run offsets per item
    touched = 0
    if histo and E:
        kk = d_keys[:K]
        touched = int(torch.unique(kk[kk >= 0] >> 14).numel())  # 16K-bin slices with >= 1 event
    alg = {
        # the metric's path: desc + frame (the UDP checksum reads all of it) + result + 4-B record per event
        # (no records and no histogram: parse + checksum only, configs[1] -- nothing written per event)
        "rx_decode": n * (16 + 8) + frame_bytes + (4 * K if keys_written else 0),
        "rx_abort": 8 * n,
        "rx_count": 8 * n,
        "rx_histo_atomic": 8 * n + 4 * K,  # + K random RMWs (priced in Gupd/s below)
        "rx_part1": 8 * K,  # keys read + bucket runs written (+ two 1.1 KB count rows per unit)
        # count scan: the decode's per-tile bucket-count rows prefixed in place, group rows summed twice
        "rx_hist_prep": 8 * 288 * (-(-n // 64)) + 12 * 288 * (-(-n // 4096)),
        "rx_part2": 6 * K + runs,
        # u16 keys + runs read, one read-modify-write of every touched slice's 16 KB of the
        # table's low-byte plane (carries into the u32 base plane: one per 256 increments)
        # (per batch: one slice pass sweeps for hist_k staged batches)
        "rx_slice_histo": 2 * K + runs + touched * 2 * (1 << 14) // hist_k,
        "rx_slice_heavy": 0,  # slices redone with u32 bins (none at uniform spectra); bytes counted above
    }
    st = {}
    for name, s in stages.items():
        if s["launches"]:
            avg_ms = s["ms"] / s["launches"]
            batch_ms = s["ms"] / s["batches"]  # the slice kernels launch once per hist_k batches
            gbs = alg[name] / (batch_ms * 1e-3) / 1e9
            st[name] = {"avg_ms": round(avg_ms, 4), "launches": s["launches"], "ms_per_batch": round(batch_ms, 4),
                        "alg_bytes": alg[name], "GB_s": round(gbs, 1), "frac_hbm": round(gbs / HBM_PEAK_GBS, 4)}

    # measured bounds on this GPU (membench.hip): streaming read over the UMEM
    # image, random u32 atomics of the same records into a scratch table
    import ctypes as C

    from dqdk_amd import _lib as LIB
    ms = C.c_double()
    # random-atomic bound of the histogram, on this batch's records (before the
    # pattern benchmarks below reuse the records buffer as their sink)
    atomic_gupd = None
    if histo and E:
        scratch = torch.zeros(D.HISTO_ENTRIES, dtype=torch.int32, device=dev)
        LIB.check(LIB.lib().dqdk_gpu_membench_atomic(scratch.data_ptr(), D.HISTO_ENTRIES, d_keys.data_ptr(), K,
                                                     stream.cuda_stream, 3, C.byref(ms)), "membench_atomic")
        del scratch
        atomic_gupd = K / (ms.value * 1e-3) / 1e9
    LIB.check(LIB.lib().dqdk_gpu_membench_read(d_umem.data_ptr(), umem_bytes // 16 * 16, stream.cuda_stream, 5,
                                               C.byref(ms)), "membench_read")
    stream_gbs = umem_bytes // 16 * 16 / (ms.value * 1e-3) / 1e9
    # the same frames read as rx_decode reads them (one wave per frame) and
    # 4 B per event written: the pattern's practical rate without arithmetic
    fbytes = (round(Lm) + 15) // 16 * 16  # mixed: every frame read at the mean length
    pattern = {}
    for name, flat, out in (("per_frame", 0, True), ("per_frame_read_only", 0, False), ("flat", 1, True),
                            ("flat_read_only", 1, False)):
        LIB.check(LIB.lib().dqdk_gpu_membench_frames(d_umem.data_ptr(), stride, fbytes, n,
                                                     d_keys.data_ptr() if (E and out) else None, 4 * E if out else 0,
                                                     flat, stream.cuda_stream, 5, C.byref(ms)), "membench_frames")
        pattern[name] = round(n * (fbytes + (4 * E if out else 0)) / (ms.value * 1e-3) / 1e9, 1)
    # contiguous 4:1 read:write copy over the same bytes (no frames): records buffer as the sink
    mix_n = min(n, d_keys.numel() * 4 // stride)
    LIB.check(LIB.lib().dqdk_gpu_membench_frames(d_umem.data_ptr(), stride, stride, mix_n, d_keys.data_ptr(), 0, 3,
                                                 stream.cuda_stream, 5, C.byref(ms)), "membench_frames")
    pattern["contiguous_mix_4to1"] = round(mix_n * stride * 1.25 / (ms.value * 1e-3) / 1e9, 1)
    cp_n = min(n, d_keys.numel() * 4 // stride)
    LIB.check(LIB.lib().dqdk_gpu_membench_frames(d_umem.data_ptr(), stride, stride, cp_n, d_keys.data_ptr(), 0, 4,
                                                 stream.cuda_stream, 5, C.byref(ms)), "membench_frames")
    pattern["contiguous_copy_1to1"] = round(cp_n * stride * 2 / (ms.value * 1e-3) / 1e9, 1)
    pattern_gbs = pattern["per_frame"]

    hist_kernels = [k for k in ("rx_histo_atomic", "rx_part1", "rx_hist_prep", "rx_part2", "rx_slice_histo",
                                "rx_slice_heavy") if k in st]
    histogram = None
    if hist_kernels:
        h_ms = sum(st[k]["ms_per_batch"] for k in hist_kernels)
        gupd = K / (h_ms * 1e-3) / 1e9
        histogram = {"kernels": hist_kernels, "updates_per_batch": K, "touched_slices": touched,
                     "batches_per_slice_pass": hist_k if "rx_slice_histo" in st else None,
                     "ms": round(h_ms, 4), "Gupd_s": round(gupd, 2),
                     "bound": {"kind": "random u32 atomic increment, measured on these records "
                                       "(dqdk_gpu_membench_atomic)", "Gupd_s": round(atomic_gupd, 2)},
                     "vs_bound": round(gupd / atomic_gupd, 3)}

    # ---- roofline: rx_decode, the kernel §8(d)'s per-packet bytes price -----
    dom = max(st, key=lambda k: st[k]["avg_ms"]) if st else "rx_decode"
    traffic = None
    try:
        pmc = json.loads(Path(args.pmc).read_text())
        w = pmc.get(f"{L}:{'csum' if not args.no_csum else 'nocsum'}:{n}", {})
        traffic = w.get("rx_decode_kernel", {}).get("hbm_bytes_per_launch")
    except Exception:
        pass
    dec = st.get("rx_decode", {})
    roofline = {"bound": "hbm", "kernel": "rx_decode",
                "achieved": dec.get("GB_s"), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": dec.get("frac_hbm"), "traffic": traffic,
                "alg_bytes_per_frame": round(16 + Lm + 8 + (4 * E if keys_written else 0), 1),
                "frames_per_launch": n,
                "measured_stream_read_GB_s": round(stream_gbs, 1),
                "frac_of_measured_stream": round(dec["GB_s"] / stream_gbs, 4) if dec else None,
                "measured_frames_pattern_GB_s": pattern,
                "frac_of_measured_pattern": round(dec["GB_s"] / pattern_gbs, 4) if dec else None,
                "slowest_kernel": dom}

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
            "config": {"workload": f"{n} x {'mixed 1500/9000' if mixed else L} B UDP frames (stride {stride}) parse+"
                                   f"{'' if args.no_csum else 'ip/udp checksum+'}TRISTAN {args.mode} decode"
                                   f"{'' if keys_written else ' (OOB counts only, no records written)'}"
                                   f"{'+histogram' if histo else ''}, device-resident",
                       "frames_per_batch": n, "frame_len": "mixed 1500/9000" if mixed else L,
                       "mean_frame_len": round(Lm, 1), "stride": stride, "payloadsz": payloadsz,
                       "events_per_frame": E, "csum": not args.no_csum, "histogram": histo,
                       "parallelism": f"queue-per-gpu x{world}"},
            "frame_GB_s": round(frame_gbs, 2),
            "step_ms_median": round(step_median_ms, 4),
            "step_ms_min": round(step_ms[0], 4),
            "kernels": st,
            "kernels_timing": "rx_decode: HIP events on the queue stream over the timed steps (the only kernel "
                              "bracketed there); the others: HIP events over a separate pass of "
                              f"{bd_steps} steps with every launch bracketed; ms_per_batch = kernel time / batches "
                              "(the slice kernels run once per batches_per_slice_pass staged batches)",
            "histogram": histogram,
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
    # one pinned worker per queue is the reference's model (src/dqdk.c:517-620):
    # 2/4/8 workers on 2/4/8 x the sample, sharing the table (relaxed atomics)
    threads = {}
    for t in (2, 4, 8):
        m = min(len(desc), t * sample)
        st, _ = O.rx_batch_threads(umem, desc[:m], cfg.payloadsz, cfg.mode, cfg.flags, hist, threads=t)
        threads[str(t)] = round(m / st / 1e6, 4)
    model = ""
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        pass
    return {"value": round(rate, 4), "unit": "Mpkt/s", "cores": 1, "kind": "port",
            "sample": f"first {sample} frames of the workload x {passes} passes ({sec:.1f} s), "
                      f"1 thread, histogram {'on (2.38 GB table)' if histo else 'off'}; "
                      f"host {model}, nproc {_os.cpu_count()}",
            "threads_Mpkt_s": threads}


if __name__ == "__main__":
    main()
