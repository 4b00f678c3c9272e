#!/usr/bin/env python3
"""bench.py -- device-resident DQDK receive path on MI355X.

One "step" = one batch through the whole hot path on the GPU: Eth/IPv4/UDP
parse + IPv4/UDP checksum verify (get_udp_payload + the checksum config,
src/dqdk.c:185-207, src/tcpip/*) + TRISTAN energy-histo decode of every
event into the queue's 2.38 GB histogram (tristan_process /
histogram_event, src/tristan.c:233-330) + the fetch_xsk counters
(src/dqdk.c:252-322).  Frames are resident in HBM before the timed region.

Default run (BASELINE.json metric "..., 1500B & 9000B"): the headline
`value` is 1,048,576 x 1500 B synthetic UDP frames at the UMEM-faithful
4096 B stride, payloadsz 1458 (E = 91), and the same JSON line carries the
north-star's second size under `by_frame_len["9000"]`: 1,048,576 x 9000 B at
stride 9216 (payloadsz 8958, E = 559), measured the same way (its own
kernels, roofline and CPU baseline).  Other BASELINE configs:

  configs[1]  --frames 262144 --no-histo --no-records   parse + checksum only
  configs[2]  --frame-len 9000 --frames 262144           jumbo, full path
  configs[3]  --gpus 4 --frame-len 0                     4 queues, 1500/9000 mix
  configs[4]  --gpus 8 --e2e                             PCIe-inclusive replay,
              pinned H2D / D2H on side streams, paced at --offered-gbps
              (100 Gbit/s over all queues) plus the unpaced maximum

Multi-GPU: one RX queue per GPU, each rank its own frames and histogram, no
collective on the data path; barrier + max-over-ranks
timing; value = all ranks' packets / max time ("scaling": "weak").  Under
torchrun (WORLD_SIZE set) the ranks come from the environment; otherwise
`--gpus N` starts N fresh child ranks itself (before any HIP call here).

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "Mpkt/s & GB/s device-resident UDP/IP parse+TRISTAN decode, 1500B & 9000B"


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 32 = one whole slice pass of 32 staged batches at 1500 B (the steady state of a
    # long capture: one pass per histogram_batches_per_pass() batches)
    p.add_argument("--steps", type=int, default=32)
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
                   help="with --no-histo: pass no record buffer (parse + checksum only, configs[1])")
    p.add_argument("--records", action="store_true",
                   help="histogram mode: also write frame-order decoded records (the unfused path)")
    p.add_argument("--no-9000", action="store_true", help="default run: skip the by_frame_len 9000 B measurement")
    p.add_argument("--no-configs", action="store_true",
                   help="default run: skip the by_config lines (BASELINE configs[1], [2], [3]'s mixed batch)")
    p.add_argument("--rotate", type=int, default=1, help="R copies of the UMEM image, batch k reads copy k %% R")
    p.add_argument("--e2e", action="store_true", help="PCIe-inclusive pipeline (configs[4])")
    p.add_argument("--e2e-frames", type=int, default=1 << 16, help="frames per e2e batch")
    p.add_argument("--offered-gbps", type=float, default=100.0, help="e2e offered load over all queues (Gbit/s)")
    p.add_argument("--cpu-baseline-sec", type=float, default=8.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-box-state", action="store_true", help="skip the sysfs record of clocks / partitions")
    # events inside the timed region (r06h: a torch event per step cost ~4 us a
    # step, HIP events around every decode ~6 us): the decode is bracketed on
    # every --decode-event-every'th batch (its mean launch time, the roofline's
    # denominator, over those launches), one torch event pair spans the region
    p.add_argument("--step-events", type=int, default=0, help=argparse.SUPPRESS)  # 1: a torch event every step
    p.add_argument("--decode-events", type=int, default=1, help=argparse.SUPPRESS)  # 0: decode timed in the breakdown
    p.add_argument("--decode-event-every", type=int, default=4, help=argparse.SUPPRESS)
    p.add_argument("--cpu-dry-run", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--share-gpu", action="store_true",
                   help="rehearsal on fewer GPUs than ranks: rank r uses GPU r %% count, control-plane "
                        "collectives over gloo (the data path has none); the numbers are not a scaling result")
    p.add_argument("--umem-alloc", choices=("torch", "contig"), default="contig",
                   help="device UMEM image: dqdk_gpu_device_alloc (contiguous, default) or torch's allocator")
    p.add_argument("--pmc", default=str(ROOT / "profiles" / "pmc_summary.json"),
                   help="rocprofv3 PMC summary used for roofline.traffic")
    return p.parse_args(argv)


# ---- rank launch -------------------------------------------------------------

def spawn_ranks(n: int) -> int:
    """`--gpus N` without torchrun: N fresh child processes, one per GPU, with
    the torchrun environment (this process never touches HIP).  Returns the
    first non-zero child exit code, else 0."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for o in alive:  # one rank failed: the collective would hang the others
                    o.terminate()
        time.sleep(0.05)
    return rc


# ---- one workload ----------------------------------------------------------------

def umem_size(D, n, L, stride, queue=0):
    import ctypes

    import dqdk_amd._lib as LIB
    c = D.rx.synth_cfg(L, stride, queue)
    return (int(LIB.lib().dqdk_synth_umem_size(ctypes.byref(c), n)) + 15) // 16 * 16


def progress(msg: str) -> None:
    """A liveness line on stderr (the JSON line alone goes to stdout)."""
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)


def synth_to_device(D, torch, dev, n, L, stride, queue, chunk=1 << 16, alloc="torch", image=None):
    """Synthetic UMEM for queue `queue`, generated in chunks straight into HBM
    (host memory stays one chunk); returns (d_umem, d_desc, desc, host sample,
    owner of a library-allocated image or None).  `image`: a DeviceBuffer
    allocated beforehand (main() allocates the images first, while the
    device's memory is unfragmented)."""
    size = umem_size(D, n, L, stride, queue)
    owner = None
    if image is not None:
        assert image.size >= size
        owner = image
        d_umem = image.tensor[:size]
    elif alloc == "contig":  # the library's device allocation (physically contiguous where possible)
        owner = D.DeviceBuffer(dev.index, size)
        d_umem = owner.tensor
    else:
        d_umem = torch.empty(size, dtype=torch.uint8, device=dev)
    descs = []
    sample = None
    for f0 in range(0, n, chunk):
        m = min(chunk, n - f0)
        u, d = D.synth_umem(m, L, stride, queue=queue, first=f0, threads=16)
        d = d.copy()
        d["addr"] += f0 * stride
        d_umem[f0 * stride:f0 * stride + u.size].copy_(torch.from_numpy(u))
        descs.append(d)
        if sample is None:
            sample = (u, d.copy())  # the CPU baseline's sample: the workload's first frames
        if (f0 // chunk) % 4 == 3:
            progress(f"queue {queue}: {f0 + m} of {n} x {L or 'mixed'} B frames generated")
    desc = np.concatenate(descs)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    return d_umem, d_desc, desc, sample, owner


def measure(args, L, torch, dist, dev, rank, world, local, cpu_sec, image=None):
    import ctypes as C

    import dqdk_amd as D
    from dqdk_amd import _lib as LIB

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
    keys_written = histo or not args.no_records
    # histogram mode hands the decode no record buffer (the fused decode buckets
    # its keys itself) unless --records asks for frame-order records as well
    pass_records = (args.records or not histo) and not args.no_records

    # ---- input: queue `rank` of the synthetic UMEM replay, resident in HBM ----
    t_in = time.time()
    d_umem, d_desc, desc, sample, owner = synth_to_device(D, torch, dev, n, L, stride, queue=rank,
                                                          alloc=args.umem_alloc, image=image)
    progress(f"rank {rank}: {n} x {L or 'mixed'} B frames resident ({time.time() - t_in:.1f} s)")
    umem_bytes = d_umem.numel()
    # --rotate R: R copies of the image, batch k reads copy k % R, so a
    # working set the 256 MB MALL could hold is not re-read from it
    # (256K x 1500 B touches 384 MB of frame bytes)
    rot = [D.DeviceBuffer(dev.index, umem_bytes) for _ in range(max(getattr(args, "rotate", 1), 1) - 1)]
    umems = [d_umem.data_ptr()]
    for b in rot:
        b.tensor[:umem_bytes].copy_(d_umem)
        umems.append(b.ptr)
    d_res = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
    d_keys = torch.zeros(max(n * E, 1), dtype=torch.int32, device=dev)
    frame_bytes = int(desc["len"].astype(np.int64).sum())  # per batch (n * L unless mixed)
    Lm = frame_bytes / n  # mean frame length
    q = D.RxQueue(dev.index, cfg, n)  # (the rank's GPU: LOCAL_RANK, or LOCAL_RANK % count when shared)
    stream = torch.cuda.current_stream(dev)
    q.set_stream(stream.cuda_stream)

    nstep = [0]

    def step():
        ptr = umems[nstep[0] % len(umems)]
        nstep[0] += 1
        q.process_device(ptr, umem_bytes, d_desc.data_ptr(), n, d_res.data_ptr(),
                         d_keys.data_ptr() if pass_records else None)

    for _ in range(args.warmup):
        step()
    # the queue's staging placement probe (include/dqdk_gpu.h: its first
    # 3 x DQDK_GPU_PROBE_CANDS fused batches try candidate piece buffers, the
    # next keeps the fastest) belongs to the warmup: extra untimed batches
    # until it has decided
    warm_extra = 0
    while q.staging_probe()["chosen"] == -1 and warm_extra < 32 and n >= 65536 and histo and E and \
            not pass_records:
        step()
        warm_extra += 1
    probe = q.staging_probe()
    progress(f"rank {rank}: {L or 'mixed'} B warm ({args.warmup + warm_extra} batches)")
    q.flush_histogram()  # no warmup batch left staged for the timed region's slice passes
    torch.cuda.synchronize(dev)
    q.read_timing()  # discard
    # only rx_decode is bracketed by HIP events inside the timed region (the
    # roofline kernel), on every `every`-th batch (each event pair is GPU
    # time in the step: r06h); the other kernels are timed in a separate pass
    # below, so the timed steps carry no event packets between their launches
    q.timing_stages(["rx_decode"])
    every = max(args.decode_event_every, 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i in range(args.steps):
        q.enable_timing(bool(args.decode_events) and i % every == 0)  # (a host flag: no GPU work)
        step()
        if args.step_events or i + 1 == args.steps:
            evs[i + 1].record(stream)  # per-step GPU time for the median (no host sync inside)
    # the histogram's slice pass runs once per few staged batches: the pending
    # one runs inside the timed region, so every timed batch is in the table
    q.flush_histogram()
    torch.cuda.synchronize(dev)
    t_rank = time.perf_counter() - t0  # this rank's own time (per-GPU rate)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    q.enable_timing(False)
    stages = q.read_timing()
    elapsed = aggregate_ranks(torch, dist, dev, world, t1 - t0)

    # correctness guard on the measured batch (cheap, outside the timed region)
    cnt = q.counters()
    expect_pkts = n * (args.warmup + warm_extra + args.steps)
    assert cnt["rcvd_pkts"] == expect_pkts, cnt
    res = d_res.cpu().numpy().view(D.RESULT_DTYPE)
    assert (res["status"] == D.RX_OK).all(), np.bincount(res["status"])

    # per-kernel breakdown: an extra pass (outside the timed region) with every
    # launch bracketed; rx_decode keeps its timed-region figure
    bd_steps = min(args.steps, 32)  # the timed region's slice-pass cadence (32 staged batches at 1500 B)
    q.timing_stages(None)
    q.enable_timing(True)
    for _ in range(bd_steps):
        step()
    q.flush_histogram()
    torch.cuda.synchronize(dev)
    q.enable_timing(False)
    for name, s in q.read_timing().items():
        if name != "rx_decode" or not args.decode_events:
            stages[name] = dict(s, batches=bd_steps)
    if args.decode_events:
        stages["rx_decode"]["batches"] = stages["rx_decode"]["launches"]  # the bracketed ones
    hist_k = q.histogram_batches_per_pass()  # partitioned batches per slice pass, at most
    slice_passes = stages.get("rx_slice_histo", {}).get("launches", 0)

    step_ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)) if args.step_events else \
        [evs[0].elapsed_time(evs[args.steps]) / args.steps]
    total_pkts = n * args.steps * world
    mpkts = total_pkts / elapsed / 1e6
    frame_gbs = frame_bytes * args.steps * world / elapsed / 1e9

    # ---- per-kernel algorithmic bytes per launch ------------
    K = n * E  # decoded records per batch
    if histo and E and not pass_records:
        # the frame-order records of this batch, for the statistics below only:
        # a decode-only queue (outside every timed region)
        with D.RxQueue(dev.index, D.RxConfig(payloadsz=payloadsz, mode=mode, flags=flags | D.F_NO_HISTO), n) as qr:
            qr.set_stream(stream.cuda_stream)
            qr.process_device(d_umem.data_ptr(), umem_bytes, d_desc.data_ptr(), n, d_res.data_ptr(),
                              d_keys.data_ptr())
            torch.cuda.synchronize(dev)
    items = K // 18432 + 284 + 1  # part2 work items (18432-key chunks of the 284 buckets, rx_kernels.h kPartChunk)
    runs = items * 129 * 2  # u16 slice-run offsets per item
    touched = 0
    if histo and E:
        # 16K-bin slices with >= 1 event: a scatter of flags in 64M-key chunks
        # (torch.unique's sort of 586M keys at 9000 B ran for minutes with two
        # ranks sharing a GPU, r06m)
        occ = torch.zeros(1 << 16, dtype=torch.uint8, device=dev)
        for c0 in range(0, K, 1 << 26):
            s = d_keys[c0:min(K, c0 + (1 << 26))]
            occ[(s[s >= 0] >> 14).long()] = 1
            del s
        touched = int(occ.sum().item())
        del occ
    alg = {
        # the metric's path: desc + frame (the UDP checksum reads all of it) + result + 4-B record per event
        # (the fused decode writes 8-B key triples, 2.67 B per event, so this over-counts
        # its writes) (no records and no histogram: parse + checksum only, configs[1] -- nothing written)
        "rx_decode": n * (16 + 8) + frame_bytes + (4 * K if keys_written else 0),
        "rx_abort": 8 * n,
        "rx_count": 8 * n,
        "rx_histo_atomic": 8 * n + 4 * K,  # + K random RMWs (priced in Gupd/s below)
        # records path: keys read + bucket runs written; fused path: the overflow list only (~0)
        "rx_part1": 8 * K if pass_records else 0,
        # fused path, a long overflow list grouped by bucket (8 B per listed key; not in the timed workload)
        "rx_fixup": 0,
        # fused path: key triples read (8 B per 3 keys) + u16 keys written; records path: u32 keys read
        "rx_part2": (4 * K if pass_records else K * 8 // 3) + 2 * K + runs,
        # u16 keys + runs read, one read-modify-write of every touched slice's 16 KB of the
        # table's low-byte plane (carries into the u32 base plane: one per 256 increments)
        # (per batch: one slice pass sweeps for up to hist_k staged batches; the timed
        # batches took `slice_passes` passes, the flush inside the timed region included)
        "rx_slice_histo": 2 * K + runs + touched * 2 * (1 << 14) * slice_passes // max(bd_steps, 1),
    }
    st = {}
    for name, s in stages.items():
        if s["launches"]:
            avg_ms = s["ms"] / s["launches"]
            batch_ms = s["ms"] / s["batches"]  # the slice kernels launch once per hist_k batches
            gbs = alg.get(name, 0) / (batch_ms * 1e-3) / 1e9
            st[name] = {"avg_ms": round(avg_ms, 4), "launches": s["launches"], "ms_per_batch": round(batch_ms, 4),
                        "alg_bytes": alg.get(name, 0), "GB_s": round(gbs, 1), "frac_hbm": round(gbs / HBM_PEAK_GBS, 4)}

    # measured bounds on this GPU (membench.hip): streaming read over the UMEM
    # image, random u32 atomics of the same records into a scratch table
    ms = C.c_double()
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
    # the same frames read one wave per frame with 4 B per event written: the
    # pattern's practical rate without arithmetic
    fbytes = (round(Lm) + 15) // 16 * 16  # mixed: every frame read at the mean length
    pattern = {}
    if E:
        LIB.check(LIB.lib().dqdk_gpu_membench_frames(d_umem.data_ptr(), stride, fbytes, n, d_keys.data_ptr(), 4 * E,
                                                     0, stream.cuda_stream, 5, C.byref(ms)), "membench_frames")
        pattern["per_frame"] = round(n * (fbytes + 4 * E) / (ms.value * 1e-3) / 1e9, 1)

    hist_kernels = [k for k in ("rx_histo_atomic", "rx_fixup", "rx_part1", "rx_part2", "rx_slice_histo") if k in st]
    histogram = None
    if hist_kernels:
        h_ms = sum(st[k]["ms_per_batch"] for k in hist_kernels)
        h_bytes = sum(alg[k] for k in hist_kernels if k != "rx_histo_atomic")
        gupd = K / (h_ms * 1e-3) / 1e9
        histogram = {"kernels": hist_kernels, "updates_per_batch": K, "touched_slices": touched,
                     "batches_per_slice_pass": hist_k if "rx_slice_histo" in st else None,
                     "slice_passes": slice_passes,  # over the per-kernel breakdown's batches
                     "ms": round(h_ms, 4), "Gupd_s": round(gupd, 2),
                     # the partitioned chain streams its staging (bytes above) once per batch: its roofline
                     "streamed_bytes": h_bytes, "streamed_GB_s": round(h_bytes / (h_ms * 1e-3) / 1e9, 1),
                     "frac_hbm": round(h_bytes / (h_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "random_atomic_Gupd_s": round(atomic_gupd, 2) if atomic_gupd else None}

    # the fused decode ran: rx_part2 without the records path's rx_part1 (the
    # fused path launches rx_part1, as "rx_fixup", only to group a long overflow list)
    fused = st.get("rx_part2", {}).get("launches", 0) > 0 and not st.get("rx_part1", {}).get("launches", 0)
    traffic = traffic_x2 = None
    traffic_src = None
    try:
        pmc = json.loads(Path(args.pmc).read_text())
        w = pmc.get(f"{L}:{'csum' if not args.no_csum else 'nocsum'}:{n}", {})
        kd = w.get("rx_decode_fused_kernel" if fused else "rx_decode_kernel", {})
        traffic = kd.get("hbm_bytes_per_launch")
        if traffic is not None:
            # reads from the request-size counters when collected (tools/pmc_summary.py),
            # else FETCH_SIZE x 2; the doubled figure kept beside the exact one
            exact = "hbm_read_bytes_by_size" in kd
            traffic_src = ("TCC_EA0_RDREQ_{32B,64B,128B} + WRITE_SIZE" if exact else "FETCH_SIZE x 2 + WRITE_SIZE")
            if exact and "hbm_read_bytes_fetch_x2" in kd:
                traffic_x2 = kd["hbm_read_bytes_fetch_x2"] + kd.get("hbm_write_bytes", 0.0)
    except Exception:
        pass
    dec = st.get("rx_decode", {})
    roofline = {"bound": "hbm", "kernel": "rx_decode_fused" if fused else "rx_decode",
                "achieved": dec.get("GB_s"), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": dec.get("frac_hbm"), "traffic": traffic, "traffic_counters": traffic_src,
                "traffic_fetch_x2": traffic_x2,
                "alg_bytes_per_frame": round(16 + Lm + 8 + (4 * E if keys_written else 0), 1),
                "frames_per_launch": n,
                # the decode launches bracketed by HIP events inside the timed region (of args.steps)
                "timed_launches": dec.get("launches"), "timed_region_launches": args.steps,
                "measured_stream_read_GB_s": round(stream_gbs, 1),
                "frac_of_measured_stream": round(dec["GB_s"] / stream_gbs, 4) if dec else None,
                "measured_frames_pattern_GB_s": pattern,
                "umem_image": {"alloc": args.umem_alloc,
                               "contiguous": bool(owner.contiguous) if owner is not None else False,
                               "va": hex(d_umem.data_ptr()),
                               "va_mod_2MiB": d_umem.data_ptr() % (2 << 20), "bytes": umem_bytes,
                               "rotated_copies": len(umems)}}

    # ---- this rank's report, gathered on rank 0 (N > 1) ----
    report = {"rank": rank, "Mpkt_s": round(n * args.steps / t_rank / 1e6, 3),
              "frame_GB_s": round(frame_bytes * args.steps / t_rank / 1e9, 2),
              "decode_ms": dec.get("avg_ms"), "decode_alg_bytes": alg["rx_decode"],
              "decode_frac": dec.get("frac_hbm"), "decode_kernel": roofline["kernel"],
              "frac_of_measured_stream": roofline["frac_of_measured_stream"],
              "staging_probe": dict(probe, warmup_extra=warm_extra), "bdf": device_bdf(torch, dev.index)}
    per_rank = gather_rank_reports(dist, world, report)

    # ---- CPU baseline: the oracle (C restatement), rank 0, outside the timed region ----
    cpu = None
    if rank == 0 and cpu_sec > 0:
        cpu = cpu_baseline(sample, cfg, histo, cpu_sec, world)
    if world > 1:
        dist.barrier()

    q.close()
    del d_umem, d_desc, d_res, d_keys
    torch.cuda.synchronize(dev)
    for b in rot:
        b.close()
    if owner is not None and image is None:
        owner.close()
    torch.cuda.empty_cache()
    return {
        "value": round(mpkts, 3), "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "config": {"workload": f"{n} x {'mixed 1500/9000' if mixed else L} B UDP frames (stride {stride}) parse+"
                               f"{'' if args.no_csum else 'ip/udp checksum+'}TRISTAN {args.mode} decode"
                               f"{'' if keys_written else ' (no event work: no records, no histogram)'}"
                               f"{'+histogram' if histo else ''}, device-resident",
                   "frames_per_batch": n, "frame_len": "mixed 1500/9000" if mixed else L,
                   "mean_frame_len": round(Lm, 1), "stride": stride, "payloadsz": payloadsz,
                   "events_per_frame": E, "csum": not args.no_csum, "histogram": histo,
                   "decode": "fused (keys bucketed in the decode)" if fused else "records",
                   "parallelism": f"queue-per-gpu x{world}" + (" (shared-GPU rehearsal)" if args.share_gpu else "")},
        "frame_GB_s": round(frame_gbs, 2),
        "per_gpu": per_rank,
        "roofline_all_gpus": aggregate_roofline(per_rank),
        "step_ms_median": round(step_ms[len(step_ms) // 2], 4),
        "step_ms_min": round(step_ms[0], 4),
        "kernels": st,
        "histogram": histogram,
        "roofline": roofline,
        "cpu_baseline": cpu,
        # the staging placement probe: kept candidate piece buffer, each
        # candidate's decode ns per frame, untimed warmup batches it added
        "staging_probe": dict(probe, warmup_extra=warm_extra),
    }


# BASELINE.json configs measured beside the headline, each
# through the same measure() as the headline: its own kernels, roofline
# (SURVEY §8(d) bytes: 16 + L + 8 per frame, + 4 B per event when events are
# decoded) and CPU baseline.  (name, BASELINE config, overrides, frame_len)
BY_CONFIG = [
    # parse + IPv4/UDP checksum only, no event work (no histogram, no records):
    # 1,524 B per frame; 4 rotated image copies (1.5 GB of frame bytes a
    # cycle) so the 384 MB the batch touches is not served from the MALL
    ("parse_csum_256Kx1500", "configs[1]", {"frames": 1 << 18, "no_histo": True, "no_records": True, "rotate": 4},
     1500),
    ("jumbo_256Kx9000", "configs[2]", {"frames": 1 << 18}, 9000),
    ("mixed_1Mx1500_9000", "configs[3] (one queue of its mixed traffic)", {"frames": 1 << 20}, 0),
]


def by_config(args, torch, dist, dev, rank, world, local, cpu_sec):
    out = {}
    for name, which, over, L in BY_CONFIG:
        a2 = argparse.Namespace(**vars(args))
        for k, v in over.items():
            setattr(a2, k, v)
        a2.stride = 0
        a2.payloadsz = 0
        r = measure(a2, L, torch, dist, dev, rank, world, local, min(cpu_sec, 2.0))
        r["baseline_config"] = which
        out[name] = r
    return out


def box_state(torch, dev_index):
    """The GPU box's memory-system state, recorded in the bench line from this
    process (the decode runs in one of two per-box speed states):
    the device's current clock levels (gfx / memory / fabric / SoC), compute
    and memory partition modes, performance level, HBM vendor, VBIOS and
    product identity, PCIe link, and temperatures, read from
    the amdgpu sysfs files of the HIP device's own PCI function (plain
    read-only file reads; no SMI tool is started), or the error that
    prevented it."""
    out = {}
    try:
        pr = torch.cuda.get_device_properties(dev_index)
        bdf = "%04x:%02x:%02x.0" % (getattr(pr, "pci_domain_id", 0), pr.pci_bus_id, pr.pci_device_id)
        base = Path("/sys/bus/pci/devices") / bdf
        out["bdf"] = bdf

        def rd(name, n=600):
            try:
                return (base / name).read_text()[:n].strip()
            except OSError as e:
                return f"<{e.strerror}>"

        def current(text):  # the pp_dpm_* level marked with '*'
            return next((l.split(":", 1)[1].strip().rstrip("*").strip() for l in text.splitlines()
                         if l.endswith("*")), text)

        for clk in ("sclk", "mclk", "fclk", "socclk"):
            t = rd(f"pp_dpm_{clk}")
            out[f"{clk}_current"] = current(t)
            out[f"{clk}_levels"] = t.replace("\n", "; ")
        # (the HBM vendor and firmware identity: candidates for what tells the
        # speed states apart, which the clocks and partitions do not)
        for f in ("current_compute_partition", "current_memory_partition", "power_dpm_force_performance_level",
                  "mem_info_vram_total", "mem_info_vram_used", "mem_info_vram_vendor", "vbios_version",
                  "product_name", "current_link_speed", "current_link_width"):
            out[f] = rd(f, 200)
        temps = {}
        for hw in sorted((base / "hwmon").glob("hwmon*")):
            for t in sorted(hw.glob("temp*_input")):
                lab = t.with_name(t.name.replace("_input", "_label"))
                try:
                    temps[lab.read_text().strip() if lab.exists() else t.name] = int(t.read_text()) / 1000
                except (OSError, ValueError):
                    pass
        out["temps_C"] = temps
    except Exception as e:  # recorded, not fatal: the measurement itself stands
        out["error"] = f"{type(e).__name__}: {e}"[:400]
    return out


def aggregate_ranks(torch, dist, dev, world, elapsed):
    """Job time = max over ranks of the barrier-bracketed time."""
    if world == 1:
        return elapsed
    if dist.get_backend() == "gloo":
        dev = torch.device("cpu")
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_rank_reports(dist, world, report):
    """Every rank's own report (rank 0 gets the list; None at N = 1): its
    packets and frame bytes over its own time, its roofline kernel's time,
    algorithmic bytes and fraction, its staging-probe choice and candidate
    times, its GPU's PCI id -- so a slow rank in an N-GPU line is visible
    (the reference runs one worker per queue,
    src/dqdk.c:517-620)."""
    if world == 1:
        return None
    out = [None] * world
    dist.all_gather_object(out, report)
    return out


def aggregate_roofline(reports, peak=HBM_PEAK_GBS):
    """The N-GPU roofline: every rank's roofline-kernel algorithmic bytes per
    launch, summed, over the slowest rank's launch time, against N x peak."""
    if not reports or any(r.get("decode_ms") in (None, 0) for r in reports):
        return None
    n = len(reports)
    alg = sum(r["decode_alg_bytes"] for r in reports)
    t = max(r["decode_ms"] for r in reports) * 1e-3
    gbs = alg / t / 1e9
    fr = [r["decode_frac"] for r in reports]
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": peak * n, "unit": "GB/s",
            "frac": round(gbs / (peak * n), 4), "per_rank_frac": fr, "min_rank_frac": min(fr),
            "slowest_rank": max(range(n), key=lambda k: reports[k]["decode_ms"])}


def device_bdf(torch, dev_index):
    try:
        pr = torch.cuda.get_device_properties(dev_index)
        return "%04x:%02x:%02x.0" % (getattr(pr, "pci_domain_id", 0), pr.pci_bus_id, pr.pci_device_id)
    except Exception as e:  # noqa: BLE001
        return f"<{type(e).__name__}>"


def dry_run(args, torch, dist, dev, rank, world):
    """--cpu-dry-run: the launch / barrier / max-over-ranks / line path with
    gloo on CPU and no GPU work (each rank sleeps a rank-dependent time per
    step); exercised by tests/test_bench_launch.py."""
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.02 * (1 + rank))
    t_rank = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = aggregate_ranks(torch, dist, dev, world, time.perf_counter() - t0)
    # the same report a GPU rank gives, from the sleep: "decode" = one step
    dec_ms = t_rank / args.steps * 1e3
    alg = args.frames * (16 + 1500 + 8 + 4 * 91)
    rep = {"rank": rank, "Mpkt_s": round(args.frames * args.steps / t_rank / 1e6, 3),
           "frame_GB_s": round(args.frames * 1500 * args.steps / t_rank / 1e9, 2),
           "decode_ms": round(dec_ms, 4), "decode_alg_bytes": alg,
           "decode_frac": round(alg / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
           "staging_probe": {"chosen": -1, "ns_per_frame": []}, "bdf": "dry-run"}
    reports = gather_rank_reports(dist, world, rep)
    return {"value": round(args.frames * args.steps * world / elapsed / 1e6, 3),
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "per_gpu": reports,
            "roofline_all_gpus": aggregate_roofline(reports),
            "config": {"workload": "dry run (no GPU work)", "parallelism": f"queue-per-gpu x{world}"}}


def cpu_baseline(sample, cfg, histo, budget_sec, world):
    """Oracle (C restatement of src/tcpip + get_udp_payload + tristan_process)
    on the host cores: the reference's one worker pthread per queue sharing one
    table through relaxed atomics (src/dqdk.c:517-620, src/tristan.c:243).
    Bounded sample: the workload's first 65,536 frames (host copy), 1 thread
    repeated for ~budget_sec, then 2/4/8 threads splitting the same frames."""
    from oracle import oracle as O
    umem, desc = sample
    hist = np.zeros(O.HISTO_ENTRIES, dtype=np.uint32) if histo else None
    if hist is not None:
        hist[:] = 0  # pre-fault the 2.38 GB table (the reference uses hugepages, tristan.c:136-139)

    def rate(threads, sec):
        passes, t = 0, 0.0
        while t < sec and passes < 1000:
            s, _ = O.rx_batch_threads(umem, desc, cfg.payloadsz, cfg.mode, cfg.flags, hist, threads=threads)
            t += s
            passes += 1
        return len(desc) * passes / t / 1e6, passes, t

    r1, passes, sec = rate(1, budget_sec)
    threads = {"1": round(r1, 4)}
    for t in (2, 4, 8):
        threads[str(t)] = round(rate(t, min(2.0, budget_sec))[0], 4)
    model = ""
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        pass
    # one worker thread per queue: the N-queue comparison is N threads
    t_match = str(min(world, 8)) if str(min(world, 8)) in threads else "1"
    l3 = ""
    try:
        l3 = Path("/sys/devices/system/cpu/cpu0/cache/index3/size").read_text().strip()
    except OSError:
        pass
    fbytes = int(desc["len"].astype(np.int64).sum())
    return {"value": threads[t_match], "unit": "Mpkt/s", "cores": int(t_match), "kind": "port",
            "sample": f"first {len(desc)} frames of the workload ({fbytes / 1e6:.0f} MB of frame bytes in a "
                      f"{umem.nbytes / 1e6:.0f} MB UMEM copy), re-read every pass: 1 thread x {passes} passes "
                      f"({sec:.1f} s); 2/4/8 threads split the same frames, so the 8-thread figure reads a "
                      f"sample that can stay resident in the host's caches (L3 {l3 or '?'} per CCD, several "
                      f"CCDs) across passes -- an upper bound for the CPU, not an HBM-sized stream; histogram "
                      f"{'on (2.38 GB table, random updates: not cache-resident)' if histo else 'off'}; "
                      f"host {model}, nproc {os.cpu_count()}",
            "sample_frames": len(desc), "sample_frame_bytes": fbytes, "host_l3": l3,
            "threads_Mpkt_s": threads}


# ---- PCIe-inclusive replay (configs[4]) --------------------------------------------

def run_e2e(args, torch, dist, dev, rank, world, local):
    import dqdk_amd as D
    from dqdk_amd.pipeline import E2EPipeline

    L = args.frame_len
    stride = args.stride or (4096 if 0 < L <= 4096 else 9216)
    payloadsz = args.payloadsz or (1458 if L == 0 else L - 42)
    cfg = D.RxConfig(payloadsz=payloadsz, mode=D.MODES[args.mode], flags=0 if args.no_csum else D.F_CSUM)
    n = args.e2e_frames
    pl = E2EPipeline(dev.index, cfg, n, L, stride, queue=rank, depth=3, images=2)

    def check(b, res, _):
        assert (res["status"] == D.RX_OK).all(), np.bincount(res["status"])

    pl.run(3, on_result=check)  # warm-up (clean frames: every result OK)
    out = {}
    for name, rate in (("unpaced", None), ("paced", args.offered_gbps * 1e9 / 8 / world)):
        if world > 1:
            dist.barrier()
        r = pl.run(args.steps, rate)
        cdev = torch.device("cpu") if world > 1 and dist.get_backend() == "gloo" else dev
        t = torch.tensor([r["sec"], r["Mpkt_s"], r["batch_latency_ms"]["p99"]], dtype=torch.float64, device=cdev)
        if world > 1:
            allr = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(allr, t)
        else:
            allr = [t]
        sec = max(float(a[0]) for a in allr)
        out[name] = {"Mpkt_s": round(r["packets"] * world / sec / 1e6, 3),
                     "frame_GB_s": round(pl.frame_bytes * args.steps * world / sec / 1e9, 2),
                     "per_gpu_Mpkt_s": [round(float(a[1]), 3) for a in allr],
                     "pcie_h2d_GB_s_per_gpu": round(r["pcie_h2d_GB_s"], 2),
                     "pcie_d2h_GB_s_per_gpu": round(r["pcie_d2h_GB_s"], 3),
                     "batch_latency_ms_p99_max": round(max(float(a[2]) for a in allr), 3),
                     "batch_latency_ms_rank0": {k: round(v, 3) for k, v in r["batch_latency_ms"].items()}}
        if rate:
            out[name]["offered_Gbit_s"] = args.offered_gbps
            out[name]["offered_Mpkt_s"] = round(args.offered_gbps * 1e9 / 8 / (pl.frame_bytes / n) / 1e6, 3)
    pl.close()
    return {
        "value": out["unpaced"]["Mpkt_s"], "ms_per_step": round(out["unpaced"]["frame_GB_s"] and
                                                                (pl.frame_bytes * world / (out["unpaced"]["frame_GB_s"] * 1e9)) * 1e3, 4),
        "config": {"workload": f"{world} queue(s) x {n} x {L or 'mixed 1500/9000'} B frames per batch, end-to-end: "
                               "pinned host UMEM -> H2D (side stream) -> parse+checksum+decode+histogram -> D2H "
                               "results (side stream), PCIe-inclusive", "frames_per_batch": n, "frame_len": L,
                   "stride": stride, "payloadsz": payloadsz, "parallelism": f"queue-per-gpu x{world}"},
        "e2e": out,
    }


def main():
    args = parse_args()
    if os.environ.get("DQDK_BENCH_WATCHDOG"):  # (diagnostics: every rank's stack on stderr every N s)
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["DQDK_BENCH_WATCHDOG"]), repeat=True)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))  # before any HIP call in this process
    world = int(env_world or 1)
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    if args.cpu_dry_run:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    elif args.share_gpu:
        dev = torch.device("cuda", local % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if world > 1:
            dist.init_process_group("gloo")  # RCCL refuses two ranks on one GPU
    else:
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        if world > 1:
            dist.init_process_group("nccl", device_id=dev)
    if world > 1:
        if dist.get_world_size() != args.gpus:
            print(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}", file=sys.stderr)
            sys.exit(2)

    cpu_sec = 0.0 if args.no_cpu_baseline else args.cpu_baseline_sec
    extra = {}
    images = {}
    if args.cpu_dry_run:
        r = dry_run(args, torch, dist, dev, rank, world)
    elif args.e2e:
        r = run_e2e(args, torch, dist, dev, rank, world, local)
    else:
        both = args.frame_len == 1500 and not args.no_9000 and not args.stride and not args.payloadsz
        if args.umem_alloc == "contig":
            # the UMEM images first, while the device's memory is unfragmented
            # (a contiguous image is what keeps the decode's address
            # translation in large fragments: DESIGN.md)
            import dqdk_amd as D
            for L in ([args.frame_len, 9000] if both else [args.frame_len]):
                stride = args.stride or (4096 if 0 < L <= 4096 else 9216)
                images[L] = D.DeviceBuffer(dev.index, umem_size(D, args.frames, L, stride, rank))
        r = measure(args, args.frame_len, torch, dist, dev, rank, world, local, cpu_sec, images.get(args.frame_len))
        if both:
            r9 = measure(args, 9000, torch, dist, dev, rank, world, local, cpu_sec / 2, images.get(9000))
            extra = {"by_frame_len": {"1500": {"value": r["value"], "frame_GB_s": r["frame_GB_s"],
                                               "ms_per_step": r["ms_per_step"]},
                                      "9000": r9}}
            if not args.no_configs:
                extra["by_config"] = by_config(args, torch, dist, dev, rank, world, local, cpu_sec)

    for im in images.values():
        torch.cuda.synchronize(dev)
        im.close()
    if rank == 0 and not args.cpu_dry_run and not args.no_box_state:
        extra["box_state"] = box_state(torch, dev.index)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": r["value"],
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": r["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded splitmix64 TRISTAN-over-UDP frames, SURVEY §8(d))",
        }
        line.update({k: v for k, v in r.items() if k not in ("value", "ms_per_step")})
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
