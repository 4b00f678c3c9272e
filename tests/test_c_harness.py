"""The C boundary exercised from C: build/fetch_xsk_harness (tests/c/) includes
include/dqdk_gpu.h, links libdqdk_gpu.so and drives it over an mmap'd +
mlock'd UMEM (hugetlb when the host has it) with a wrapping RX descriptor ring
and fill-ring reuse (src/dqdk.c:109-127, :252-322), two ways:

proc=batch, INTEGRATION.md's fetch_xsk patch (dqdk_gpu_rx_batch):
  * one batch = F4's 1,024 frames, wrapping the ring end: the worker stats and
    GPU counters equal the reference's recorded F4 counters and the CSV equals
    the reference's table (tests/golden/gen_tristan.py);
  * 31 batches of 100 over the stream repeated three times (batch abort on):
    equal to the oracle (pinned to F4) applied batch by batch;
  * three workers over a UMEM each (the reference's layout) or one shared
    UMEM: three times the oracle's counters, every teardown clean.

proc=fp, the reference's plugin API: fetch_xsk / process_frame /
get_udp_payload unpatched, dqdk_gpu_frame_processor registered as the
worker's dqdk_frame_processor_t like src/tristan.c:589-590 registers
process_unbuffered_frame, dqdk_gpu_fp_fini feeding tristan_fini:
  * F4 in one batch: the worker stats, tristan_t's totals, the host table and
    the GPU CSV equal the reference's recorded batch-abort run (the
    reference's loop aborts on its first -ENOBUFS);
  * many batches, small staging slots (every slot size, partial last slot),
    atomic and partitioned histograms, one and three workers: equal to the
    oracle per batch (times the workers).
"""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import dqdk_amd as D
from oracle import oracle as O
from test_gpu_egress import ref_csv
from test_gpu_parity import _need_gpu

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
HARNESS = ROOT / "build" / "fetch_xsk_harness"
GOLD = Path(__file__).resolve().parent / "golden"
STATS = ["rcvd_frames", "rcvd_pkts", "rcvd_bytes", "invalid_ip_pkts", "invalid_udp_pkts", "failing_batches",
         "total_events", "total_bytes", "oob_events", "empty_pkts"]


def run_harness(tmp_path, umem, desc, batch, ring, start, repeat, psz, mode, flags, proc="batch", workers=1,
                slot=0, want_csv=True, env=None):
    _need_gpu()
    assert HARNESS.exists(), "build/fetch_xsk_harness not built (python -m dqdk_amd._build)"
    (tmp_path / "umem.bin").write_bytes(np.ascontiguousarray(umem).tobytes())
    (tmp_path / "desc.bin").write_bytes(np.ascontiguousarray(desc).tobytes())
    csv = tmp_path / "histo.csv"
    p = subprocess.run([str(HARNESS), str(tmp_path / "umem.bin"), str(tmp_path / "desc.bin"), str(batch), str(ring),
                        str(start), str(repeat), str(psz), str(mode), str(flags), str(csv) if want_csv else "-", proc,
                        str(workers), str(slot)],
                       capture_output=True, text=True, timeout=120, env=dict(os.environ, **(env or {})))
    assert p.returncode == 0, p.stderr  # (teardown included: every queue's unregister and destroy)
    out = dict(l.split() for l in p.stdout.splitlines() if l.strip())
    return {k: int(v) for k, v in out.items()}, csv.read_text() if want_csv else None


@pytest.mark.parametrize("csum", [0, 1])
@pytest.mark.parametrize("abort", [0, 1])
def test_single_wrapping_batch_equals_reference_f4(tmp_path, csum, abort):
    z = np.load(GOLD / "f4_batch.npz")
    mode, psz = (int(x) for x in z["cfg"])
    flags = (D.F_CSUM if csum else 0) | (D.F_BATCH_ABORT if abort else 0)
    got, csv = run_harness(tmp_path, z["umem"], z["desc"], batch=1024, ring=2048, start=1500, repeat=1, psz=psz,
                           mode=mode, flags=flags)
    assert got["wrapped_batches"] == 1 and got["batches"] == 1
    k = f"csum{csum}_abort{abort}_"
    want = dict(zip((str(n) for n in z["counter_names"]), (int(x) for x in z[k + "counters"])))
    for name in STATS:
        want_v = want[name] if not (name == "failing_batches" and not abort) else 0
        assert got[name] == want_v, (name, got[name], want_v)
    assert got["fill_submitted"] == (0 if abort else 1024)  # an aborted batch is not submitted (:317-321)
    assert csv == ref_csv(z[k + "hist_idx"], z[k + "hist_cnt"].astype(np.uint64))


def test_many_batches_over_wrapping_ring(tmp_path):
    z = np.load(GOLD / "f4_batch.npz")
    mode, psz = (int(x) for x in z["cfg"])
    flags = D.F_CSUM | D.F_BATCH_ABORT
    batch, repeat = 100, 3
    got, csv = run_harness(tmp_path, z["umem"], z["desc"], batch=batch, ring=256, start=200, repeat=repeat, psz=psz,
                           mode=mode, flags=flags)
    stream = np.concatenate([z["desc"]] * repeat)
    table = np.zeros(O.HISTO_ENTRIES, np.uint32)
    tot = dict.fromkeys(STATS, 0)
    umem = z["umem"].copy()
    for b0 in range(0, len(stream), batch):
        _, c, _ = O.rx_batch(umem, stream[b0:b0 + batch], psz, mode, flags, want_keys=False, hist=table)
        for k in STATS:
            tot[k] += c[k]
    assert got["batches"] == -(-len(stream) // batch) and got["wrapped_batches"] > 0
    for k in STATS:
        assert got[k] == tot[k], (k, got[k], tot[k])
    nz = np.flatnonzero(table)
    assert got["histo_nonzero"] == len(nz)
    assert csv == ref_csv(nz.astype(np.uint32), table[nz].astype(np.uint64))


@pytest.mark.parametrize("shared", [0, 1])
def test_three_workers_batch_patch_either_umem_layout(tmp_path, shared):
    """Three workers, a queue each, every one running the whole descriptor
    stream: over a UMEM each (as umem_info_create makes one per worker,
    src/dqdk.c:562) or over one shared UMEM (DQDK_HARNESS_SHARED_UMEM=1: the
    library's reference-counted registration, include/dqdk_gpu.h).  Worker
    stats and GPU counters are three times the oracle's, and every queue's
    unregister and destroy succeed."""
    z = np.load(GOLD / "f4_batch.npz")
    mode, psz = (int(x) for x in z["cfg"])
    flags = D.F_CSUM | D.F_BATCH_ABORT
    batch, repeat = 100, 2
    got, _ = run_harness(tmp_path, z["umem"], z["desc"], batch=batch, ring=256, start=200, repeat=repeat, psz=psz,
                         mode=mode, flags=flags, workers=3, want_csv=False,
                         env={"DQDK_HARNESS_SHARED_UMEM": str(shared)})
    assert got["workers"] == 3 and got["umem_count"] == (1 if shared else 3)
    stream = np.concatenate([z["desc"]] * repeat)
    tot = dict.fromkeys(STATS, 0)
    umem = z["umem"].copy()
    for b0 in range(0, len(stream), batch):
        _, c, _ = O.rx_batch(umem, stream[b0:b0 + batch], psz, mode, flags, want_keys=False)
        for k in STATS:
            tot[k] += c[k]
    for k in STATS:
        assert got[k] == 3 * tot[k], (k, got[k], 3 * tot[k])


# ---- the plugin API: dqdk_gpu_frame_processor behind the unpatched loop ----

FP_STATS = [k for k in STATS if k != "empty_pkts"]  # (the processor never sees an empty payload)


def test_frame_processor_f4_equals_reference(tmp_path):
    z = np.load(GOLD / "f4_batch.npz")
    mode, psz = (int(x) for x in z["cfg"])
    got, csv = run_harness(tmp_path, z["umem"], z["desc"], batch=1024, ring=2048, start=1500, repeat=1, psz=psz,
                           mode=mode, flags=0, proc="fp")
    assert got["wrapped_batches"] == 1 and got["batches"] == 1
    # the reference's loop is batch-abort by construction (src/dqdk.c:294-296)
    want = dict(zip((str(n) for n in z["counter_names"]), (int(x) for x in z["csum0_abort1_counters"])))
    for name in FP_STATS:
        assert got[name] == want[name], (name, got[name], want[name])
    assert got["fill_submitted"] == 0
    # one processor call per frame before the abort with datalen != 0
    assert got["fp_calls"] == want["rcvd_pkts"] - want["invalid_ip_pkts"] - want["invalid_udp_pkts"] - 1
    idx, cnt = z["csum0_abort1_hist_idx"], z["csum0_abort1_hist_cnt"]
    assert got["histo_nonzero"] == len(idx)   # tristan_t::histo filled by dqdk_gpu_fp_fini
    assert csv == ref_csv(idx, cnt.astype(np.uint64))  # the merged table's CSV, formatted on the GPU


@pytest.mark.parametrize("workers,slot,hflags", [(1, 7, 0), (1, 100, D.F_HISTO_PARTITIONED), (3, 64, 0),
                                                (3, 4096, D.F_HISTO_PARTITIONED)])
def test_frame_processor_many_batches_vs_oracle(tmp_path, workers, slot, hflags):
    z = np.load(GOLD / "f4_batch.npz")
    mode, psz = (int(x) for x in z["cfg"])
    batch, repeat = 100, 3
    got, csv = run_harness(tmp_path, z["umem"], z["desc"], batch=batch, ring=256, start=200, repeat=repeat, psz=psz,
                           mode=mode, flags=hflags, proc="fp", workers=workers, slot=slot)
    stream = np.concatenate([z["desc"]] * repeat)
    table = np.zeros(O.HISTO_ENTRIES, np.uint32)
    tot = dict.fromkeys(STATS, 0)
    umem = z["umem"].copy()
    for b0 in range(0, len(stream), batch):
        _, c, _ = O.rx_batch(umem, stream[b0:b0 + batch], psz, mode, D.F_BATCH_ABORT, want_keys=False, hist=table)
        for k in STATS:
            tot[k] += c[k]
    assert got["workers"] == workers
    for k in FP_STATS:
        assert got[k] == workers * tot[k], (k, got[k], workers * tot[k])
    table = table * np.uint32(workers)
    nz = np.flatnonzero(table)
    assert got["histo_nonzero"] == len(nz)
    assert csv == ref_csv(nz.astype(np.uint32), table[nz].astype(np.uint64))
