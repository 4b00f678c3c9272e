"""The frame-processor plugin (dqdk_gpu_frame_processor, a
dqdk_frame_processor_t: src/dqdk.h:84-85) driven from Python through
dqdk_amd.FrameProcessor, against the reference's recorded F4 batch.

process_frame (src/dqdk.c:231-250) calls the processor for every frame whose
get_udp_payload succeeded with datalen != 0; here the reference's own
verdicts (F4 status/datalen, per-packet accounting) pick those frames, and
each call hands the payload pointer + datalen, alternating over two worker
addresses.  dqdk_gpu_fp_fini's totals and host table must equal the
reference's tristan_t after the same calls (F4 csum0_abort0: total_events,
total_bytes, the rejected-event count, the sparse histogram)."""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

import dqdk_amd as D
from test_gpu_parity import _need_gpu

pytestmark = pytest.mark.gpu

GOLD = Path(__file__).resolve().parent / "golden"


@pytest.mark.parametrize("slot", [0, 17])
def test_plugin_calls_equal_reference_tristan_totals_and_table(slot):
    _need_gpu()
    z = np.load(GOLD / "f4_batch.npz")
    mode, psz = (int(x) for x in z["cfg"])
    umem = np.zeros(z["umem"].size + (1 << 16), np.uint8)  # the UMEM, then zeros (reads past its end)
    umem[: z["umem"].size] = z["umem"]
    desc, status, datalen = z["desc"], z["status_csum0"], z["datalen_csum0"]
    want = dict(zip((str(n) for n in z["counter_names"]), (int(x) for x in z["csum0_abort0_counters"])))
    fp = D.FrameProcessor(D.RxConfig(payloadsz=psz, mode=mode), slot_payloads=slot)
    workers = [C.create_string_buffer(64) for _ in range(2)]  # two dqdk_worker addresses
    try:
        fp.bind(C.addressof(workers[0]), 0, umem)
        base = umem.ctypes.data
        calls = 0
        for i in range(len(desc)):
            if status[i] != D.RX_OK:  # invalid or datalen == 0: process_frame returns -ENOBUFS first
                continue
            off = 14 + 4 * (int(umem[int(desc["addr"][i]) + 14]) & 0xF) + 8  # get_udp_payload's payload
            rc = fp(C.addressof(workers[calls & 1]), base + int(desc["addr"][i]) + off, int(datalen[i]))
            assert rc == 0  # tristan_process's result (src/tristan.c:329)
            calls += 1
        host = np.zeros(D.HISTO_ENTRIES, np.uint32)
        tot = fp.fini(host)
    finally:
        del fp
    assert tot["rcvd_pkts"] == calls
    assert tot["total_events"] == want["total_events"]
    assert tot["total_bytes"] == want["total_bytes"]  # u32-wrapped datalens included
    assert tot["oob_events"] == want["oob_events"]
    idx, cnt = z["csum0_abort0_hist_idx"], z["csum0_abort0_hist_cnt"]
    nz = np.flatnonzero(host)
    np.testing.assert_array_equal(nz.astype(np.uint32), idx)
    np.testing.assert_array_equal(host[nz], cnt)


@pytest.mark.parametrize("peer", ["0", "1"], ids=["same-device", "peer-branch"])
def test_plugin_fini_merges_workers_into_the_csv(peer, tmp_path, monkeypatch):
    """fp_fini's CSV merge of three workers' tables into the first's (the
    histogram file of tristan_fini, src/tristan.c:197-216), both merge
    branches: a worker on w0's GPU copied device-locally, or (test hook
    DQDK_GPU_FP_PEER_MERGE=1) the cross-device branch -- the table copied on
    the worker's GPU, hipMemcpyPeer into w0's buffer, added -- which a
    one-GPU box can only reach this way (a peer copy within one device is
    legal).  The CSV equals the reference's file for F4's calls."""
    _need_gpu()
    import os

    from test_gpu_egress import ref_csv
    monkeypatch.setenv("DQDK_GPU_FP_PEER_MERGE", peer)
    z = np.load(GOLD / "f4_batch.npz")
    mode, psz = (int(x) for x in z["cfg"])
    umem = np.zeros(z["umem"].size + (1 << 16), np.uint8)
    umem[: z["umem"].size] = z["umem"]
    desc, status, datalen = z["desc"], z["status_csum0"], z["datalen_csum0"]
    fp = D.FrameProcessor(D.RxConfig(payloadsz=psz, mode=mode), slot_payloads=64)
    workers = [C.create_string_buffer(64) for _ in range(3)]
    path = tmp_path / "histo.csv"
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        for w in workers:
            fp.bind(C.addressof(w), 0, umem)
        base = umem.ctypes.data
        calls = 0
        for i in range(len(desc)):
            if status[i] != D.RX_OK:
                continue
            off = 14 + 4 * (int(umem[int(desc["addr"][i]) + 14]) & 0xF) + 8
            assert fp(C.addressof(workers[calls % 3]), base + int(desc["addr"][i]) + off, int(datalen[i])) == 0
            calls += 1
        tot = fp.fini(None, fd)
    finally:
        os.close(fd)
        del fp
    assert tot["rcvd_pkts"] == calls
    assert path.read_text() == ref_csv(z["csum0_abort0_hist_idx"], z["csum0_abort0_hist_cnt"])
