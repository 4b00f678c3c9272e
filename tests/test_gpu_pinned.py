"""HIP path vs the REFERENCE's own outputs (not via the oracle), through the C ABI.

The expected arrays below were recorded from the reference itself
(tests/golden/gen_golden.py: src/tcpip compiled verbatim; gen_tristan.py:
histogram_event / process_events_unrolled16 / tristan_process extracted
verbatim from src/tristan.{c,h}):

  F1  get_udp_payload verdicts, datalen, payload offsets (2,736 crafted frames)
  F3  (a) 6,000 crafted events: histogram_event's verdicts and the table
      (b) 10 frame cases: per-frame OOB lines, totals, the sparse table
      (c) async bursts: tristan_process(buffer, len, ret) -> table, totals, raw bytes
  F4  a 1,024-frame fetch_xsk batch: counters under per-packet and batch-abort
      accounting, with and without the checksum configuration, and the table
"""
from pathlib import Path

import numpy as np
import pytest

import dqdk_amd as D
from test_gpu_parity import _need_gpu, run_gpu

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

GOLD = Path(__file__).resolve().parent / "golden"
HPATHS = [D.F_HISTO_ATOMIC, D.F_HISTO_PARTITIONED]
HIDS = ["atomic", "partitioned"]


def sparse(table):
    nz = np.flatnonzero(table)
    return nz.astype(np.uint32), table[nz]


def assert_table(table, idx, cnt, what=""):
    u, c = sparse(table)
    np.testing.assert_array_equal(u, idx, err_msg=what)
    np.testing.assert_array_equal(c, cnt, err_msg=what)


@pytest.fixture(scope="module")
def f3():
    return np.load(GOLD / "f3_decode.npz")


# ---- F1: get_udp_payload verdicts ------------------------------------------

def f1_expected_status(e, csum):
    """get_udp_payload (src/dqdk.c:185-207) + the checksum configuration,
    composed from the reference's recorded ip4_audit/udp_audit(+_checksum)."""
    st = np.full(len(e), D.RX_OK, dtype=np.uint8)
    st[e["datalen"] == 0] = D.RX_EMPTY
    if csum:
        st[e["udpc_ok"] == 0] = D.RX_INVALID_UDP_CSUM
    st[e["udp_ok"] == 0] = D.RX_INVALID_UDP
    if csum:
        st[e["ipc_ok"] == 0] = D.RX_INVALID_IP_CSUM
    st[e["ip_ok"] == 0] = D.RX_INVALID_IP
    return st


@pytest.mark.parametrize("csum", [False, True])
def test_f1_gpu_equals_reference(csum):
    z = np.load(GOLD / "f1_parse.npz")
    umem, desc, e = z["umem"].copy(), z["desc"], z["expected"]
    keep = np.ones(len(e), bool)
    if csum:  # ip4_audit_checksum is undefined in the reference for ihl > 5
        keep = (e["ipc_ok"] != 255) | (e["ip_ok"] == 0)
    desc, e = desc[keep], e[keep]
    cfg = D.RxConfig(payloadsz=64, mode=D.MODE_ENERGYHISTO, flags=D.F_CSUM if csum else 0)
    res, _, _, _, _ = run_gpu(umem, desc, cfg, keys=True)
    want = f1_expected_status(e, csum)
    np.testing.assert_array_equal(res["status"], want)
    okm = (want == D.RX_OK) | (want == D.RX_EMPTY)
    np.testing.assert_array_equal(res["datalen"][okm], e["datalen"][okm])
    np.testing.assert_array_equal(res["payload_off"][okm], e["payload_off"][okm])
    assert ((want == D.RX_OK) & (e["datalen"] > 0xFFFF0000)).sum() > 0  # the udplen < 8 wrap, accepted


# ---- F3 (a): single events wrapped in frames ---------------------------------

def frames_around(events: np.ndarray, per_frame: int):
    """Valid Eth/IPv4/UDP frames whose payloads are consecutive slices of events."""
    nf = len(events) // per_frame
    psz = 16 * per_frame
    L = 42 + psz
    stride = (L + 127) // 128 * 128
    umem = np.zeros(nf * stride + 256, np.uint8)
    for i in range(nf):
        f = umem[i * stride:]
        f[12], f[13], f[14] = 0x08, 0x00, 0x45
        f[16], f[17] = (L - 14) >> 8, (L - 14) & 0xFF
        f[23] = 17
        f[38], f[39] = (L - 34) >> 8, (L - 34) & 0xFF
        f[42:42 + psz] = events[i * per_frame:(i + 1) * per_frame].reshape(-1)
    desc = np.zeros(nf, D.DESC_DTYPE)
    desc["addr"] = np.arange(nf) * stride
    desc["len"] = L
    return umem, desc, psz


@pytest.mark.parametrize("hpath", HPATHS, ids=HIDS)
def test_f3_events_gpu_equals_reference(f3, hpath):
    ev = f3["ev_events"]
    umem, desc, psz = frames_around(ev, 100)
    cfg = D.RxConfig(payloadsz=psz, mode=D.MODE_ENERGYHISTO, flags=hpath)
    res, cnt, keys, hist, _ = run_gpu(umem, desc, cfg, keys=True, histogram=True)
    assert (res["status"] == D.RX_OK).all()
    rejected = (f3["ev_verdict"] != 0).reshape(len(desc), 100)
    np.testing.assert_array_equal(keys.reshape(len(desc), 100) == D.KEY_NONE, rejected)
    np.testing.assert_array_equal(res["oob_events"], rejected.sum(axis=1))
    assert_table(hist, f3["ev_hist_idx"], f3["ev_hist_cnt"])
    ev_tot, by_tot, oob = (int(x) for x in f3["ev_totals"])
    assert (cnt["total_events"], cnt["total_bytes"], cnt["oob_events"]) == (ev_tot, by_tot, oob)


# ---- F3 (b): frame cases -------------------------------------------------------

@pytest.mark.parametrize("hpath,records", [(D.F_HISTO_ATOMIC, True), (D.F_HISTO_PARTITIONED, True),
                                           (D.F_HISTO_PARTITIONED, False)], ids=["atomic", "partitioned", "fused"])
def test_f3_frame_cases_gpu_equal_reference(f3, hpath, records):
    for i, name in enumerate(str(n) for n in f3["case_names"]):
        p = f"c{i}_"
        mode, psz, E = (int(x) for x in f3[p + "cfg"])
        cfg = D.RxConfig(payloadsz=psz, mode=mode, flags=hpath)
        assert cfg.events == E
        histo = D.histo_enabled(mode, hpath)
        res, cnt, _, hist, _ = run_gpu(f3[p + "umem"].copy(), f3[p + "desc"], cfg, keys=records, histogram=histo)
        np.testing.assert_array_equal(res["status"], f3[p + "status"], err_msg=name)
        ok = res["status"] == D.RX_OK
        np.testing.assert_array_equal(res["datalen"][ok], f3[p + "datalen"][ok], err_msg=name)
        np.testing.assert_array_equal(res["oob_events"][ok], f3[p + "oob"][ok], err_msg=name)
        assert (cnt["total_events"], cnt["total_bytes"]) == tuple(int(x) for x in f3[p + "totals"]), name
        assert cnt["oob_events"] == int(f3[p + "oob"].sum()), name
        if histo:
            assert_table(hist, f3[p + "hist_idx"], f3[p + "hist_cnt"], name)
        else:
            assert len(f3[p + "hist_idx"]) == 0, name


# ---- F3 (c): the async consumer's bursts ----------------------------------------

def test_f3_async_bursts_gpu_equal_reference(f3):
    _need_gpu()
    for i in range(int(f3["async_cases"])):
        p = f"a{i}_"
        mode, psz, strip = (int(x) for x in f3[p + "cfg"])
        ring = f3[p + "ring"]
        bursts = f3[p + "bursts"]
        want_raw = f3[p + "raw"].tobytes()
        cfg = D.RxConfig(payloadsz=psz, mode=mode)
        with D.RxQueue(0, cfg, 1) as q:
            d_ring = torch.from_numpy(ring).cuda()
            out = torch.full((len(want_raw) + 64,), 0xAB, dtype=torch.uint8, device="cuda:0")
            q.set_stream(torch.cuda.current_stream().cuda_stream)
            n = q.async_process_device(d_ring.data_ptr(), ring.size // psz, bursts, bool(strip), out.data_ptr(),
                                       len(want_raw))
            torch.cuda.synchronize()
            assert n == len(want_raw), i
            got = out.cpu().numpy()
            assert got[:n].tobytes() == want_raw, i
            assert (got[n:] == 0xAB).all()
            cnt = q.counters()
            assert (cnt["total_events"], cnt["total_bytes"]) == tuple(int(x) for x in f3[p + "totals"]), i
            assert cnt["oob_events"] == int(f3[p + "oob"].sum()), i
            if D.histo_enabled(mode, 0):
                assert_table(q.histogram(), f3[p + "hist_idx"], f3[p + "hist_cnt"], str(i))
            else:
                assert len(f3[p + "hist_idx"]) == 0


def test_async_rejects_what_the_reference_ring_cannot_hold():
    _need_gpu()
    ring = torch.zeros(4 * 1458, dtype=torch.uint8, device="cuda:0")
    with D.RxQueue(0, D.RxConfig(payloadsz=1458, mode=D.MODE_LISTMODE), 1) as q:  # 1458 % 4 != 0
        with pytest.raises(D.DqdkError):
            q.async_process_device(ring.data_ptr(), 4, [1, 1])
    with D.RxQueue(0, D.RxConfig(payloadsz=1456, mode=D.MODE_LISTMODE), 1) as q:
        with pytest.raises(D.DqdkError):
            q.async_process_device(ring.data_ptr(), 4, [3, 2])  # overruns the ring
        assert q.async_process_device(ring.data_ptr(), 4, [3, 1]) == (3 + 1) * 1456  # len * ret per burst


# ---- F4: one fetch_xsk batch ---------------------------------------------------

@pytest.mark.parametrize("hpath,records", [(D.F_HISTO_ATOMIC, True), (D.F_HISTO_PARTITIONED, True),
                                           (D.F_HISTO_PARTITIONED, False)], ids=["atomic", "partitioned", "fused"])
@pytest.mark.parametrize("csum", [0, 1])
@pytest.mark.parametrize("abort", [0, 1])
def test_f4_batch_gpu_equals_reference(abort, csum, hpath, records):
    z = np.load(GOLD / "f4_batch.npz")
    mode, psz = (int(x) for x in z["cfg"])
    flags = (D.F_CSUM if csum else 0) | (D.F_BATCH_ABORT if abort else 0) | hpath
    cfg = D.RxConfig(payloadsz=psz, mode=mode, flags=flags)
    res, cnt, _, hist, _ = run_gpu(z["umem"].copy(), z["desc"], cfg, keys=records, histogram=True)
    np.testing.assert_array_equal(res["status"], z[f"status_csum{csum}"])
    ok = res["status"] == D.RX_OK
    np.testing.assert_array_equal(res["datalen"][ok], z[f"datalen_csum{csum}"][ok])
    k = f"csum{csum}_abort{abort}_"
    for name, v in zip((str(n) for n in z["counter_names"]), (int(x) for x in z[k + "counters"])):
        assert cnt[name] == v, (name, cnt[name], v)
    assert_table(hist, z[k + "hist_idx"], z[k + "hist_cnt"])
