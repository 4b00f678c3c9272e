"""Oracle vs the golden fixtures made from the reference's own src/tcpip build.

tests/golden/f1_parse.npz and f2_csum.npz hold the outputs of
/root/reference/src/tcpip/{ipv4,udp,inet_csum}.c compiled verbatim
(tests/golden/gen_golden.py); this pins the C restatement in oracle/.
"""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O

GOLD = Path(__file__).resolve().parent / "golden"
OK, INV_IP, INV_UDP, EMPTY, IP_CSUM, UDP_CSUM = 0, 1, 2, 3, 4, 5


def expected_status(e, csum):
    """get_udp_payload (src/dqdk.c:185-207) + checksum config composition."""
    st = np.full(len(e), OK, dtype=np.uint8)
    st[e["datalen"] == 0] = EMPTY
    if csum:
        st[(e["udpc_ok"] == 0)] = UDP_CSUM
    st[e["udp_ok"] == 0] = INV_UDP
    if csum:
        st[(e["ipc_ok"] == 0)] = IP_CSUM
    st[e["ip_ok"] == 0] = INV_IP
    return st


@pytest.mark.parametrize("csum", [False, True])
def test_f1_parse_verdicts(csum):
    z = np.load(GOLD / "f1_parse.npz")
    umem, desc, e = z["umem"].copy(), z["desc"], z["expected"]
    res, cnt, _ = O.rx_batch(umem, desc, payloadsz=0, mode=3, flags=1 if csum else 0, want_keys=False)
    exp = expected_status(e, csum)
    keep = np.ones(len(e), bool)
    if csum:  # ip4_audit_checksum is undefined in the reference for ihl > 5
        keep = (e["ipc_ok"] != 255) | (e["ip_ok"] == 0)
    assert keep.sum() > 1500
    np.testing.assert_array_equal(res["status"][keep], exp[keep])
    okm = keep & ((exp == OK) | (exp == EMPTY))
    np.testing.assert_array_equal(res["datalen"][okm], e["datalen"][okm])
    np.testing.assert_array_equal(res["payload_off"][okm], e["payload_off"][okm])
    # every branch of the composition is exercised by the fixture
    for s in ((OK, EMPTY, INV_IP, INV_UDP, IP_CSUM, UDP_CSUM) if csum else (OK, EMPTY, INV_IP, INV_UDP)):
        assert (exp[keep] == s).sum() > 0, s
    # the udplen < 8 wrap (datalen ~ 4G) is present and accepted as OK
    assert ((exp == OK) & (e["datalen"] > 0xFFFF0000)).sum() > 0


def test_f2_checksums():
    z = np.load(GOLD / "f2_csum.npz")
    pool = z["pool"].copy()
    base = pool.ctypes.data
    assert base % 64 == 0 or True  # parity of (base + off) matters only mod 2/4: numpy aligns >= 16
    assert base % 16 == 0
    lib = O.oracle()
    kinds = [str(k) for k in z["kinds"]]
    fn = {
        "inet_csum": lambda r: lib.or_inet_csum(base + int(r["a"]), int(r["b"])),
        "inet_fast_csum": lambda r: lib.or_inet_fast_csum(base + int(r["a"]), int(r["b"])),
        "ip_fast_csum": lambda r: lib.or_ip_fast_csum(base + int(r["a"]), int(r["b"])),
        "udp_csum": lambda r: lib.or_udp_csum(int(r["x"]), int(r["y"]), int(r["b"]), 17, base + int(r["a"])),
        "from32to16": lambda r: lib.or_from32to16(int(r["x"])),
        "from64to32": lambda r: lib.or_from64to32(int(r["x"])),
        "csum_fold": lambda r: lib.or_csum_fold(int(r["x"])),
        "csum_tcpudp_nofold": lambda r: lib.or_csum_tcpudp_nofold(int(r["x"]), int(r["y"]), int(r["b"]), 17,
                                                                   int(r["a"])),
        "csum_tcpudp_magic": lambda r: lib.or_csum_tcpudp_magic(int(r["x"]), int(r["y"]), int(r["b"]), 17,
                                                                 int(r["a"])),
    }
    seen = set()
    for r in z["tab"]:
        k = kinds[r["kind"]]
        seen.add(k)
        assert fn[k](r) == int(r["out"]), (k, r)
    assert seen == set(fn)


def test_f2_audit_checksums():
    z = np.load(GOLD / "f2_csum.npz")
    lib = O.oracle()
    for h, ok in zip(z["hdrs"], z["hdr_ok"]):
        buf = np.zeros(64, np.uint8)
        buf[:20] = h
        assert lib.or_ip4_audit_checksum(buf.ctypes.data) == ok
    meta = z["udp_meta"]
    assert set(np.unique(meta["ok"])) == {0, 1}
    for u, m in zip(z["udp_bufs"], meta):
        w = u.copy()
        got = lib.or_udp_audit_checksum(w.ctypes.data, int(m["sa"]), int(m["da"]), int(m["len"]), 1)
        assert got == m["ok"]
        # udp->check is zeroed in place (src/tcpip/udp.c:17) unless it was 0
        assert int(w[6]) | (int(w[7]) << 8) == m["check_after"]


# ---- F3 / F4: the TRISTAN decode and the batch accounting, from the reference --------
# tests/golden/f3_decode.npz and f4_batch.npz hold the outputs of the reference's
# own histogram_event / process_events_unrolled16 / tristan_process (extracted
# verbatim from src/tristan.{c,h}, oracle/ref_tristan.py) and src/tcpip
# (tests/golden/gen_tristan.py).

def _sparse(table):
    nz = np.flatnonzero(table)
    return nz.astype(np.uint32), table[nz]


@pytest.fixture(scope="module")
def f3():
    return np.load(GOLD / "f3_decode.npz")


@pytest.fixture(scope="module")
def table():
    return np.zeros(O.HISTO_ENTRIES, np.uint32)


def test_f3_event_keys_and_verdicts(f3):
    ev = f3["ev_events"]
    keys = O.event_keys(ev)
    np.testing.assert_array_equal(keys == 0xFFFFFFFF, f3["ev_verdict"] != 0)  # histogram_event's -1
    u, c = np.unique(keys[keys != 0xFFFFFFFF], return_counts=True)
    np.testing.assert_array_equal(u, f3["ev_hist_idx"])
    np.testing.assert_array_equal(c, f3["ev_hist_cnt"])
    ev_tot, by_tot, oob = f3["ev_totals"]
    assert (ev_tot, by_tot, oob) == (len(ev), 16 * len(ev), int((keys == 0xFFFFFFFF).sum()))
    # every bounds edge is in the fixture
    ch = ev[:, 2].astype(np.int64) | (ev[:, 3].astype(np.int64) << 8)
    assert {1511, 1512, 65535} <= set(ch.tolist())
    assert ((ev[:, 8] & 7) >= 6).any() and (ev[:, 8] >> 3).any()


def _f3_cases(f3):
    return [(i, str(n)) for i, n in enumerate(f3["case_names"])]


def test_f3_frame_cases(f3, table):
    for i, name in _f3_cases(f3):
        p = f"c{i}_"
        mode, psz, E = (int(x) for x in f3[p + "cfg"])
        assert O.events_per_payload(mode, psz) == E, name
        table[:] = 0
        umem = f3[p + "umem"].copy()
        res, cnt, _ = O.rx_batch(umem, f3[p + "desc"], psz, mode, 0, hist=table)
        np.testing.assert_array_equal(res["status"], f3[p + "status"], err_msg=name)
        ok = res["status"] == 0
        np.testing.assert_array_equal(res["datalen"][ok], f3[p + "datalen"][ok], err_msg=name)
        np.testing.assert_array_equal(res["oob_events"][ok], f3[p + "oob"][ok], err_msg=name)
        assert (cnt["total_events"], cnt["total_bytes"]) == tuple(int(x) for x in f3[p + "totals"]), name
        assert cnt["oob_events"] == int(f3[p + "oob"].sum()), name
        u, c = _sparse(table)
        np.testing.assert_array_equal(u, f3[p + "hist_idx"], err_msg=name)
        np.testing.assert_array_equal(c, f3[p + "hist_cnt"], err_msg=name)


def test_f3_async_bursts(f3, table):
    for i in range(int(f3["async_cases"])):
        p = f"a{i}_"
        mode, psz, strip = (int(x) for x in f3[p + "cfg"])
        table[:] = 0
        cnt, raw = O.async_process(f3[p + "ring"], f3[p + "bursts"], psz, mode, bool(strip), hist=table)
        assert raw == f3[p + "raw"].tobytes(), i
        assert (cnt["total_events"], cnt["total_bytes"]) == tuple(int(x) for x in f3[p + "totals"]), i
        assert cnt["oob_events"] == int(f3[p + "oob"].sum()), i
        u, c = _sparse(table)
        np.testing.assert_array_equal(u, f3[p + "hist_idx"])
        np.testing.assert_array_equal(c, f3[p + "hist_cnt"])
        if int(f3[p + "bursts"].max()) > 1 and mode != 0:
            assert f3[p + "hist_cnt"].max() > 1  # first payload counted `burst` times


@pytest.mark.parametrize("csum", [0, 1])
@pytest.mark.parametrize("abort", [0, 1])
def test_f4_batch_accounting(csum, abort, table):
    z = np.load(GOLD / "f4_batch.npz")
    mode, psz = (int(x) for x in z["cfg"])
    table[:] = 0
    flags = (1 if csum else 0) | (2 if abort else 0)
    res, cnt, _ = O.rx_batch(z["umem"].copy(), z["desc"], psz, mode, flags, hist=table)
    np.testing.assert_array_equal(res["status"], z[f"status_csum{csum}"])
    ok = res["status"] == 0
    np.testing.assert_array_equal(res["datalen"][ok], z[f"datalen_csum{csum}"][ok])
    k = f"csum{csum}_abort{abort}_"
    want = dict(zip([str(n) for n in z["counter_names"]], (int(x) for x in z[k + "counters"])))
    for name, v in want.items():
        assert cnt[name] == v, (name, cnt[name], v)
    u, c = _sparse(table)
    np.testing.assert_array_equal(u, z[k + "hist_idx"])
    np.testing.assert_array_equal(c, z[k + "hist_cnt"])
