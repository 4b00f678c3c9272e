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
