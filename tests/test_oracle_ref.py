"""Differential test: every restated src/tcpip function vs the reference's own
src/tcpip/{ipv4,udp,inet_csum}.c compiled verbatim (oracle/_ref, built by
`make -C oracle ref` where /root/reference exists; skipped elsewhere -- the
committed golden fixtures cover the same functions)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (no reference here)")


def test_random_differential():
    ref, orc = O.ref(), O.oracle()
    rng = np.random.default_rng(99)
    buf = rng.integers(0, 256, size=80000, dtype=np.uint8)
    b = buf.ctypes.data
    for _ in range(3000):
        off = int(rng.integers(0, 64))
        ln = int(rng.integers(0, 3000))
        assert orc.or_inet_csum(b + off, ln) == ref.inet_csum(b + off, ln)
        ihl = int(rng.integers(0, 16))
        assert orc.or_ip_fast_csum(b + off, ihl) == ref.ip_fast_csum(b + off, ihl)
        sa, da = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))
        L = int(rng.integers(0, 9001))
        assert orc.or_udp_csum(sa, da, L, 17, b + off) == ref.udp_csum(sa, da, L, 17, b + off)
        al = int(rng.integers(0, 65536))
        assert orc.or_ip4_audit(b + off, al) == ref.ip4_audit(b + off, al)
        assert orc.or_udp_audit(b + off, sa, da, al) == ref.udp_audit(b + off, sa, da, al)
        x = int(rng.integers(0, 2**32))
        assert orc.or_csum_fold(x) == ref.csum_fold(x)
    for _ in range(2000):
        h = np.zeros(64, np.uint8)
        h[:20] = rng.integers(0, 256, size=20, dtype=np.uint8)
        h[0] = (h[0] & 0xF0) | int(rng.integers(0, 6))
        if rng.random() < 0.5:
            h[10] = h[11] = 0
            ck = ref.ip_fast_csum(h.ctypes.data, int(h[0]) & 0xF)
            h[10], h[11] = ck & 0xFF, ck >> 8
        assert orc.or_ip4_audit_checksum(h.ctypes.data) == ref.ip4_audit_checksum(h.ctypes.data)
    for _ in range(500):
        u = rng.integers(0, 256, size=4096, dtype=np.uint8)
        sa, da, L = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)), int(rng.integers(0, 4000))
        if rng.random() < 0.5:
            u[6] = u[7] = 0
            ck = ref.udp_csum(sa, da, L, 17, u.ctypes.data)
            u[6], u[7] = ck & 0xFF, ck >> 8
        u1, u2 = u.copy(), u.copy()
        assert orc.or_udp_audit_checksum(u1.ctypes.data, sa, da, L, 1) == \
            ref.udp_audit_checksum(u2.ctypes.data, sa, da, L)
        assert np.array_equal(u1, u2)  # same in-place side effect (udp.c:17)
