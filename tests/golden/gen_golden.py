#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs only where /root/reference exists (this container): it loads
oracle/_ref/libref_tcpip.so -- the reference's src/tcpip/{ipv4,udp,inet_csum}.c
compiled verbatim by `make -C oracle ref` -- and records its outputs on
seeded inputs.  The fixtures are data (inputs + the reference's outputs);
no reference source is copied.

  f1_parse.npz  get_udp_payload verdicts (src/dqdk.c:185-207) on crafted
                frames, composed exactly as dqdk.c does from the reference's
                ip4_audit / udp_audit (and, for the checksum config,
                ip4_audit_checksum / udp_audit_checksum).
  f2_csum.npz   inet_csum / ip_fast_csum / udp_csum / csum_* / from* /
                ip4_audit_checksum / udp_audit_checksum known answers.

The composition in f1 (u32 udplen, (u16) truncations, datalen = udplen - 8)
restates the five lines of get_udp_payload; everything that decides a
verdict is a call into the reference build.

Usage: python tests/golden/gen_golden.py   (after `make -C oracle ref`)
"""
from __future__ import annotations

import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle as O  # noqa: E402

OUT = Path(__file__).resolve().parent
SEED = 20261015
PAD = 70000  # zero tail so a wrapped u16 udplen checksum read stays in the image


def be16(b, o):
    return (int(b[o]) << 8) | int(b[o + 1])


def le16(b, o):
    return int(b[o]) | (int(b[o + 1]) << 8)


def le32(b, o):
    return int(b[o]) | (int(b[o + 1]) << 8) | (int(b[o + 2]) << 16) | (int(b[o + 3]) << 24)


def make_frames(rng):
    """Crafted frames: edge sizes, every ihl, right/wrong lengths, udplen < 8, == 8."""
    frames = []
    sizes = [0, 1, 13, 14, 15, 20, 33, 34, 35, 41, 42, 43, 44, 50, 60, 64, 100, 128, 200]
    for _ in range(2600):
        L = int(rng.choice(sizes)) if rng.random() < 0.5 else int(rng.integers(0, 240))
        frames.append(L)
    big = [1500, 3434, 9000, 1501, 3435, 8999, 9001, 1499, 4095]
    for _ in range(80):
        frames.append(int(rng.choice(big)))
    return frames


def fill_frame(rng, f, L, kind):
    """Write headers into frame view f (len >= max(L, 128))."""
    f[:] = rng.integers(0, 256, size=f.size, dtype=np.uint8)
    f[12], f[13] = 0x08, 0x00
    ihl = int(rng.integers(0, 16)) if kind == "anyihl" else (5 if rng.random() < 0.8 else int(rng.integers(5, 16)))
    f[14] = 0x40 | ihl
    hs = ihl * 4
    tot = (L - 14) & 0xFFFF
    r = rng.random()
    if r < 0.15:
        tot = (tot + int(rng.integers(1, 5))) & 0xFFFF     # wrong tot_len
    elif r < 0.2:
        tot = int(rng.integers(0, 65536))
    f[16], f[17] = tot >> 8, tot & 0xFF
    f[23] = 17
    udplen = (tot - hs) & 0xFFFFFFFF
    u = 14 + hs
    ul = udplen & 0xFFFF
    r = rng.random()
    if r < 0.1:
        ul = (ul + 2) & 0xFFFF                               # wrong udp.len
    elif r < 0.15:
        ul = int(rng.integers(0, 65536))
    f[u + 4], f[u + 5] = ul >> 8, ul & 0xFF
    if rng.random() < 0.2:
        f[u + 6] = f[u + 7] = 0                              # "no checksum"
    return ihl


def gen_f1(ref, rng):
    frames = make_frames(rng)
    # forced quirk frames: udplen < 8 (datalen wraps) and == 8 (datalen 0)
    extra = []
    for L in (40, 41, 42, 38, 34, 30, 22):
        extra.append(L)
    frames += extra * 8
    addrs, lens = [], []
    off = 0
    for L in frames:
        off = (off + 63) // 64 * 64 + int(rng.integers(0, 8))   # include odd / 2-aligned frame starts
        addrs.append(off)
        lens.append(L)
        off += max(L, 128) + 96
    size = (off + PAD + 15) // 16 * 16
    umem = np.zeros(size, dtype=np.uint8)
    for k, (a, L) in enumerate(zip(addrs, lens)):
        fill_frame(rng, umem[a:a + max(L, 128) + 96], L, "anyihl" if k % 3 == 0 else "std")
        if L in (40, 41, 42, 38, 34, 30, 22) and k >= len(frames) - len(extra) * 8:
            # make tot_len and udp.len consistent so the udplen quirks are reached
            f = umem[a:]
            f[14] = 0x45
            tot = (L - 14) & 0xFFFF
            f[16], f[17] = tot >> 8, tot & 0xFF
            ul = (tot - 20) & 0xFFFF
            f[38], f[39] = ul >> 8, ul & 0xFF
    n = len(addrs)
    base = umem.ctypes.data
    # give most frames a VALID ip / udp checksum (computed by the reference's
    # own ip_fast_csum / udp_csum) so the checksum config reaches its success
    # path, not only failures
    for k in range(n):
        a = addrs[k]
        f = umem[a:]
        ihl = int(f[14]) & 0xF
        if rng.random() < 0.7 and ihl <= 5:
            hdr = np.zeros(64, np.uint8)
            hdr[:20] = f[14:34]
            hdr[10] = hdr[11] = 0
            ck = ref.ip_fast_csum(hdr.ctypes.data, ihl)
            f[24], f[25] = ck & 0xFF, ck >> 8
        if rng.random() < 0.7:
            hs = ihl * 4
            u = a + 14 + hs
            if le16(umem, u + 6) != 0:
                udplen = (be16(f, 16) - hs) & 0xFFFF
                saddr, daddr = le32(f, 26), le32(f, 30)
                umem[u + 6] = umem[u + 7] = 0
                ck = ref.udp_csum(saddr, daddr, udplen, 17, base + u)
                umem[u + 6], umem[u + 7] = ck & 0xFF, ck >> 8
    exp = np.zeros(n, dtype=[("ip_ok", "u1"), ("udp_ok", "u1"), ("ipc_ok", "u1"), ("udpc_ok", "u1"),
                             ("hs", "<u4"), ("udplen", "<u4"), ("datalen", "<u4"), ("payload_off", "<u4")])
    for k in range(n):
        a, L = addrs[k], lens[k]
        f = umem[a:]
        iph = base + a + 14
        ip_ok = ref.ip4_audit(iph, (L - 14) & 0xFFFF)                          # dqdk.c:191
        ihl = int(f[14]) & 0xF
        hs = ihl * 4                                                          # dqdk.c:196
        udplen = (be16(f, 16) - hs) & 0xFFFFFFFF                              # dqdk.c:197
        saddr, daddr = le32(f, 26), le32(f, 30)
        udp = iph + hs                                                        # dqdk.c:198
        udp_ok = ref.udp_audit(udp, saddr, daddr, udplen & 0xFFFF)            # dqdk.c:200
        ipc_ok = ref.ip4_audit_checksum(iph) if ihl <= 5 else 255             # ipv4.c:6-11 (UB for ihl>5)
        # udp_audit_checksum zeroes udp->check in place: run it on a copy
        scratch = np.ascontiguousarray(umem[a:a + 14 + hs + 8 + 65536 + 2].copy())
        # keep the same address parity as in the image
        pad = np.zeros(len(scratch) + 16, dtype=np.uint8)
        sh = (a - pad.ctypes.data) % 16
        pad[sh:sh + len(scratch)] = scratch
        udpc_ok = ref.udp_audit_checksum(pad.ctypes.data + sh + 14 + hs, saddr, daddr, udplen & 0xFFFF)
        exp[k] = (ip_ok, udp_ok, ipc_ok, udpc_ok, hs, udplen, (udplen - 8) & 0xFFFFFFFF, 14 + hs + 8)
    desc = np.zeros(n, dtype=O.DESC_DTYPE)
    desc["addr"] = addrs
    desc["len"] = lens
    np.savez_compressed(OUT / "f1_parse.npz", umem=umem, desc=desc, expected=exp)
    return n


def gen_f2(ref, rng):
    pool = rng.integers(0, 256, size=65536 + 64, dtype=np.uint8)
    pool[-64:] = rng.integers(1, 256, size=64, dtype=np.uint8)
    base = pool.ctypes.data
    rows = []
    # inet_csum / inet_fast_csum on every alignment
    for _ in range(1500):
        off = int(rng.integers(0, 64))
        ln = int(rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 20, 60, int(rng.integers(0, 9001))]))
        rows.append(("inet_csum", off, ln, 0, 0, ref.inet_csum(base + off, ln)))
        rows.append(("inet_fast_csum", off, ln, 0, 0, ref.inet_fast_csum(base + off, ln)))
    for _ in range(300):
        off = int(rng.integers(0, 64))
        ihl = int(rng.integers(0, 16))
        rows.append(("ip_fast_csum", off, ihl, 0, 0, ref.ip_fast_csum(base + off, ihl)))
    # udp_csum: odd lengths read the byte AT len (pool tail bytes are non-zero)
    for _ in range(1500):
        off = int(rng.integers(0, 64)) * 2 + int(rng.integers(0, 2))
        ln = int(rng.integers(0, 9001)) if rng.random() < 0.8 else int(rng.integers(0, 65536 - 200))
        sa, da = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))
        rows.append(("udp_csum", off, ln, sa, da, ref.udp_csum(sa, da, ln, 17, base + off)))
    # pure arithmetic helpers
    for _ in range(500):
        x = int(rng.integers(0, 2**32))
        y = int(rng.integers(0, 2**63)) * 2 + int(rng.integers(0, 2))
        rows.append(("from32to16", 0, 0, x, 0, ref.from32to16(x)))
        rows.append(("from64to32", 0, 0, y, 0, ref.from64to32(y)))
        rows.append(("csum_fold", 0, 0, x, 0, ref.csum_fold(x)))
        sa, da, ln, s = (int(rng.integers(0, 2**32)) for _ in range(4))
        ln &= 0xFFFF
        rows.append(("csum_tcpudp_nofold", s, ln, sa, da, ref.csum_tcpudp_nofold(sa, da, ln, 17, s)))
        rows.append(("csum_tcpudp_magic", s, ln, sa, da, ref.csum_tcpudp_magic(sa, da, ln, 17, s)))
    kinds = sorted({r[0] for r in rows})
    kind_id = {k: i for i, k in enumerate(kinds)}
    tab = np.array([(kind_id[r[0]], r[1], r[2], r[3], r[4], r[5]) for r in rows],
                   dtype=[("kind", "u1"), ("a", "<u8"), ("b", "<u8"), ("x", "<u8"), ("y", "<u8"), ("out", "<u8")])

    # ip4_audit_checksum on headers with ihl <= 5, valid and corrupted
    hdr_rows = []
    hdrs = np.zeros((400, 20), dtype=np.uint8)
    for k in range(400):
        h = rng.integers(0, 256, size=20, dtype=np.uint8)
        h[0] = 0x40 | int(rng.integers(0, 6))
        h[10] = h[11] = 0
        buf = np.zeros(32, dtype=np.uint8)
        buf[:20] = h
        ck = ref.ip_fast_csum(buf.ctypes.data, int(h[0]) & 0xF)
        if rng.random() < 0.5:
            ck ^= int(rng.integers(1, 65536))
        h[10], h[11] = ck & 0xFF, ck >> 8
        hdrs[k] = h
        buf[:20] = h
        hdr_rows.append(ref.ip4_audit_checksum(buf.ctypes.data))
    # udp_audit_checksum: check == 0, valid, corrupted, computed-0 vs 0xFFFF
    udp_bufs = np.zeros((400, 2048), dtype=np.uint8)
    udp_meta = np.zeros(400, dtype=[("len", "<u4"), ("sa", "<u4"), ("da", "<u4"), ("ok", "u1"),
                                    ("check_after", "<u2")])
    for k in range(400):
        ln = int(rng.integers(8, 2000))
        u = rng.integers(0, 256, size=2048, dtype=np.uint8)
        sa, da = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))
        u[6] = u[7] = 0
        calc = ref.udp_csum(sa, da, ln, 17, u.ctypes.data)
        mode = k % 4
        if mode == 0:
            ck = 0
        elif mode == 1:
            ck = calc
        elif mode == 2:
            ck = calc ^ int(rng.integers(1, 65536))
        else:
            ck = 0xFFFF if calc == 0 else calc  # the one's-complement "-0" case
        u[6], u[7] = ck & 0xFF, ck >> 8
        udp_bufs[k] = u
        w = u.copy()
        ok = ref.udp_audit_checksum(w.ctypes.data, sa, da, ln)
        udp_meta[k] = (ln, sa, da, ok, le16(w, 6))
    np.savez_compressed(OUT / "f2_csum.npz", pool=pool, tab=tab, kinds=np.array(kinds), hdrs=hdrs,
                        hdr_ok=np.array(hdr_rows, dtype=np.uint8), udp_bufs=udp_bufs, udp_meta=udp_meta)
    return len(rows)


def main():
    if not O.ref_available():
        sys.exit("oracle/_ref/libref_tcpip.so missing: run `make -C oracle ref` where /root/reference exists")
    ref = O.ref()
    ref.udp_csum.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint8, C.c_void_p]
    rng = np.random.default_rng(SEED)
    n1 = gen_f1(ref, rng)
    n2 = gen_f2(ref, rng)
    print(f"f1_parse: {n1} frames; f2_csum: {n2} rows")


if __name__ == "__main__":
    main()
