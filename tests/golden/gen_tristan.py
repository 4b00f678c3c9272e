#!/usr/bin/env python3
"""Generate the TRISTAN-side golden fixtures from the REFERENCE itself.

Runs only where /root/reference exists (this container).  It loads

  oracle/_ref/libref_tristan.so  the reference's histogram_event,
                                 process_events_unrolled16, tristan_process,
                                 get_energy_events_count, is_store_histo and
                                 the tristan_histo_t / energy_evt layout,
                                 extracted verbatim from src/tristan.{c,h} and
                                 compiled by oracle/ref_tristan.py
  oracle/_ref/libref_tcpip.so    src/tcpip/{ipv4,udp,inet_csum}.c verbatim

and records their outputs on seeded inputs.  Fixtures are data (inputs +
the reference's outputs); no reference source is copied.

  f3_decode.npz  (a) single events: histogram_event's verdict per event and
                     the table after tristan_process over all of them;
                 (b) frame cases: per OK frame tristan_process(payload,
                     datalen, burst = 1) -- process_unbuffered_frame,
                     src/tristan.c:377-381 -- in descriptor order into one
                     table: sparse histogram, total_events, total_bytes and
                     the out-of-bounds lines histogram_event printed per frame;
                 (c) async bursts: tristan_process(buffer, len, burst) as
                     async_processor calls it (src/tristan.c:332-375; len =
                     16 with strip_wfm, else payloadsz): histogram, totals,
                     and the bytes it write()s to the raw fd.
  f4_batch.npz   one 1024-frame fetch_xsk batch (src/dqdk.c:252-322) over a
                 UMEM image: per-frame verdicts from the reference's
                 ip4_audit / udp_audit (+ ip4_audit_checksum /
                 udp_audit_checksum), then tristan_process per processed OK
                 frame, under per-packet and batch-abort accounting, with and
                 without the checksum configuration.

Restated glue (the reference's own code for it cannot be built here: its
only type, dqdk_worker_t, needs libxdp -- oracle/ref_tristan.py): the
get_udp_payload composition (u32 udplen, (u16) casts, datalen = udplen - 8,
src/dqdk.c:185-207), process_frame's datalen != 0 test and rcvd_bytes
(:231-250) and fetch_xsk's counters and abort (:289-321).  Everything that
decides a verdict, a bin, a count or a total is a call into the reference.

Usage: python tests/golden/gen_tristan.py   (after `make -C oracle ref`)
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle as O  # noqa: E402

OUT = Path(__file__).resolve().parent
SEED = 20261016
TRISTAN_LIB = ROOT / "oracle" / "_ref" / "libref_tristan.so"
OOB_TAG = b"Out of bounds Energy Event"
MODE_WAVEFORM, MODE_LISTWAVE, MODE_LISTMODE, MODE_ENERGYHISTO = range(4)
OK, INV_IP, INV_UDP, EMPTY, IP_CSUM, UDP_CSUM = range(6)


def load_tristan():
    t = C.CDLL(str(TRISTAN_LIB))
    t.rt_sizeof_energy_evt.restype = C.c_size_t
    t.rt_histo_sz.restype = C.c_ulonglong
    t.rt_chnls_count.restype = C.c_int
    t.rt_is_store_histo.restype = C.c_int
    t.rt_is_store_histo.argtypes = [C.c_int]
    t.rt_get_energy_events_count.restype = C.c_uint32
    t.rt_get_energy_events_count.argtypes = [C.c_int, C.c_uint32]
    t.rt_histogram_event.restype = C.c_int
    t.rt_histogram_event.argtypes = [C.c_void_p, C.c_void_p]
    t.rt_tristan_process.restype = C.c_int
    t.rt_tristan_process.argtypes = [C.c_int, C.c_uint32, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_uint32,
                                     C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    t.rt_flush_stdout.restype = None
    assert t.rt_sizeof_energy_evt() == 16
    assert t.rt_histo_sz() == O.HISTO_ENTRIES * 4
    return t


class StdoutTap:
    """fd 1 -> a temp file, so histogram_event's dlog_errorv lines (one per
    out-of-bounds event, src/tristan.c:239) can be counted per call."""

    def __init__(self, lib):
        self.lib = lib
        self.f = tempfile.TemporaryFile()
        self.saved = os.dup(1)
        sys.stdout.flush()
        os.dup2(self.f.fileno(), 1)
        self.pos = 0

    def take(self) -> int:
        self.lib.rt_flush_stdout()
        self.f.seek(self.pos)
        data = self.f.read()
        self.pos += len(data)
        return data.count(OOB_TAG)

    def close(self):
        self.lib.rt_flush_stdout()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        self.f.close()


class RefTristan:
    """One tristan_t-shaped state: the reference's table + its two atomics."""

    def __init__(self, lib, tap, mode, payloadsz):
        self.lib, self.tap, self.mode, self.payloadsz = lib, tap, mode, payloadsz
        self.table = np.zeros(O.HISTO_ENTRIES, np.uint32)  # calloc'd tristan_histo_t (src/tristan.c:97)
        self.events = C.c_uint64(0)
        self.bytes = C.c_uint64(0)
        self.histo_fd = 3 if lib.rt_is_store_histo(mode) else -1  # tristan_init :135-150 (fd only tested > 0)

    def process(self, ptr, length, burst=1, raw_fd=-1) -> int:
        """tristan_process(private, buffer, len, burst); returns the OOB lines printed."""
        rc = self.lib.rt_tristan_process(self.mode, self.payloadsz, self.table.ctypes.data, self.histo_fd, raw_fd,
                                         ptr, length, burst, C.byref(self.events), C.byref(self.bytes))
        assert rc == 0, rc
        return self.tap.take()

    def sparse(self):
        nz = np.flatnonzero(self.table)
        return nz.astype(np.uint32), self.table[nz].astype(np.uint32)


# ---- synthetic inputs --------------------------------------------------------

def craft_events(rng, n, hot=0.0):
    """16-B energy events (src/tristan.h:13-25) with every bounds edge."""
    ev = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    ch = rng.integers(0, 1512, size=n)
    r = rng.random(n)
    edge = np.array([0, 1, 1510, 1511, 1512, 1513, 2047, 4096, 32768, 65535])
    sel = r < 0.08
    ch[sel] = rng.choice(edge, size=int(sel.sum()))
    ev[:, 2] = ch & 0xFF
    ev[:, 3] = ch >> 8
    hc = rng.integers(0, 6, size=n)
    sel = rng.random(n) < 0.05
    hc[sel] = rng.integers(6, 8, size=int(sel.sum()))
    reserved = np.where(rng.random(n) < 0.5, rng.integers(0, 32, size=n), 0)
    ev[:, 8] = (hc | (reserved << 3)).astype(np.uint8)
    en = rng.integers(0, 1 << 24, size=n)
    sel = rng.random(n) < 0.05
    en[sel] = rng.choice(np.array([0, 0xFF, 0x100, 0xFFFF, 0x10000, 0xFFFF00, 0xFFFFFF]), size=int(sel.sum()))
    ev[:, 4] = en & 0xFF
    ev[:, 5] = (en >> 8) & 0xFF
    ev[:, 6] = (en >> 16) & 0xFF
    if hot:
        sel = rng.random(n) < hot  # a few hot bins (peaked spectra, counts well past 256)
        pk = np.array([[3, 0, 0x12, 0x34, 1], [700, 0, 0xFF, 0xFF, 4], [1511, 0, 0, 0, 5]])
        k = rng.integers(0, len(pk), size=int(sel.sum()))
        ev[sel, 2] = pk[k, 0] & 0xFF
        ev[sel, 3] = pk[k, 0] >> 8
        ev[sel, 5] = pk[k, 2]
        ev[sel, 6] = pk[k, 3]
        ev[sel, 8] = pk[k, 4]
    return ev


def put_frame(umem, a, L, payload, rng, ihl=5, tot_delta=0, ulen_delta=0):
    """Eth + IPv4 + UDP headers at umem[a:] for a frame of L bytes, then payload."""
    f = umem[a:a + max(L, 64)]
    hs = ihl * 4
    f[:14] = rng.integers(0, 256, size=14, dtype=np.uint8)
    f[12], f[13] = 0x08, 0x00
    f[14] = 0x40 | ihl
    f[15] = 0
    tot = (L - 14 + tot_delta) & 0xFFFF
    f[16], f[17] = tot >> 8, tot & 0xFF
    f[18:22] = rng.integers(0, 256, size=4, dtype=np.uint8)
    f[22], f[23] = 64, 17
    f[24] = f[25] = 0
    f[26:30] = [192, 168, 10, 103]
    f[30:34] = [192, 168, 10, 1]
    if hs > 20:
        f[34:14 + hs] = rng.integers(0, 256, size=hs - 20, dtype=np.uint8)
    u = 14 + hs
    f[u:u + 2] = [0x13, 0x88]
    f[u + 2:u + 4] = [0x13, 0x88]
    ul = (tot - hs + ulen_delta) & 0xFFFF
    f[u + 4], f[u + 5] = ul >> 8, ul & 0xFF
    f[u + 6] = f[u + 7] = 0
    p = u + 8
    m = max(0, min(len(payload), L - p))
    f[p:p + m] = payload[:m]


def set_checksums(tcp, umem, a, rng, p_ip=0.9, p_udp=0.9, p_bad=0.1):
    """Valid IPv4 / UDP checksums by the reference's own ip_fast_csum / udp_csum
    (some corrupted, some UDP check = 0 'no checksum')."""
    f = umem[a:]
    ihl = int(f[14]) & 0xF
    if rng.random() < p_ip:
        hdr = np.zeros(64, np.uint8)
        hdr[:ihl * 4] = f[14:14 + ihl * 4]
        hdr[10] = hdr[11] = 0
        ck = tcp.ip_fast_csum(hdr.ctypes.data, ihl)
        if rng.random() < p_bad:
            ck ^= 0x0101
        f[24], f[25] = ck & 0xFF, ck >> 8
    if rng.random() < p_udp:
        hs = ihl * 4
        u = a + 14 + hs
        udplen = ((int(f[16]) << 8 | int(f[17])) - hs) & 0xFFFF
        umem[u + 6] = umem[u + 7] = 0
        saddr = int.from_bytes(bytes(f[26:30]), "little")
        daddr = int.from_bytes(bytes(f[30:34]), "little")
        ck = tcp.udp_csum(saddr, daddr, udplen, 17, umem.ctypes.data + u)
        if rng.random() < p_bad:
            ck ^= 0x0800
        umem[u + 6], umem[u + 7] = ck & 0xFF, ck >> 8


def verdict(tcp, umem, a, L, csum):
    """get_udp_payload (src/dqdk.c:185-207) + the checksum configuration, every
    decision a call into the reference's src/tcpip.  Returns (status, datalen, poff)."""
    base = umem.ctypes.data
    f = umem[a:]
    iph = base + a + 14
    if not tcp.ip4_audit(iph, (L - 14) & 0xFFFF):                           # :191
        return INV_IP, 0, 0
    ihl = int(f[14]) & 0xF
    if csum and not tcp.ip4_audit_checksum(iph):                            # ipv4.c:16 (commented upstream)
        return IP_CSUM, 0, 0
    hs = ihl * 4                                                            # :196
    udplen = ((int(f[16]) << 8 | int(f[17])) - hs) & 0xFFFFFFFF             # :197
    saddr = int.from_bytes(bytes(f[26:30]), "little")
    daddr = int.from_bytes(bytes(f[30:34]), "little")
    if not tcp.udp_audit(iph + hs, saddr, daddr, udplen & 0xFFFF):          # :200
        return INV_UDP, 0, 0
    if csum:  # udp_audit_checksum zeroes udp->check in place: a copy, same address parity
        scratch = np.zeros(14 + hs + 8 + 65536 + 64, np.uint8)
        sh = (a - scratch.ctypes.data) % 16
        n = min(len(scratch) - sh, umem.size - a)
        scratch[sh:sh + n] = umem[a:a + n]
        if not tcp.udp_audit_checksum(scratch.ctypes.data + sh + 14 + hs, saddr, daddr, udplen & 0xFFFF):
            return UDP_CSUM, 0, 0
    datalen = (udplen - 8) & 0xFFFFFFFF                                     # :205
    return (OK if datalen else EMPTY), datalen, 14 + hs + 8                 # process_frame :243-248


def frame_layout(rng, lens, slot_pad=64):
    """Frames packed one after another at random byte alignments."""
    addrs, off = [], 64
    for L in lens:
        off = (off + 15) // 16 * 16 + int(rng.integers(0, 16))
        addrs.append(off)
        off += max(L, 64) + slot_pad
    return np.array(addrs, np.uint64), (off + 65536 + 15) // 16 * 16


# ---- F3 ------------------------------------------------------------------------

def f3_events(t, tap, rng):
    """(a) single events: histogram_event's verdict + tristan_process over all."""
    ev = craft_events(rng, 6000, hot=0.02)
    scratch = np.zeros(O.HISTO_ENTRIES, np.uint32)
    verdicts = np.array([t.rt_histogram_event(scratch.ctypes.data, ev[i].ctypes.data) for i in range(len(ev))],
                        np.int8)
    tap.take()
    del scratch
    st = RefTristan(t, tap, MODE_ENERGYHISTO, 16 * len(ev))
    buf = np.ascontiguousarray(ev.reshape(-1))
    oob = st.process(buf.ctypes.data, buf.size)
    idx, cnt = st.sparse()
    assert oob == int((verdicts != 0).sum())
    return {"ev_events": ev, "ev_verdict": verdicts, "ev_hist_idx": idx, "ev_hist_cnt": cnt,
            "ev_totals": np.array([st.events.value, st.bytes.value, oob], np.uint64)}


F3_CASES = [
    # name, mode, payloadsz, frame lengths (choice), nframes, hot share
    ("ehisto_1500", MODE_ENERGYHISTO, 1458, [1500], 160, 0.0),
    ("ehisto_hot", MODE_ENERGYHISTO, 1458, [1500], 160, 0.6),
    ("listmode_3434", MODE_LISTMODE, 3392, [3434], 64, 0.0),
    ("ehisto_9000", MODE_ENERGYHISTO, 8958, [9000], 24, 0.0),
    ("payloadsz_gt_datalen", MODE_ENERGYHISTO, 2000, [1500, 700, 64, 43], 96, 0.0),  # E*16 runs past the datagram
    ("payloadsz_lt_datalen", MODE_ENERGYHISTO, 800, [1500], 64, 0.0),
    ("listwave_E1", MODE_LISTWAVE, 1458, [1500, 300], 96, 0.0),
    ("waveform_nohisto", MODE_WAVEFORM, 1458, [1500], 48, 0.0),
    ("E0", MODE_ENERGYHISTO, 8, [1500, 100], 48, 0.0),
    ("mixed_sizes", MODE_ENERGYHISTO, 1458, [1500, 9000, 600, 42, 41], 64, 0.1),
]


def f3_frames(t, tcp, tap, rng):
    out = {}
    for ci, (name, mode, psz, lens, nf, hot) in enumerate(F3_CASES):
        L = rng.choice(np.array(lens), size=nf)
        addrs, size = frame_layout(rng, L.tolist())
        umem = rng.integers(0, 256, size=size, dtype=np.uint8)  # bytes past a frame are random, as in a UMEM
        for a, l in zip(addrs.tolist(), L.tolist()):
            nev = max(1, (max(l, psz) + 15) // 16)
            put_frame(umem, a, int(l), craft_events(rng, nev, hot).reshape(-1), rng)
        st = RefTristan(t, tap, mode, psz)
        status = np.zeros(nf, np.uint8)
        datalen = np.zeros(nf, np.uint32)
        oob = np.zeros(nf, np.uint32)
        for i, (a, l) in enumerate(zip(addrs.tolist(), L.tolist())):
            s, dl, poff = verdict(tcp, umem, a, int(l), csum=False)
            status[i], datalen[i] = s, dl
            if s == OK:
                oob[i] = st.process(umem.ctypes.data + a + poff, dl)            # process_unbuffered_frame
        idx, cnt = st.sparse()
        desc = np.zeros(nf, O.DESC_DTYPE)
        desc["addr"], desc["len"] = addrs, L
        p = f"c{ci}_"
        out.update({p + "umem": umem, p + "desc": desc, p + "status": status, p + "datalen": datalen,
                    p + "oob": oob, p + "hist_idx": idx, p + "hist_cnt": cnt,
                    p + "cfg": np.array([mode, psz, t.rt_get_energy_events_count(mode, psz)], np.uint32),
                    p + "totals": np.array([st.events.value, st.bytes.value], np.uint64)})
        assert (status == OK).sum() > nf // 2, name
    out["case_names"] = np.array([c[0] for c in F3_CASES])
    return out


def f3_async(t, tap, rng):
    """(c) async_processor's tristan_process(buffer, len = strip_wfm ? 16 :
    payloadsz, burst = ret) over ring elements of payloadsz bytes."""
    out, rows = {}, []
    cases = [(MODE_LISTMODE, 3392, 0, [16, 16, 5, 1, 16, 3]), (MODE_LISTMODE, 3392, 1, [16, 2, 7, 16, 1]),
             (MODE_LISTWAVE, 1456, 1, [4, 16, 9, 1]), (MODE_ENERGYHISTO, 1456, 0, [1, 2, 3, 16]),
             (MODE_WAVEFORM, 1456, 0, [16, 8, 1])]
    for ci, (mode, psz, strip, bursts) in enumerate(cases):
        nel = sum(bursts)
        ring = craft_events(rng, nel * psz // 16, hot=0.05).reshape(nel, psz)
        st = RefTristan(t, tap, mode, psz)
        length = 16 if strip else psz                                        # src/tristan.c:343
        raw = tempfile.TemporaryFile()
        oob, e0 = [], 0
        for r in bursts:                                                     # :345-349 one fetch of `ret` elements
            buf = np.ascontiguousarray(ring[e0:e0 + r].reshape(-1))
            oob.append(st.process(buf.ctypes.data, length, r, raw_fd=raw.fileno()))
            e0 += r
        raw.seek(0)
        idx, cnt = st.sparse()
        p = f"a{ci}_"
        out.update({p + "ring": ring.reshape(-1), p + "bursts": np.array(bursts, np.uint32),
                    p + "cfg": np.array([mode, psz, strip], np.uint32), p + "raw": np.frombuffer(raw.read(), np.uint8),
                    p + "hist_idx": idx, p + "hist_cnt": cnt, p + "oob": np.array(oob, np.uint32),
                    p + "totals": np.array([st.events.value, st.bytes.value], np.uint64)})
        raw.close()
    out["async_cases"] = np.array(len(cases), np.uint32)
    return out


# ---- F4 ------------------------------------------------------------------------

def f4_batch(t, tcp, tap, rng, n=1024, psz=1458):
    L = rng.choice(np.array([1500, 1500, 1500, 1200, 800, 64, 42, 43, 41, 60]), size=n)
    # the first failing frame must sit deep in the batch for the abort case:
    # the first 600 frames are clean 1500-B frames with good checksums
    L[:600] = 1500
    addrs, size = frame_layout(rng, L.tolist(), slot_pad=16)
    umem = rng.integers(0, 256, size=size, dtype=np.uint8)
    faults = rng.random(n)
    faults[:600] = 0.5
    for i, (a, l) in enumerate(zip(addrs.tolist(), L.tolist())):
        tot_d = 2 if 0.02 < faults[i] < 0.03 else 0             # wrong tot_len -> invalid_ip
        ul_d = 2 if 0.03 < faults[i] < 0.04 else 0              # wrong udp.len -> invalid_udp
        put_frame(umem, a, int(l), craft_events(rng, (psz + 15) // 16, 0.05).reshape(-1), rng,
                  tot_delta=tot_d, ulen_delta=ul_d)  # ihl 5: ip4_audit_checksum is UB for ihl > 5 (F1 covers ihl)
        set_checksums(tcp, umem, a, rng, p_ip=1.0 if i < 600 else 0.97, p_bad=0.0 if i < 600 else 0.004)
    desc = np.zeros(n, O.DESC_DTYPE)
    desc["addr"], desc["len"] = addrs, L
    out = {"umem": umem, "desc": desc, "cfg": np.array([MODE_ENERGYHISTO, psz], np.uint32)}
    for csum in (0, 1):
        vs = [verdict(tcp, umem, int(a), int(l), bool(csum)) for a, l in zip(addrs.tolist(), L.tolist())]
        status = np.array([v[0] for v in vs], np.uint8)
        out[f"status_csum{csum}"] = status
        out[f"datalen_csum{csum}"] = np.array([v[1] for v in vs], np.uint32)
        for abort in (0, 1):
            st = RefTristan(t, tap, MODE_ENERGYHISTO, psz)
            c = dict(rcvd_frames=n, rcvd_pkts=0, rcvd_bytes=0, invalid_ip_pkts=0, invalid_udp_pkts=0,
                     failing_batches=0, oob_events=0, empty_pkts=0, first_abort_idx=n)   # :289 rcvd_frames += rcvd
            for i, (a, l) in enumerate(zip(addrs.tolist(), L.tolist())):
                s, dl, poff = vs[i]
                c["rcvd_pkts"] += 1                                          # :189
                if s in (INV_IP, IP_CSUM):
                    c["invalid_ip_pkts"] += 1                                # :192
                elif s in (INV_UDP, UDP_CSUM):
                    c["invalid_udp_pkts"] += 1                               # :201
                elif s == EMPTY:
                    c["empty_pkts"] += 1                                     # :248 -ENOBUFS
                else:
                    c["oob_events"] += st.process(umem.ctypes.data + a + poff, dl)
                    c["rcvd_bytes"] += dl                                    # :245-246
                if s != OK and c["first_abort_idx"] == n:
                    c["first_abort_idx"] = i
                    c["failing_batches"] = 1                                 # :317-319
                    if abort:
                        break                                                # :294-296
            c["total_events"], c["total_bytes"] = st.events.value, st.bytes.value
            idx, cnt = st.sparse()
            k = f"csum{csum}_abort{abort}_"
            out[k + "counters"] = np.array([c[f] for f in COUNTERS], np.uint64)
            out[k + "hist_idx"], out[k + "hist_cnt"] = idx, cnt
    assert 500 < out["csum1_abort1_counters"][COUNTERS.index("first_abort_idx")] < n - 100
    return out


COUNTERS = ["rcvd_frames", "rcvd_pkts", "rcvd_bytes", "invalid_ip_pkts", "invalid_udp_pkts", "failing_batches",
            "total_events", "total_bytes", "oob_events", "empty_pkts", "first_abort_idx"]


def main():
    if not (O.ref_available() and TRISTAN_LIB.exists()):
        sys.exit("oracle/_ref/lib{ref_tcpip,ref_tristan}.so missing: run `make -C oracle ref` where /root/reference exists")
    t = load_tristan()
    tcp = O.ref()
    tcp.udp_csum.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint8, C.c_void_p]
    rng = np.random.default_rng(SEED)
    tap = StdoutTap(t)
    try:
        f3 = {}
        f3.update(f3_events(t, tap, rng))
        f3.update(f3_frames(t, tcp, tap, rng))
        f3.update(f3_async(t, tap, rng))
        f4 = f4_batch(t, tcp, tap, rng)
    finally:
        tap.close()
    f4["counter_names"] = np.array(COUNTERS)
    np.savez_compressed(OUT / "f3_decode.npz", **f3)
    np.savez_compressed(OUT / "f4_batch.npz", **f4)
    print(f"f3_decode: {len(F3_CASES)} frame cases, {len(f3['ev_events'])} events; f4_batch: "
          f"{len(f4['desc'])} frames, abort at {f4['csum1_abort1_counters'][-1]}")


if __name__ == "__main__":
    main()
