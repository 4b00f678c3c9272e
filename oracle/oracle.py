"""ctypes wrapper of the test-only oracle libraries.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by dqdk_amd/.

  liboracle.so        the C restatement (dqdk_oracle.c)
  _ref/libref_tcpip.so the reference's own src/tcpip compiled verbatim
                      (present only where /root/reference existed at build)
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ORACLE_LIB = HERE / "liboracle.so"
REF_LIB = HERE / "_ref" / "libref_tcpip.so"

DESC_DTYPE = np.dtype([("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
RESULT_DTYPE = np.dtype([("datalen", "<u4"), ("status", "u1"), ("payload_off", "u1"), ("oob_events", "<u2")])
COUNTER_FIELDS = ("rcvd_frames", "rcvd_pkts", "rcvd_bytes", "invalid_ip_pkts", "invalid_udp_pkts",
                  "failing_batches", "total_events", "total_bytes", "oob_events", "empty_pkts",
                  "filtered_frames", "first_abort_idx")
HISTO_ENTRIES = 1512 * 6 * 65536


class Counters(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in COUNTER_FIELDS]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f in COUNTER_FIELDS}


class Cfg(C.Structure):
    _fields_ = [("payloadsz", C.c_uint32), ("mode", C.c_uint32), ("flags", C.c_uint32),
                ("port_start", C.c_uint16), ("port_end", C.c_uint16)]


_P = C.c_void_p
_U8 = C.c_uint8
_U16, _U32, _U64 = C.c_uint16, C.c_uint32, C.c_uint64

# (oracle name, reference name, restype, argtypes)
TCPIP_FUNCS = [
    ("or_from32to16", "from32to16", C.c_ushort, [C.c_uint]),
    ("or_from64to32", "from64to32", _U32, [_U64]),
    ("or_inet_csum", "inet_csum", C.c_uint, [_P, C.c_int]),
    ("or_inet_fast_csum", "inet_fast_csum", _U16, [_P, C.c_uint]),
    ("or_ip_fast_csum", "ip_fast_csum", _U16, [_P, C.c_uint]),
    ("or_csum_tcpudp_nofold", "csum_tcpudp_nofold", _U32, [_U32, _U32, _U32, _U8, _U32]),
    ("or_csum_fold", "csum_fold", _U16, [_U32]),
    ("or_csum_tcpudp_magic", "csum_tcpudp_magic", _U16, [_U32, _U32, _U32, _U8, _U32]),
    ("or_udp_csum", "udp_csum", _U16, [_U32, _U32, _U32, _U8, _P]),
    ("or_ip4_audit", "ip4_audit", C.c_int, [_P, _U16]),
    ("or_ip4_audit_checksum", "ip4_audit_checksum", C.c_int, [_P]),
    ("or_udp_audit", "udp_audit", C.c_int, [_P, _U32, _U32, _U16]),
]

_oracle = None
_ref = None


def oracle() -> C.CDLL:
    global _oracle
    if _oracle is None:
        if not ORACLE_LIB.exists():
            raise ImportError(f"{ORACLE_LIB} not built (make -C oracle)")
        h = C.CDLL(str(ORACLE_LIB))
        for name, _, res, args in TCPIP_FUNCS:
            f = getattr(h, name)
            f.restype, f.argtypes = res, args
        h.or_udp_audit_checksum.restype = C.c_int
        h.or_udp_audit_checksum.argtypes = [_P, _U32, _U32, _U16, C.c_int]
        h.or_prefilter.restype = C.c_int
        h.or_prefilter.argtypes = [_P, _U32, _U16, _U16]
        h.or_events_per_payload.restype = _U32
        h.or_events_per_payload.argtypes = [_U32, _U32]
        h.or_rx_batch.restype = C.c_int
        h.or_rx_batch.argtypes = [_P, _U64, _P, _U32, C.POINTER(Cfg), _P, C.POINTER(Counters), _P, _P]
        h.or_event_key.restype = _U32
        h.or_event_key.argtypes = [_P]
        h.or_async_process.restype = C.c_int
        h.or_async_process.argtypes = [_P, _U64, _P, _U32, C.POINTER(Cfg), C.c_int, C.POINTER(Counters), _P, _P, _U64,
                                       C.POINTER(_U64)]
        h.or_rx_batch_mt.restype = C.c_int
        h.or_rx_batch_mt.argtypes = [_P, _U64, _P, _U32, C.POINTER(Cfg), _P, C.POINTER(Counters), _P, _P, C.c_int]
        h.or_rx_batch_threads.restype = C.c_double
        h.or_rx_batch_threads.argtypes = [_P, _U64, _P, _U32, C.POINTER(Cfg), _P, C.POINTER(Counters), _P,
                                          C.c_int]
        _oracle = h
    return _oracle


def ref_available() -> bool:
    return REF_LIB.exists()


def ref() -> C.CDLL:
    """The reference's src/tcpip, compiled verbatim (oracle/Makefile `ref`)."""
    global _ref
    if _ref is None:
        h = C.CDLL(str(REF_LIB))
        for _, name, res, args in TCPIP_FUNCS:
            f = getattr(h, name)
            f.restype, f.argtypes = res, args
        h.udp_audit_checksum.restype = C.c_int
        h.udp_audit_checksum.argtypes = [_P, _U32, _U32, _U16]
        _ref = h
    return _ref


def events_per_payload(mode: int, payloadsz: int) -> int:
    return int(oracle().or_events_per_payload(mode, payloadsz))


def rx_batch(umem: np.ndarray, desc: np.ndarray, payloadsz: int, mode: int = 3, flags: int = 0,
             port_start: int = 0, port_end: int = 0, want_keys: bool = True, hist: np.ndarray | None = None,
             threads: int = 1):
    """Run one fetch_xsk batch through the C restatement.

    Returns (results, counters dict, keys[n*E] or None).  ``hist`` (u32,
    HISTO_ENTRIES) is accumulated in place when given.  threads > 1 splits
    the frames over host threads with identical outputs (or_rx_batch_mt).
    """
    assert umem.dtype == np.uint8 and umem.flags.c_contiguous
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    n = len(desc)
    E = events_per_payload(mode, payloadsz)
    res = np.zeros(n, dtype=RESULT_DTYPE)
    keys = np.full(n * E, 0xFFFFFFFF, dtype=np.uint32) if want_keys else None
    cnt = Counters()
    cfg = Cfg(payloadsz, mode, flags, port_start, port_end)
    if hist is not None:
        assert hist.dtype == np.uint32 and hist.size == HISTO_ENTRIES
    oracle().or_rx_batch_mt(umem.ctypes.data, umem.nbytes, desc.ctypes.data, n, C.byref(cfg), res.ctypes.data,
                            C.byref(cnt), hist.ctypes.data if hist is not None else None,
                            keys.ctypes.data if keys is not None else None, threads)
    return res, cnt.as_dict(), keys


def rx_batch_threads(umem: np.ndarray, desc: np.ndarray, payloadsz: int, mode: int = 3, flags: int = 0,
                     hist: np.ndarray | None = None, threads: int = 1):
    """CPU-baseline driver: returns (seconds, counters)."""
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    n = len(desc)
    res = np.zeros(n, dtype=RESULT_DTYPE)
    cnt = Counters()
    cfg = Cfg(payloadsz, mode, flags, 0, 0)
    sec = oracle().or_rx_batch_threads(umem.ctypes.data, umem.nbytes, desc.ctypes.data, n, C.byref(cfg),
                                       res.ctypes.data, C.byref(cnt),
                                       hist.ctypes.data if hist is not None else None, threads)
    return sec, cnt.as_dict()


def event_keys(events: np.ndarray) -> np.ndarray:
    """histogram_event's key per 16-B event (KEY_NONE when out of bounds)."""
    ev = np.ascontiguousarray(events, dtype=np.uint8).reshape(-1, 16)
    lib = oracle()
    base = ev.ctypes.data
    return np.array([lib.or_event_key(base + 16 * i) for i in range(len(ev))], dtype=np.uint32)


def async_process(ring: np.ndarray, bursts, payloadsz: int, mode: int, strip_wfm: bool, flags: int = 0,
                  hist: np.ndarray | None = None):
    """async_processor's tristan_process(buffer, len, ret) per burst.
    Returns (counters dict, raw bytes)."""
    ring = np.ascontiguousarray(ring, dtype=np.uint8)
    b = np.ascontiguousarray(bursts, dtype=np.uint32)
    nelem = ring.size // payloadsz if payloadsz else 0
    cnt = Counters()
    cfg = Cfg(payloadsz, mode, flags, 0, 0)
    cap = int(b.astype(np.uint64).sum()) * max(payloadsz, 16)
    raw = np.zeros(max(cap, 1), np.uint8)
    tot = C.c_uint64()
    rc = oracle().or_async_process(ring.ctypes.data, nelem, b.ctypes.data, len(b), C.byref(cfg), int(strip_wfm),
                                   C.byref(cnt), hist.ctypes.data if hist is not None else None, raw.ctypes.data,
                                   raw.size, C.byref(tot))
    assert rc == 0
    return cnt.as_dict(), raw[:tot.value].tobytes()


def sparse_histogram(keys: np.ndarray, res: np.ndarray, E: int, limit: int | None = None):
    """(unique keys, counts) of the events the histogram receives: keys of
    OK frames (index < limit), OOB records excluded."""
    n = len(res)
    if limit is None:
        limit = n
    ok = (res["status"] == 0) & (np.arange(n) < limit)
    k = keys.reshape(n, E)[ok].ravel() if E else np.zeros(0, np.uint32)
    k = k[k != 0xFFFFFFFF]
    u, c = np.unique(k, return_counts=True)
    return u.astype(np.uint32), c.astype(np.uint64)
