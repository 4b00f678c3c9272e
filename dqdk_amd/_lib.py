"""ctypes binding of libdqdk_gpu.so (the C ABI in include/dqdk_gpu.h).

The library is loaded from dqdk_amd/lib/ (built in-tree by
``__graft_entry__.build()`` / ``python -m dqdk_amd._build``).  There is no
Python or CPU implementation of the receive path behind this module: if the
library is missing, importing the bindings raises, and without a gfx950
device every queue constructor fails with ``-ENODEV``.
"""
from __future__ import annotations

import ctypes as C
import errno
import os
from pathlib import Path

import numpy as np

LIB_PATH = Path(os.environ.get("DQDK_GPU_LIB", Path(__file__).resolve().parent / "lib" / "libdqdk_gpu.so"))

# ---- C structs (include/dqdk_gpu.h) ---------------------------------------


class Desc(C.Structure):
    _fields_ = [("addr", C.c_uint64), ("len", C.c_uint32), ("options", C.c_uint32)]


class RxResult(C.Structure):
    _fields_ = [("datalen", C.c_uint32), ("status", C.c_uint8), ("payload_off", C.c_uint8),
                ("oob_events", C.c_uint16)]


COUNTER_FIELDS = ("rcvd_frames", "rcvd_pkts", "rcvd_bytes", "invalid_ip_pkts", "invalid_udp_pkts",
                  "failing_batches", "total_events", "total_bytes", "oob_events", "empty_pkts",
                  "filtered_frames", "first_abort_idx")


class Counters(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in COUNTER_FIELDS]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f in COUNTER_FIELDS}


class Cfg(C.Structure):
    _fields_ = [("payloadsz", C.c_uint32), ("mode", C.c_uint32), ("flags", C.c_uint32),
                ("port_start", C.c_uint16), ("port_end", C.c_uint16)]


class FpCfg(C.Structure):
    _fields_ = [("cfg", Cfg), ("slot_payloads", C.c_uint32), ("nslots", C.c_uint32), ("device_first", C.c_int),
                ("ndevices", C.c_int)]


class SynthCfg(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("queue", C.c_uint32), ("frame_len", C.c_uint32),
                ("stride", C.c_uint32), ("faulty", C.c_uint32)]


# numpy views of the same layouts
DESC_DTYPE = np.dtype([("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
RESULT_DTYPE = np.dtype([("datalen", "<u4"), ("status", "u1"), ("payload_off", "u1"), ("oob_events", "<u2")])
assert DESC_DTYPE.itemsize == C.sizeof(Desc) == 16
assert RESULT_DTYPE.itemsize == C.sizeof(RxResult) == 8

# enums
RX_OK, RX_INVALID_IP, RX_INVALID_UDP, RX_EMPTY, RX_INVALID_IP_CSUM, RX_INVALID_UDP_CSUM, \
    RX_FILTER_DROP, RX_FILTER_PASS = range(8)
MODE_WAVEFORM, MODE_LISTWAVE, MODE_LISTMODE, MODE_ENERGYHISTO = range(4)
MODES = {"waveform": MODE_WAVEFORM, "listwave": MODE_LISTWAVE, "listmode": MODE_LISTMODE,
         "energy-histo": MODE_ENERGYHISTO}  # src/tristan.c:13-18
F_CSUM, F_BATCH_ABORT, F_PREFILTER, F_NO_HISTO, F_CSUM_WRITEBACK = 1, 2, 4, 8, 16
F_HISTO_ATOMIC, F_HISTO_PARTITIONED, F_HISTO_EAGER, F_HISTO_UNFUSED = 32, 64, 128, 256
KEY_NONE = 0xFFFFFFFF
TIMING_STAGES = 10
HISTO_CHANNELS, HISTO_HISTS, HISTO_BINS = 1512, 6, 65536
HISTO_ENTRIES = HISTO_CHANNELS * HISTO_HISTS * HISTO_BINS

# every entry point declared in include/dqdk_gpu.h: name -> (restype, argtypes)
_P = C.c_void_p
SIGNATURES = {
    "dqdk_gpu_abi_version": (C.c_int, []),
    "dqdk_gpu_device_count": (C.c_int, []),
    "dqdk_gpu_queue_create": (C.c_int, [C.c_int, C.POINTER(Cfg), C.c_uint32, C.POINTER(_P)]),
    "dqdk_gpu_queue_destroy": (C.c_int, [_P]),
    "dqdk_gpu_queue_set_stream": (C.c_int, [_P, _P]),
    "dqdk_gpu_queue_stream": (_P, [_P]),
    "dqdk_gpu_queue_own_stream": (_P, [_P]),
    "dqdk_gpu_rx_batch_device": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint32, _P, _P]),
    "dqdk_gpu_queue_sync": (C.c_int, [_P]),
    "dqdk_gpu_umem_register": (C.c_int, [_P, _P, C.c_uint64]),
    "dqdk_gpu_umem_unregister": (C.c_int, [_P, _P]),
    "dqdk_gpu_rx_batch": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint32, _P, C.POINTER(Counters)]),
    "dqdk_gpu_counters_get": (C.c_int, [_P, C.POINTER(Counters)]),
    "dqdk_gpu_counters_reset": (C.c_int, [_P]),
    "dqdk_gpu_histogram_get": (C.c_int, [_P, _P]),
    "dqdk_gpu_histogram_accumulate": (C.c_int, [_P, _P]),
    "dqdk_gpu_histogram_reset": (C.c_int, [_P]),
    "dqdk_gpu_histogram_device_ptr": (_P, [_P]),
    "dqdk_gpu_fp_init": (C.c_int, [C.POINTER(FpCfg)]),
    "dqdk_gpu_fp_bind": (C.c_int, [_P, C.c_int, _P, C.c_uint64]),
    "dqdk_gpu_frame_processor": (C.c_int, [_P, _P, C.c_uint32]),
    "dqdk_gpu_fp_flush": (C.c_int, [_P]),
    "dqdk_gpu_fp_fini": (C.c_int, [_P, C.c_int, C.POINTER(Counters)]),
    "dqdk_gpu_raw_compact_device": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint32, _P, _P, C.c_uint64,
                                              C.POINTER(C.c_uint64)]),
    "dqdk_gpu_queue_set_raw_fd": (C.c_int, [_P, C.c_int]),
    "dqdk_gpu_queue_set_raw_deferred": (C.c_int, [_P, C.c_int]),
    "dqdk_gpu_async_process_device": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint32, C.c_int, _P, C.c_uint64,
                                                C.POINTER(C.c_uint64)]),
    "dqdk_gpu_histogram_copy": (C.c_int, [_P, _P]),
    "dqdk_gpu_histogram_add": (C.c_int, [_P, _P]),
    "dqdk_gpu_histogram_nonzero": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "dqdk_gpu_histogram_write_csv": (C.c_int, [_P, C.c_int, C.POINTER(C.c_uint64)]),
    "dqdk_gpu_tristan_summary": (C.c_int, [C.POINTER(C.POINTER(Counters)), C.c_int, C.POINTER(C.c_uint64),
                                           C.c_char_p, C.c_char_p, C.c_uint64]),
    "dqdk_gpu_membench_read": (C.c_int, [_P, C.c_uint64, _P, C.c_int, C.POINTER(C.c_double)]),
    "dqdk_gpu_membench_atomic": (C.c_int, [_P, C.c_uint64, _P, C.c_uint64, _P, C.c_int, C.POINTER(C.c_double)]),
    "dqdk_gpu_device_alloc": (C.c_int, [C.c_int, C.c_uint64, C.POINTER(C.c_void_p)]),
    "dqdk_gpu_device_free": (C.c_int, [C.c_int, _P]),
    "dqdk_gpu_membench_frames": (C.c_int, [_P, C.c_uint64, C.c_uint32, C.c_uint32, _P, C.c_uint32, C.c_int, _P,
                                           C.c_int, C.POINTER(C.c_double)]),
    "dqdk_gpu_timing_enable": (C.c_int, [_P, C.c_int]),
    "dqdk_gpu_timing_stages": (C.c_int, [_P, C.c_uint32]),
    "dqdk_gpu_histogram_flush": (C.c_int, [_P]),
    "dqdk_gpu_histogram_batches_per_pass": (C.c_int, [_P]),
    "dqdk_gpu_timing_read": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.c_int]),
    "dqdk_gpu_queue_staging_probe": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_float), C.c_int]),
    "dqdk_gpu_timing_stage_name": (C.c_char_p, [C.c_int]),
    "dqdk_gpu_last_error": (C.c_char_p, []),
    "dqdk_synth_umem_size": (C.c_uint64, [C.POINTER(SynthCfg), C.c_uint32]),
    "dqdk_synth_frame_len": (C.c_uint32, [C.POINTER(SynthCfg), C.c_uint64]),
    "dqdk_synth_frames": (C.c_int, [C.POINTER(SynthCfg), C.c_uint64, C.c_uint32, _P, C.c_uint64, _P, C.c_int]),
}

_lib = None


def lib() -> C.CDLL:
    """Load libdqdk_gpu.so; raise loudly when it is missing (no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(f"{LIB_PATH} not built: run `python -m dqdk_amd._build` "
                              "(the receive path has no non-HIP implementation)")
        h = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


class DqdkError(OSError):
    pass


def check(rc: int, what: str) -> int:
    if rc < 0:
        msg = lib().dqdk_gpu_last_error().decode(errors="replace")
        raise DqdkError(-rc, f"{what}: {errno.errorcode.get(-rc, rc)} ({msg})")
    return rc
