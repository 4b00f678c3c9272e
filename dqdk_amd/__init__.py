"""dqdk_amd -- MI355X-native receive hot path of DQDK (kit-ipe/dqdk).

Eth/IPv4/UDP parse + validate (src/tcpip via get_udp_payload, src/dqdk.c)
and TRISTAN energy-event decode + histogram (src/tristan.c) as gfx950 HIP
kernels behind the C ABI in include/dqdk_gpu.h.  Python is only the host
mirror of the reference's queue / frame-processor interface; every byte of
the receive path is processed by the HIP library.
"""
from . import _lib
from ._lib import (F_HISTO_ATOMIC, F_HISTO_EAGER, F_HISTO_UNFUSED, F_HISTO_PARTITIONED, F_BATCH_ABORT, F_CSUM, F_CSUM_WRITEBACK, F_NO_HISTO, F_PREFILTER, KEY_NONE,
                   MODE_ENERGYHISTO, MODE_LISTMODE, MODE_LISTWAVE, MODE_WAVEFORM, MODES,
                   RX_EMPTY, RX_FILTER_DROP, RX_FILTER_PASS, RX_INVALID_IP, RX_INVALID_IP_CSUM,
                   RX_INVALID_UDP, RX_INVALID_UDP_CSUM, RX_OK, DESC_DTYPE, RESULT_DTYPE, HISTO_ENTRIES,
                   DqdkError)
from .rx import DeviceBuffer, FrameProcessor, RxConfig, RxQueue, device_count, events_per_payload, histo_enabled, synth_umem, tristan_summary, SEED

__all__ = [
    "DeviceBuffer", "FrameProcessor", "RxConfig", "RxQueue", "device_count", "events_per_payload", "histo_enabled", "synth_umem", "tristan_summary", "SEED",
    "DESC_DTYPE", "RESULT_DTYPE", "HISTO_ENTRIES", "KEY_NONE", "MODES", "DqdkError",
    "F_CSUM", "F_BATCH_ABORT", "F_HISTO_ATOMIC", "F_HISTO_UNFUSED", "F_HISTO_PARTITIONED", "F_HISTO_EAGER", "F_PREFILTER", "F_NO_HISTO", "F_CSUM_WRITEBACK",
    "MODE_WAVEFORM", "MODE_LISTWAVE", "MODE_LISTMODE", "MODE_ENERGYHISTO",
    "RX_OK", "RX_INVALID_IP", "RX_INVALID_UDP", "RX_EMPTY", "RX_INVALID_IP_CSUM", "RX_INVALID_UDP_CSUM",
    "RX_FILTER_DROP", "RX_FILTER_PASS",
]
