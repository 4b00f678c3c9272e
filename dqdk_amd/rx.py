"""Host-side mirror of DQDK's receive-path plugin interface over the GPU engine.

Reference interface being mirrored (src/dqdk.h, src/tristan.c):

* ``dqdk_ctx_init(..., payloadsz, ..., proc, ...)`` + ``tristan_init`` pick the
  mode and the frame processor -> :class:`RxQueue` (one per RX queue / GPU).
* ``fetch_xsk`` (src/dqdk.c:252-322) hands a peeked batch of ``xdp_desc`` to
  ``process_frame`` one by one -> :meth:`RxQueue.process_batch` hands the whole
  batch to ``dqdk_gpu_rx_batch`` (host UMEM) and :meth:`RxQueue.process_device`
  to ``dqdk_gpu_rx_batch_device`` (device-resident UMEM).
* ``dqdk_stats_t`` / ``tristan_t`` counters -> :meth:`RxQueue.counters`.
* ``tristan_t::histo`` -> :meth:`RxQueue.histogram`.

Return conventions follow the reference: failures raise :class:`DqdkError`
carrying the negative errno the C ABI returned.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L


def events_per_payload(mode: int, payloadsz: int) -> int:
    """get_energy_events_count, src/tristan.c:72-85."""
    if mode in (L.MODE_LISTMODE, L.MODE_ENERGYHISTO):
        return payloadsz // 16
    if mode in (L.MODE_LISTWAVE, L.MODE_WAVEFORM):
        return 1
    return 0


def histo_enabled(mode: int, flags: int) -> bool:
    """is_store_histo, src/tristan.c:65-70."""
    return not (flags & L.F_NO_HISTO) and mode in (L.MODE_LISTWAVE, L.MODE_LISTMODE, L.MODE_ENERGYHISTO)


@dataclass
class RxConfig:
    payloadsz: int = 3392                 # -s default (src/tristan.c:419)
    mode: int = L.MODE_ENERGYHISTO
    flags: int = 0
    port_start: int = 0
    port_end: int = 0

    def to_c(self) -> L.Cfg:
        return L.Cfg(self.payloadsz, self.mode, self.flags, self.port_start, self.port_end)

    @property
    def events(self) -> int:
        return events_per_payload(self.mode, self.payloadsz)


def device_count() -> int:
    return L.lib().dqdk_gpu_device_count()


class RxQueue:
    """One RX queue bound to one GPU (the reference's dqdk_worker_t)."""

    def __init__(self, device: int, cfg: RxConfig, max_batch: int):
        self.cfg = cfg
        self.device = device
        self.max_batch = max_batch
        h = C.c_void_p()
        L.check(L.lib().dqdk_gpu_queue_create(device, C.byref(cfg.to_c()), max_batch, C.byref(h)),
                "dqdk_gpu_queue_create")
        self._h = h
        # host UMEMs the queue holds registered, by address: kept alive until
        # unregistered (a freed registered buffer would leave its registration
        # to a new buffer at the same address)
        self._pinned = {}

    # -- lifecycle ---------------------------------------------------------
    def close(self) -> None:
        """Destroy the queue; raises DqdkError when its last work or its
        teardown failed (a device fault is reported here, by the queue that
        ran the work, not by a later call)."""
        if getattr(self, "_h", None):
            rc = L.lib().dqdk_gpu_queue_destroy(self._h)
            self._h = None
            self._pinned = {}
            L.check(rc, "dqdk_gpu_queue_destroy")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        if exc[0] is None:
            self.close()
        else:  # the body's exception is the one reported
            try:
                self.close()
            except L.DqdkError:
                pass

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_stream(self, hip_stream_ptr: int) -> None:
        """Order the queue's work on this hipStream_t (0 = the legacy default
        stream, which is what torch's default stream reports)."""
        L.check(L.lib().dqdk_gpu_queue_set_stream(self._h, hip_stream_ptr), "set_stream")

    def use_own_stream(self) -> None:
        L.check(L.lib().dqdk_gpu_queue_set_stream(self._h, L.lib().dqdk_gpu_queue_own_stream(self._h)),
                "set_stream")

    def sync(self) -> None:
        L.check(L.lib().dqdk_gpu_queue_sync(self._h), "queue_sync")

    # -- batches -----------------------------------------------------------
    def process_device(self, umem_ptr: int, umem_size: int, desc_ptr: int, n: int,
                       results_ptr: int, keys_ptr: int | None = None) -> None:
        """Async device-resident batch: all pointers are device pointers."""
        L.check(L.lib().dqdk_gpu_rx_batch_device(self._h, umem_ptr, umem_size, desc_ptr, n,
                                                 results_ptr, keys_ptr or None),
                "dqdk_gpu_rx_batch_device")

    def process_batch(self, umem: np.ndarray, desc: np.ndarray) -> tuple[np.ndarray, dict]:
        """Host drop-in for the loop at src/dqdk.c:291-298 (synchronous).

        ``umem`` is the host UMEM (uint8, registered/pinned on first use),
        ``desc`` a DESC_DTYPE array.  Returns (per-frame results, counter delta).
        """
        assert umem.dtype == np.uint8 and umem.flags.c_contiguous
        desc = np.ascontiguousarray(desc, dtype=L.DESC_DTYPE)
        n = len(desc)
        res = np.zeros(n, dtype=L.RESULT_DTYPE)
        delta = L.Counters()
        self._keep(umem)  # (registered on first use: held while registered)
        L.check(L.lib().dqdk_gpu_rx_batch(self._h, umem.ctypes.data, umem.nbytes, desc.ctypes.data, n,
                                          res.ctypes.data, C.byref(delta)), "dqdk_gpu_rx_batch")
        return res, delta.as_dict()

    def raw_compact_device(self, umem_ptr: int, umem_size: int, desc_ptr: int, n: int, results_ptr: int,
                           out_ptr: int | None = None, out_cap: int = 0, sync: bool = True) -> int | None:
        """Gather the batch's raw payload stream (src/tristan.c:318-324) on the GPU."""
        tot = C.c_uint64()
        L.check(L.lib().dqdk_gpu_raw_compact_device(self._h, umem_ptr, umem_size, desc_ptr, n, results_ptr,
                                                    out_ptr or None, out_cap, C.byref(tot) if sync else None),
                "raw_compact_device")
        return int(tot.value) if sync else None

    def async_process_device(self, ring_ptr: int, nelem: int, bursts, strip_wfm: bool = False,
                             out_ptr: int | None = None, out_cap: int = 0) -> int:
        """The async consumer's tristan_process(buffer, len, ret) per burst
        (async_processor, src/tristan.c:332-375) over a device ring of
        payloadsz-byte elements; returns the raw stream length."""
        b = np.ascontiguousarray(bursts, dtype=np.uint32)
        tot = C.c_uint64()
        L.check(L.lib().dqdk_gpu_async_process_device(self._h, ring_ptr, nelem, b.ctypes.data, len(b), int(strip_wfm),
                                                      out_ptr or None, out_cap, C.byref(tot)),
                "async_process_device")
        return int(tot.value)

    def set_raw_fd(self, fd: int, deferred: bool | None = None) -> None:
        """Append every host batch's raw payload stream to fd (-1 = off).
        deferred=True: each batch's write() happens during the next call (or
        at sync / set_raw_fd / close), overlapped with that batch's kernels;
        default: written before process_batch returns (tristan.c:318-324)."""
        if deferred is not None:
            L.check(L.lib().dqdk_gpu_queue_set_raw_deferred(self._h, int(deferred)), "set_raw_deferred")
        L.check(L.lib().dqdk_gpu_queue_set_raw_fd(self._h, fd), "set_raw_fd")

    def register_umem(self, umem: np.ndarray) -> None:
        L.check(L.lib().dqdk_gpu_umem_register(self._h, umem.ctypes.data, umem.nbytes), "umem_register")
        self._keep(umem)

    def _keep(self, umem: np.ndarray) -> None:
        """Hold a buffer the C side registers for it (dqdk_gpu_umem_register's
        rules): nothing when a held registration already covers it (a view
        inside a registered UMEM creates none), else the buffer, replacing a
        smaller one at the same address (the C side replaces that
        registration too).  Held until unregistered or the queue closes."""
        a, n = umem.ctypes.data, umem.nbytes
        for base, buf in self._pinned.items():
            if base <= a and a + n <= base + buf.nbytes:
                return
        self._pinned[a] = umem

    def unregister_umem(self, umem: np.ndarray) -> None:
        L.check(L.lib().dqdk_gpu_umem_unregister(self._h, umem.ctypes.data), "umem_unregister")
        self._pinned.pop(umem.ctypes.data, None)

    # -- egress ------------------------------------------------------------
    def counters(self) -> dict:
        c = L.Counters()
        L.check(L.lib().dqdk_gpu_counters_get(self._h, C.byref(c)), "counters_get")
        return c.as_dict()

    def reset_counters(self) -> None:
        L.check(L.lib().dqdk_gpu_counters_reset(self._h), "counters_reset")

    def histogram(self, out: np.ndarray | None = None) -> np.ndarray:
        """The queue's u32[1512*6*65536] histogram (src/tristan.h:71-77)."""
        if out is None:
            out = np.empty(L.HISTO_ENTRIES, dtype=np.uint32)
        assert out.dtype == np.uint32 and out.size == L.HISTO_ENTRIES and out.flags.c_contiguous
        L.check(L.lib().dqdk_gpu_histogram_get(self._h, out.ctypes.data), "histogram_get")
        return out

    def load_histogram(self, table: np.ndarray) -> None:
        """Replace the queue's table with a host u32 table (reset, then add a
        device copy of it): dqdk_amd.multi's host-side merge."""
        import torch

        assert table.dtype == np.uint32 and table.size == L.HISTO_ENTRIES
        buf = torch.from_numpy(np.ascontiguousarray(table).view(np.int32)).to(torch.device("cuda", self.device))
        self.reset_histogram()
        self.histogram_add(buf.data_ptr())
        self.sync()
        del buf

    def accumulate_histogram(self, into: np.ndarray) -> None:
        assert into.dtype == np.uint32 and into.size == L.HISTO_ENTRIES and into.flags.c_contiguous
        L.check(L.lib().dqdk_gpu_histogram_accumulate(self._h, into.ctypes.data), "histogram_accumulate")

    def flush_histogram(self) -> None:
        """Run the pending slice pass of staged partitioned batches (async)."""
        L.check(L.lib().dqdk_gpu_histogram_flush(self._h), "histogram_flush")

    def histogram_batches_per_pass(self) -> int:
        return int(L.lib().dqdk_gpu_histogram_batches_per_pass(self._h))

    def reset_histogram(self) -> None:
        L.check(L.lib().dqdk_gpu_histogram_reset(self._h), "histogram_reset")

    def histogram_device_ptr(self) -> int | None:
        return L.lib().dqdk_gpu_histogram_device_ptr(self._h)

    def histogram_copy(self, d_dst_ptr: int) -> None:
        """Async device copy of the table into a caller buffer (e.g. an RCCL reduce buffer)."""
        L.check(L.lib().dqdk_gpu_histogram_copy(self._h, d_dst_ptr), "histogram_copy")

    def histogram_add(self, d_src_ptr: int) -> None:
        """Async table += caller device buffer (u32 wrap): the cross-queue merge."""
        L.check(L.lib().dqdk_gpu_histogram_add(self._h, d_src_ptr), "histogram_add")

    def histogram_nonzero(self) -> int:
        c = C.c_uint64()
        L.check(L.lib().dqdk_gpu_histogram_nonzero(self._h, C.byref(c)), "histogram_nonzero")
        return int(c.value)

    def write_histogram_csv(self, fd: int) -> int:
        """The histogram file of tristan_fini (src/tristan.c:197-216), formatted on the GPU."""
        n = C.c_uint64()
        L.check(L.lib().dqdk_gpu_histogram_write_csv(self._h, fd, C.byref(n)), "histogram_write_csv")
        return int(n.value)

    def staging_probe(self) -> dict:
        """The staging placement probe's outcome: the kept candidate piece
        buffer (-1: undecided, -2: off) and each candidate's best decode ns per
        frame (include/dqdk_gpu.h)."""
        ch = C.c_int(-1)
        ns = (C.c_float * 16)()
        k = L.check(L.lib().dqdk_gpu_queue_staging_probe(self._h, C.byref(ch), ns, 16), "staging_probe")
        return {"chosen": ch.value, "ns_per_frame": [round(ns[i], 4) for i in range(min(k, 16))]}

    # -- stage timing --------------------------------------------------------
    def enable_timing(self, on: bool = True) -> None:
        L.check(L.lib().dqdk_gpu_timing_enable(self._h, int(on)), "timing_enable")

    def timing_stages(self, names=None) -> None:
        """Time only the named stages (None: all)."""
        mask = 0xFFFFFFFF
        if names is not None:
            all_names = [(L.lib().dqdk_gpu_timing_stage_name(k) or b"").decode() for k in range(L.TIMING_STAGES)]
            mask = sum(1 << all_names.index(n) for n in names)
        L.check(L.lib().dqdk_gpu_timing_stages(self._h, mask), "timing_stages")

    def read_timing(self) -> dict:
        """Per-kernel HIP-event totals since the last read: {kernel: {ms, launches}}."""
        ns = L.TIMING_STAGES
        ms = (C.c_double * ns)()
        cnt = (C.c_uint64 * ns)()
        L.check(L.lib().dqdk_gpu_timing_read(self._h, ms, cnt, ns), "timing_read")
        names = [L.lib().dqdk_gpu_timing_stage_name(k) for k in range(ns)]
        return {nm.decode(): {"ms": ms[k], "launches": int(cnt[k])} for k, nm in enumerate(names)
                if nm and not nm.startswith(b"(")}  # "(unused)" stage slots


class FrameProcessor:
    """DQDK's frame-processor plugin on the GPU: ``dqdk_gpu_frame_processor``
    is a ``dqdk_frame_processor_t`` (src/dqdk.h:84-85) that the unmodified
    receive loop calls once per valid payload (process_frame,
    src/dqdk.c:231-250), standing in for process_unbuffered_frame
    (src/tristan.c:377-381).  Workers are any distinct addresses (the
    reference's dqdk_worker_t pointers); one GPU queue per worker.

    ``fn_ptr`` is the C function pointer to register as ``proc`` in
    dqdk_ctx_init (src/tristan.c:589-590); ``__call__`` calls it from Python.
    """

    def __init__(self, cfg: RxConfig, slot_payloads: int = 0, nslots: int = 0, device_first: int = 0,
                 ndevices: int = 0):
        self.cfg = cfg
        c = L.FpCfg(cfg.to_c(), slot_payloads, nslots, device_first, ndevices)
        L.check(L.lib().dqdk_gpu_fp_init(C.byref(c)), "dqdk_gpu_fp_init")
        self._open = True

    @property
    def fn_ptr(self) -> int:
        return C.cast(L.lib().dqdk_gpu_frame_processor, C.c_void_p).value

    def bind(self, worker: int, device: int = -1, umem: np.ndarray | None = None) -> None:
        """Give the worker its GPU (and UMEM bound) before its first frame."""
        L.check(L.lib().dqdk_gpu_fp_bind(worker, device, umem.ctypes.data if umem is not None else None,
                                         umem.nbytes if umem is not None else 0), "dqdk_gpu_fp_bind")

    def __call__(self, worker: int, data_ptr: int, datalen: int) -> int:
        """One tristan_process(data, datalen, 1) call; returns 0 or -errno like the reference."""
        return L.lib().dqdk_gpu_frame_processor(worker, data_ptr, datalen)

    def flush(self, worker: int) -> None:
        L.check(L.lib().dqdk_gpu_fp_flush(worker), "dqdk_gpu_fp_flush")

    def fini(self, host_hist: np.ndarray | None = None, csv_fd: int = -1) -> dict:
        """Drain every worker; add their tables into host_hist (tristan_t::histo),
        write the merged CSV to csv_fd; return the summed counters."""
        if host_hist is not None:
            assert host_hist.dtype == np.uint32 and host_hist.size == L.HISTO_ENTRIES and host_hist.flags.c_contiguous
        tot = L.Counters()
        self._open = False
        L.check(L.lib().dqdk_gpu_fp_fini(host_hist.ctypes.data if host_hist is not None else None, csv_fd,
                                         C.byref(tot)), "dqdk_gpu_fp_fini")
        return tot.as_dict()

    def __del__(self):
        if getattr(self, "_open", False):
            try:
                L.lib().dqdk_gpu_fp_fini(None, -1, None)
            except Exception:
                pass


def tristan_summary(counters: list[dict], runtime_ns: list[int] | None = None, directory: str = "") -> str:
    """tristan_fini's controller status line (src/tristan.c:171-189) via the C ABI."""
    objs = [L.Counters(**{f: int(c.get(f, 0)) for f in L.COUNTER_FIELDS}) for c in counters]
    arr = (C.POINTER(L.Counters) * max(len(objs), 1))(*[C.pointer(o) for o in objs])
    rt = (C.c_uint64 * max(len(objs), 1))(*(runtime_ns or [0] * len(objs)))
    buf = C.create_string_buffer(8192)  # buffersz in tristan_fini
    L.check(L.lib().dqdk_gpu_tristan_summary(arr, len(objs), rt, directory.encode(), buf, 8192), "tristan_summary")
    return buf.value.decode()


class DeviceBuffer:
    """HBM from dqdk_gpu_device_alloc (physically contiguous where the driver
    allows): a device UMEM image or frame staging slot.  ``tensor`` is a torch
    uint8 view of it (torch imported lazily; the buffer outlives the view only
    until close())."""

    def __init__(self, device: int, size: int):
        p = C.c_void_p()
        rc = L.lib().dqdk_gpu_device_alloc(device, size, C.byref(p))
        L.check(min(rc, 0), "device_alloc")
        self.device, self.size, self.ptr = device, size, int(p.value)
        self.contiguous = rc == 0

    @property
    def tensor(self):
        import torch

        ptr, size = self.ptr, self.size

        class _View:  # __cuda_array_interface__ of the raw allocation
            __cuda_array_interface__ = {"shape": (size,), "typestr": "|u1", "data": (ptr, False), "version": 3,
                                        "strides": None}
        return torch.as_tensor(_View(), device=torch.device("cuda", self.device))

    def close(self) -> None:
        if self.ptr:
            rc = L.lib().dqdk_gpu_device_free(self.device, self.ptr)
            self.ptr = 0
            L.check(rc, "dqdk_gpu_device_free")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ---- synthetic UMEM (bench / test input) ------------------------------------

SEED = 20261015


SYNTH_PEAKED = 2  # dqdk_synth_cfg_t.faulty bit 1: skewed spectrum (hot bins)


def synth_cfg(frame_len: int, stride: int, queue: int = 0, faulty: bool = False, seed: int = SEED,
              peaked: bool = False) -> L.SynthCfg:
    return L.SynthCfg(seed, queue, frame_len, stride, int(bool(faulty)) | (SYNTH_PEAKED if peaked else 0))


def synth_umem(n: int, frame_len: int, stride: int, queue: int = 0, faulty: bool = False, seed: int = SEED,
               first: int = 0, threads: int = 8, pad: int = 0, out: np.ndarray | None = None, peaked: bool = False
               ) -> tuple[np.ndarray, np.ndarray]:
    """Fill a host UMEM image with n synthetic frames; returns (umem u8, desc).
    faulty: header/checksum/event faults; peaked: 3/8 of the events on four hot bins."""
    c = synth_cfg(frame_len, stride, queue, faulty, seed, peaked)
    size = int(L.lib().dqdk_synth_umem_size(C.byref(c), n)) + pad
    size = (size + 15) // 16 * 16
    umem = out if out is not None else np.empty(size, dtype=np.uint8)
    assert umem.nbytes >= size
    desc = np.zeros(n, dtype=L.DESC_DTYPE)
    L.check(L.lib().dqdk_synth_frames(C.byref(c), first, n, umem.ctypes.data, umem.nbytes, desc.ctypes.data,
                                      threads), "dqdk_synth_frames")
    return umem, desc
