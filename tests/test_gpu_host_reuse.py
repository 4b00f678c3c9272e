"""Host UMEM registration, then the same address reused by a new buffer.

VERDICT r5 item 1 / ADVICE r5: four -m gpu runs (r04b, r04d, r05h, r05ac)
stopped with hipErrorIllegalAddress at a test's FIRST pageable host-to-device
copy.  In r05ac the test before was `test_small_batches_single_launch[256-4]`:
a 1 MiB host UMEM (a numpy array: an mmap'd malloc chunk, data 16 B into
its first page) copied to the device by torch, registered by the host
drop-in (`dqdk_gpu_rx_batch` -> hipHostRegister), unregistered, the queue
destroyed, the array freed (munmap); the faulting copy then read a fresh
1,144,352-B array, which can sit at the same address.

This runs exactly that ordering with the address reuse forced (the second
buffer is mapped at the first one's address, MAP_FIXED_NOREPLACE), for the
same, a larger and a smaller second buffer, with and without the pageable
copy before the registration, and with the registration dropped by
unregister or by the queue's destroy.  The ownership rule it rests on is the
reference's: frames are valid until the descriptors are released
(src/dqdk.c:300) and the UMEM lives as long as its worker (src/dqdk.c:562,
freed at :476-479).
"""
import ctypes as C

import numpy as np
import pytest

import dqdk_amd as D
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

_libc = C.CDLL(None, use_errno=True)
_libc.mmap.restype = C.c_void_p
_libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
_libc.munmap.restype = C.c_int
_libc.munmap.argtypes = [C.c_void_p, C.c_size_t]
PROT_RW = 0x1 | 0x2
MAP_PRIVATE, MAP_ANONYMOUS, MAP_FIXED_NOREPLACE = 0x02, 0x20, 0x100000
OFF = 16  # glibc's mmap'd chunks hand out memory 16 B into the first page
PAGE = 4096


def _span(nbytes: int) -> int:
    return (OFF + nbytes + PAGE - 1) // PAGE * PAGE


def _map(nbytes: int, at: int = 0, span: int = 0) -> int:
    flags = MAP_PRIVATE | MAP_ANONYMOUS | (MAP_FIXED_NOREPLACE if at else 0)
    p = _libc.mmap(at or None, span or _span(nbytes), PROT_RW, flags, -1, 0)
    if p is None or p == C.c_void_p(-1).value:
        raise OSError(C.get_errno(), "mmap")
    return p


def _view(base: int, nbytes: int) -> np.ndarray:
    return np.frombuffer((C.c_uint8 * nbytes).from_address(base + OFF), dtype=np.uint8)


def _need_gpu():
    if not torch.cuda.is_available() or D.device_count() < 1:
        pytest.fail("GPU tests need a gfx950 device (none visible)")


@pytest.mark.parametrize("unreg", ["unregister", "destroy"])
@pytest.mark.parametrize("pre_copy", [True, False])
@pytest.mark.parametrize("second", [1_048_576, 1_144_352, 524_288])
def test_registered_umem_freed_then_address_reused_by_pageable_copy(second, pre_copy, unreg):
    _need_gpu()
    n = 256
    c = D.rx.synth_cfg(1500, 4096, faulty=True)
    first_len = (int(D._lib.lib().dqdk_synth_umem_size(C.byref(c), n)) + 15) // 16 * 16
    span = max(_span(first_len), _span(second))  # (room for the larger second buffer at the same address)
    a = _map(first_len, span=span)
    umem = _view(a, first_len)
    _, desc = D.synth_umem(n, 1500, 4096, faulty=True, first=7 * n, out=umem)
    if pre_copy:  # as compare() does before the host drop-in
        d = torch.from_numpy(umem).to("cuda:0")
        torch.cuda.synchronize()
        assert bool((d.cpu().numpy() == umem).all())
        del d
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_PREFILTER | D.F_HISTO_ATOMIC, port_start=5000, port_end=5000)
    q = D.RxQueue(0, cfg, 256)
    q.enable_timing(True)
    res, delta = q.process_batch(umem, desc)
    q.read_timing()
    ores, ocnt, _ = O.rx_batch(umem.copy(), desc, cfg.payloadsz, cfg.mode, cfg.flags, cfg.port_start, cfg.port_end)
    np.testing.assert_array_equal(res, ores)
    assert delta["rcvd_pkts"] == ocnt["rcvd_pkts"]
    if unreg == "unregister":
        q.unregister_umem(umem)
    q.close()  # raises on any failure of the queue's work or teardown
    torch.cuda.synchronize()
    del umem
    assert _libc.munmap(a, span) == 0

    b = _map(second, at=a)  # the freed buffer's address, forced
    assert b == a
    try:
        fresh = _view(b, second)
        fresh[:] = np.random.default_rng(second).integers(0, 256, second, dtype=np.uint8)
        d = torch.from_numpy(fresh).to("cuda:0")  # the copy r05ac faulted in
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d.cpu().numpy(), fresh)
        del d, fresh
    finally:
        torch.cuda.synchronize()
        _libc.munmap(b, _span(second))


def test_destroy_reports_success_and_device_free_checks():
    """destroy and device_free return their calls' results (0 here); a
    double destroy is impossible through the Python queue (closed once)."""
    _need_gpu()
    q = D.RxQueue(0, D.RxConfig(payloadsz=1458), 1024)
    q.close()
    q.close()  # no-op
    buf = D.DeviceBuffer(0, 1 << 20)
    buf.close()
    buf.close()  # no-op


@pytest.mark.parametrize("close_first", [0, 1])
def test_queues_sharing_one_umem_keep_their_mapping(close_first):
    """Several queues over one host UMEM (the drop-in harness's workers read
    one mlock'ed image, tests/c/fetch_xsk_harness.c; the reference gives each
    worker its own, src/dqdk.c:562): every queue registers it, but HIP keeps
    ONE registration per host range.  The library counts the
    queues holding it, so closing one queue leaves the others' zero-copy
    mapping in place (before round 6 the first destroy unregistered the range
    from under the others, and their own destroy then failed).  Three queues
    over one host UMEM: batches on each, one closed, the others run another
    batch each (results and counters vs the oracle), all close cleanly."""
    _need_gpu()
    n = 2048
    umem, desc = D.synth_umem(2 * n, 1500, 4096, faulty=True)
    d0, d1 = desc[:n].copy(), desc[n:].copy()
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM | D.F_HISTO_ATOMIC)
    qs = [D.RxQueue(0, cfg, n) for _ in range(3)]
    try:
        for q in qs:
            res, _ = q.process_batch(umem, d0)
        qs[close_first].close()  # raises if its teardown failed
        ores, ocnt, _ = O.rx_batch(umem.copy(), d1, cfg.payloadsz, cfg.mode, cfg.flags)
        for k, q in enumerate(qs):
            if k == close_first:
                continue
            res, delta = q.process_batch(umem, d1)
            np.testing.assert_array_equal(res, ores)
            assert delta["rcvd_pkts"] == ocnt["rcvd_pkts"] and delta["total_events"] == ocnt["total_events"]
        torch.cuda.synchronize()
    finally:
        for q in qs:
            q.close()


def test_view_inside_another_queues_umem_shares_its_registration():
    """A queue handed a view INSIDE a UMEM another queue registered (an
    interior address: HIP refuses a second, overlapping registration) shares
    that registration at the view's offset, and keeps it after the first
    queue closes: its batches before and after equal the oracle's."""
    _need_gpu()
    n = 1024
    umem, desc = D.synth_umem(2 * n, 1500, 4096, faulty=True)
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM | D.F_HISTO_ATOMIC)
    off = n * 4096  # the view starts at frame n
    view = umem[off:]
    dv = desc[n:].copy()
    dv["addr"] -= off
    ores, ocnt, _ = O.rx_batch(view.copy(), dv, cfg.payloadsz, cfg.mode, cfg.flags)
    qa, qb = D.RxQueue(0, cfg, 2 * n), D.RxQueue(0, cfg, n)
    try:
        qa.process_batch(umem, desc)
        res, delta = qb.process_batch(view, dv)
        np.testing.assert_array_equal(res, ores)
        qa.close()
        res, delta = qb.process_batch(view, dv)
        np.testing.assert_array_equal(res, ores)
        assert delta["rcvd_pkts"] == ocnt["rcvd_pkts"]
    finally:
        qa.close()
        qb.close()
