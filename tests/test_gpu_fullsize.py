"""The benchmarked form at the benchmarked sizes, against the oracle.

bench.py runs histogram batches with NO record buffer: partitioned batches
then take rx_decode_fused (keys bucketed in the decode's LDS stages and
appended to per-block pieces, the decode taking back frames that fail the
UDP checksum afterwards, rx_part2 gathering the pieces), at 1M x 1500 B and
1M x 9000 B (BASELINE north star) and 256K x 9000 B (configs[2]).  Here the
same calls run on the same synthetic UMEM and every per-frame result, every
counter and the WHOLE 2.38 GB table are compared with the oracle
(or_rx_batch_mt: the C restatement on host threads, identical outputs).

At 1M frames each of the 256 persistent decode blocks iterates four
super-tiles (rx_kernels.hip, rx_decode_fused_kernel's `st` loop), so the
piece cursors accumulate across super-tiles; the faulty variants give
the decode's take-back thousands of checksum-failed frames; the peaked
variant fills the LDS stages and the per-block pieces of three buckets, so
keys take the overflow path (device atomics, or the list rx_fixup groups).
"""
import numpy as np
import pytest

import dqdk_amd as D
from oracle import oracle as O
from test_gpu_parity import _need_gpu

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

HOST_THREADS = 16  # the GPU box's CPU share


def run_bench_form(umem: np.ndarray, desc: np.ndarray, cfg: D.RxConfig, batches: int = 1):
    """bench.py's step on one queue: device-resident UMEM, no record buffer,
    flush, then results / counters / table.  Returns (res, counters, table,
    per-kernel launches)."""
    _need_gpu()
    n = len(desc)
    dev = torch.device("cuda:0")
    d_umem = torch.from_numpy(umem).to(dev)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    d_res = torch.full((n * 8,), 0xEE, dtype=torch.uint8, device=dev)
    with D.RxQueue(0, cfg, n) as q:
        q.set_stream(torch.cuda.current_stream().cuda_stream)
        q.enable_timing(True)
        for _ in range(batches):
            q.process_device(d_umem.data_ptr(), umem.nbytes, d_desc.data_ptr(), n, d_res.data_ptr(), None)
        q.flush_histogram()
        torch.cuda.synchronize()
        launches = {k: v["launches"] for k, v in q.read_timing().items()}
        cnt = q.counters()
        del d_umem, d_desc
        table = q.histogram()
    res = d_res.cpu().numpy().view(D.RESULT_DTYPE)
    return res, cnt, table, launches


def fused_ran(launches: dict, batches: int) -> bool:
    """The fused decode ran every batch: rx_part2 once a batch and no
    rx_part1 (the records path's bucket grouping); rx_fixup, the fused path's
    overflow grouping, only in the listed-overflow form."""
    return launches.get("rx_part2", 0) == batches and launches.get("rx_part1", 0) == 0 and \
        launches.get("rx_decode", 0) == batches


def oracle_full(umem, desc, cfg):
    table = np.zeros(D.HISTO_ENTRIES, np.uint32)
    ores, ocnt, _ = O.rx_batch(umem, desc, cfg.payloadsz, cfg.mode, cfg.flags, want_keys=False, hist=table,
                               threads=HOST_THREADS)
    return ores, ocnt, table


def assert_same(res, cnt, table, ores, ocnt, otable):
    assert (res["status"] != 0xEE).all(), "unwritten results"
    np.testing.assert_array_equal(res["status"], ores["status"])
    np.testing.assert_array_equal(res["datalen"], ores["datalen"])
    np.testing.assert_array_equal(res["payload_off"], ores["payload_off"])
    np.testing.assert_array_equal(res["oob_events"], ores["oob_events"])
    assert cnt == ocnt, (cnt, ocnt)
    if not np.array_equal(table, otable):
        bad = np.flatnonzero(table != otable)
        raise AssertionError(f"{len(bad)} bins differ, first {bad[:8]}: gpu {table[bad[:8]]} oracle {otable[bad[:8]]}")


FULL = [
    # (frames, L, stride, payloadsz, faulty)
    (1 << 20, 1500, 4096, 1458, False),   # the default bench line, exactly
    (1 << 20, 9000, 9216, 8958, False),   # its by_frame_len["9000"]
    (1 << 18, 9000, 9216, 8958, False),   # configs[2] at its own batch
    (1 << 20, 1500, 4096, 1458, True),
    (1 << 20, 9000, 9216, 8958, True),
]


@pytest.mark.parametrize("n,L,stride,payloadsz,faulty", FULL,
                         ids=["1M-1500-clean", "1M-9000-clean", "256K-9000-clean", "1M-1500-faulty",
                              "1M-9000-faulty"])
def test_fused_full_size_vs_oracle(n, L, stride, payloadsz, faulty):
    umem, desc = D.synth_umem(n, L, stride, faulty=faulty, threads=HOST_THREADS)
    cfg = D.RxConfig(payloadsz=payloadsz, flags=D.F_CSUM)  # bench.py's flags: auto histogram path
    res, cnt, table, launches = run_bench_form(umem, desc, cfg)
    assert fused_ran(launches, 1), launches
    ores, ocnt, otable = oracle_full(umem, desc, cfg)
    assert_same(res, cnt, table, ores, ocnt, otable)
    if faulty:
        assert (ores["status"] == D.RX_INVALID_UDP_CSUM).sum() > 1000  # the decode takes these back
        assert ocnt["oob_events"] > 0
    else:
        assert (ores["status"] == D.RX_OK).all()


@pytest.mark.parametrize("ovf", ["auto", "atomics", "list"])
def test_fused_peaked_faulty_overflows_pieces(monkeypatch, ovf):
    """1M x 1500 B, faulty headers and checksums AND a peaked spectrum (3/8
    of the events on four hot bins in three L1 buckets): the LDS stages of
    those buckets overflow every round and their per-block pieces fill, so
    keys go through the block overflow regions -- to the table by device
    atomics, or listed and grouped by rx_part1 (DQDK_GPU_OVF_LIST; auto: by
    the previous batch's overflow); bins receive far more than 65535 events.
    Two batches: the second adds onto the first in the table."""
    if ovf != "auto":
        monkeypatch.setenv("DQDK_GPU_OVF_LIST", "1" if ovf == "list" else "0")
    n = 1 << 20
    umem, desc = D.synth_umem(n, 1500, 4096, faulty=True, peaked=True, threads=HOST_THREADS)
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM)
    res, cnt, table, launches = run_bench_form(umem, desc, cfg, batches=2)
    assert fused_ran(launches, 2) and launches.get("rx_slice_histo", 0) >= 1, launches
    if ovf != "auto":
        assert launches.get("rx_fixup", 0) == (2 if ovf == "list" else 0), launches
    ores, ocnt, otable = oracle_full(umem, desc, cfg)
    otable *= 2
    ocnt = {k: (v if k == "first_abort_idx" else 2 * v) for k, v in ocnt.items()}
    assert_same(res, cnt, table, ores, ocnt, otable)
    assert int(otable.max()) > 0xFFFF


@pytest.mark.parametrize("ovf", ["atomics", "list"])
@pytest.mark.parametrize("L,stride,payloadsz", [(1500, 4096, 1458), (9000, 9216, 8958)])
def test_fused_overflow_regions_spill_to_the_table(monkeypatch, L, stride, payloadsz, ovf):
    """The fused decode's per-block overflow regions are bounded (64K keys, or
    an eighth of a block's keys); past that a key goes to the table by a
    device atomic.  With the regions forced down to 64 keys (DQDK_GPU_OVF_BLK)
    and the peaked spectrum overflowing every round, most overflow keys take
    that spill: the table, results and counters still equal the oracle's."""
    monkeypatch.setenv("DQDK_GPU_OVF_BLK", "64")
    monkeypatch.setenv("DQDK_GPU_OVF_LIST", "1" if ovf == "list" else "0")
    n = 1 << 18
    umem, desc = D.synth_umem(n, L, stride, faulty=True, peaked=True, threads=HOST_THREADS)
    cfg = D.RxConfig(payloadsz=payloadsz, flags=D.F_CSUM)
    res, cnt, table, launches = run_bench_form(umem, desc, cfg)
    assert fused_ran(launches, 1) and launches.get("rx_fixup", 0) == (1 if ovf == "list" else 0), launches
    ores, ocnt, otable = oracle_full(umem, desc, cfg)
    assert_same(res, cnt, table, ores, ocnt, otable)


def test_records_path_full_size_vs_oracle():
    """The records path (frame-order 4-B records, rx_part1 grouping them) at
    1M x 1500 B: every result, record, counter and the whole table."""
    _need_gpu()
    n = 1 << 20
    umem, desc = D.synth_umem(n, 1500, 4096, faulty=True, threads=HOST_THREADS)
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM)
    E = cfg.events
    dev = torch.device("cuda:0")
    d_umem = torch.from_numpy(umem).to(dev)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    d_res = torch.full((n * 8,), 0xEE, dtype=torch.uint8, device=dev)
    d_keys = torch.full((n * E,), -1, dtype=torch.int32, device=dev)
    with D.RxQueue(0, cfg, n) as q:
        q.set_stream(torch.cuda.current_stream().cuda_stream)
        q.process_device(d_umem.data_ptr(), umem.nbytes, d_desc.data_ptr(), n, d_res.data_ptr(), d_keys.data_ptr())
        torch.cuda.synchronize()
        cnt = q.counters()
        del d_umem, d_desc
        table = q.histogram()
    res = d_res.cpu().numpy().view(D.RESULT_DTYPE)
    keys = d_keys.cpu().numpy().view(np.uint32)
    otable = np.zeros(D.HISTO_ENTRIES, np.uint32)
    ores, ocnt, okeys = O.rx_batch(umem, desc, cfg.payloadsz, cfg.mode, cfg.flags, hist=otable,
                                   threads=HOST_THREADS)
    assert_same(res, cnt, table, ores, ocnt, otable)
    ok = ores["status"] == D.RX_OK
    np.testing.assert_array_equal(keys.reshape(n, E)[ok], okeys.reshape(n, E)[ok])


def test_slice_pass_over_a_full_stage_of_batches():
    """256K x 9000 B batches (configs[2]) staged as deep as the queue allows
    (32): one slice pass takes ~1100 runs per two-slice span (more than one
    1024-entry chunk of its LDS) and ~1M events per span, so its packed-u16
    bins are drained into the base plane between groups many times.  The
    same batch k times: the table is k times the oracle's."""
    n = 1 << 18
    umem, desc = D.synth_umem(n, 9000, 9216, faulty=True, threads=HOST_THREADS)
    cfg = D.RxConfig(payloadsz=8958, flags=D.F_CSUM)
    with D.RxQueue(0, cfg, n) as q:
        k = q.histogram_batches_per_pass()
    assert k == 32
    res, cnt, table, launches = run_bench_form(umem, desc, cfg, batches=k)
    assert fused_ran(launches, k) and launches.get("rx_slice_histo", 0) == 1, launches
    ores, ocnt, otable = oracle_full(umem, desc, cfg)
    otable *= k
    ocnt = {kk: (v if kk == "first_abort_idx" else k * v) for kk, v in ocnt.items()}
    assert_same(res, cnt, table, ores, ocnt, otable)


def test_staging_probe_switches_piece_buffers_exactly(monkeypatch):
    """The staging placement probe (include/dqdk_gpu.h): a queue's first
    3 x DQDK_GPU_PROBE_CANDS fused batches of >= 64K frames run on the
    candidate piece buffers (untimed, then timed in order and in reverse
    order; the decode's pieces and its overflow
    regions live there), the next on the fastest, the others freed.  Faulty,
    peaked frames (pieces and overflow regions both used) over three batches
    more than the probe takes: the table, results and counters are k times
    the oracle's, and the probe has decided (on by default)."""
    _need_gpu()
    monkeypatch.delenv("DQDK_GPU_STAGING_PROBE", raising=False)
    n = 1 << 16
    umem, desc = D.synth_umem(n, 1500, 4096, faulty=True, peaked=True, threads=HOST_THREADS)
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM)
    dev = torch.device("cuda:0")
    d_umem = torch.from_numpy(umem).to(dev)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    d_res = torch.full((n * 8,), 0xEE, dtype=torch.uint8, device=dev)
    with D.RxQueue(0, cfg, n) as q:
        ncand = len(q.staging_probe()["ns_per_frame"])
        k = 3 * ncand + 3
        q.set_stream(torch.cuda.current_stream().cuda_stream)
        for b in range(k):
            q.process_device(d_umem.data_ptr(), umem.nbytes, d_desc.data_ptr(), n, d_res.data_ptr(), None)
            if b == 3:
                assert q.staging_probe()["chosen"] == -1  # still probing
        q.flush_histogram()
        torch.cuda.synchronize()
        probe = q.staging_probe()
        cnt = q.counters()
        table = q.histogram()
    res = d_res.cpu().numpy().view(D.RESULT_DTYPE)
    assert 0 <= probe["chosen"] < ncand and all(t > 0 for t in probe["ns_per_frame"]), probe
    ores, ocnt, otable = oracle_full(umem, desc, cfg)
    otable *= k
    ocnt = {kk: (v if kk == "first_abort_idx" else k * v) for kk, v in ocnt.items()}
    assert_same(res, cnt, table, ores, ocnt, otable)


def test_staging_probe_off_and_below_its_batch_size(monkeypatch):
    """DQDK_GPU_STAGING_PROBE=0 at queue creation (chosen -2), or batches
    under 64K frames (on, unset or =1, but never started: -1): nothing
    timed."""
    _need_gpu()
    for env, n, want in (("0", 1 << 16, -2), (None, 4096, -1), ("1", 4096, -1)):
        if env is None:
            monkeypatch.delenv("DQDK_GPU_STAGING_PROBE", raising=False)
        else:
            monkeypatch.setenv("DQDK_GPU_STAGING_PROBE", env)
        umem, desc = D.synth_umem(n, 1500, 4096, threads=HOST_THREADS)
        dev = torch.device("cuda:0")
        d_umem = torch.from_numpy(umem).to(dev)
        d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
        d_res = torch.empty((n * 8,), dtype=torch.uint8, device=dev)
        with D.RxQueue(0, D.RxConfig(payloadsz=1458, flags=D.F_CSUM | D.F_HISTO_PARTITIONED), n) as q:
            q.set_stream(torch.cuda.current_stream().cuda_stream)
            for _ in range(8):
                q.process_device(d_umem.data_ptr(), umem.nbytes, d_desc.data_ptr(), n, d_res.data_ptr(), None)
            torch.cuda.synchronize()
            p = q.staging_probe()
        assert p["chosen"] == want and not any(p["ns_per_frame"]), (env, n, p)
