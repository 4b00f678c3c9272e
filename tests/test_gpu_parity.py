"""HIP path vs the oracle on identical UMEM (bit-exact), through the C ABI.

Every test here runs the gfx950 kernels in dqdk_amd/lib/libdqdk_gpu.so and
compares per-frame verdicts, payload offsets, datalen, decoded records,
counters and the histogram with oracle/ (the C restatement pinned by
tests/golden/).  Full BASELINE sizes are covered through size-independent
properties at the end of the file.
"""
import numpy as np
import pytest

import dqdk_amd as D
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _need_gpu():
    if not torch.cuda.is_available() or D.device_count() < 1:
        pytest.fail("GPU tests need a gfx950 device (none visible)")


def to_dev(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to("cuda:0")


def run_gpu(umem, desc, cfg: D.RxConfig, keys=True, histogram=False, q=None):
    """One device-resident batch; returns (res, counters, keys, hist|None)."""
    _need_gpu()
    n = len(desc)
    own = q is None
    if own:
        q = D.RxQueue(0, cfg, max(n, 1))
    E = cfg.events
    d_umem = to_dev(umem)
    d_desc = to_dev(desc)
    d_res = torch.full((n * 8,), 0xEE, dtype=torch.uint8, device="cuda:0")  # poison: every result must be written
    d_keys = torch.full((max(n * E, 1),), -1, dtype=torch.int32, device="cuda:0") if keys else None
    stream = torch.cuda.current_stream().cuda_stream
    q.set_stream(stream)
    q.process_device(d_umem.data_ptr(), umem.nbytes, d_desc.data_ptr(), n, d_res.data_ptr(),
                     d_keys.data_ptr() if keys else None)
    torch.cuda.synchronize()
    res = d_res.cpu().numpy().view(D.RESULT_DTYPE)
    unwritten = np.flatnonzero(res["status"] == 0xEE)
    assert len(unwritten) == 0, ("unwritten results", len(unwritten), unwritten[:16])
    cnt = q.counters()
    k = d_keys.cpu().numpy().view(np.uint32)[: n * E] if keys else None
    hist = q.histogram() if histogram else None
    umem_after = d_umem.cpu().numpy() if cfg.flags & D.F_CSUM_WRITEBACK else None
    if own:
        q.close()
    return res, cnt, k, hist, umem_after


def compare(umem, desc, cfg: D.RxConfig, check_hist=False, records=True):
    """records=False passes no record buffer: a partitioned batch then takes
    the fused decode (keys bucketed in the decode, never in frame order)."""
    gres, gcnt, gkeys, ghist, gumem = run_gpu(umem, desc, cfg, keys=records, histogram=check_hist)
    oumem = umem.copy()
    ores, ocnt, okeys = O.rx_batch(oumem, desc, cfg.payloadsz, cfg.mode, cfg.flags, cfg.port_start, cfg.port_end)
    np.testing.assert_array_equal(gres["status"], ores["status"])
    np.testing.assert_array_equal(gres["datalen"], ores["datalen"])
    np.testing.assert_array_equal(gres["payload_off"], ores["payload_off"])
    np.testing.assert_array_equal(gres["oob_events"], ores["oob_events"])
    E = cfg.events
    ok = ores["status"] == D.RX_OK
    if E and records:
        np.testing.assert_array_equal(gkeys.reshape(-1, E)[ok], okeys.reshape(-1, E)[ok])
    for k, v in ocnt.items():
        assert gcnt[k] == v, (k, gcnt[k], v)
    if cfg.flags & D.F_CSUM_WRITEBACK:
        np.testing.assert_array_equal(gumem, oumem)
    if check_hist:
        limit = ocnt["first_abort_idx"] if cfg.flags & D.F_BATCH_ABORT else None
        u, c = O.sparse_histogram(okeys, ores, E, limit)
        nz = np.flatnonzero(ghist)
        np.testing.assert_array_equal(nz.astype(np.uint32), u)
        np.testing.assert_array_equal(ghist[nz].astype(np.uint64), c)
    return ores, ocnt


# ---- golden fixture frames (reference-pinned inputs) ------------------------

@pytest.mark.parametrize("flags", [0, D.F_CSUM, D.F_CSUM | D.F_BATCH_ABORT, D.F_PREFILTER])
def test_golden_f1_frames(flags):
    z = np.load(__import__("pathlib").Path(__file__).parent / "golden" / "f1_parse.npz")
    umem, desc = z["umem"].copy(), z["desc"]
    e = z["expected"]
    if flags & D.F_CSUM:  # reference ip4_audit_checksum is undefined for ihl > 5
        keep = ~((e["ipc_ok"] == 255) & (e["ip_ok"] == 1))
        desc = desc[keep]
    cfg = D.RxConfig(payloadsz=64, mode=D.MODE_ENERGYHISTO, flags=flags | D.F_HISTO_PARTITIONED,
                     port_start=0, port_end=65535)
    ores, _ = compare(umem, desc, cfg, check_hist=True)
    assert len(np.unique(ores["status"])) >= 3


# ---- synthetic TRISTAN traffic -------------------------------------------

CASES = [
    # (frame_len, stride, faulty, payloadsz, mode, flags)
    (1500, 4096, False, 1458, D.MODE_ENERGYHISTO, 0),
    (1500, 4096, True, 1458, D.MODE_ENERGYHISTO, 0),
    (1500, 4096, True, 1458, D.MODE_ENERGYHISTO, D.F_CSUM),
    (1500, 4096, True, 1458, D.MODE_ENERGYHISTO, D.F_CSUM | D.F_BATCH_ABORT),
    (9000, 9216, False, 8958, D.MODE_ENERGYHISTO, D.F_CSUM),
    (9000, 9216, True, 8958, D.MODE_ENERGYHISTO, D.F_CSUM),
    (3434, 4096, True, 3392, D.MODE_LISTMODE, D.F_CSUM),       # production -s 3392
    (1500, 1536, True, 2000, D.MODE_ENERGYHISTO, D.F_CSUM),     # E*16 > datalen: reads past the datagram
    (0, 9216, True, 1458, D.MODE_ENERGYHISTO, D.F_CSUM),        # mixed 1500/9000
    (1500, 4096, True, 1458, D.MODE_LISTWAVE, D.F_CSUM),        # E = 1
    (1500, 4096, True, 1458, D.MODE_WAVEFORM, 0),               # no histogram
    (1500, 4096, True, 1458, D.MODE_ENERGYHISTO, D.F_NO_HISTO | D.F_CSUM),
    (1500, 4096, True, 8, D.MODE_ENERGYHISTO, D.F_CSUM),        # E = 0
    (9000, 9216, True, 12000, D.MODE_ENERGYHISTO, D.F_CSUM),    # E = 750: part1 stages a tile in two chunks
]


HPATHS = [D.F_HISTO_ATOMIC, D.F_HISTO_PARTITIONED]


@pytest.mark.parametrize("hpath", HPATHS, ids=["atomic", "partitioned"])
@pytest.mark.parametrize("L,stride,faulty,payloadsz,mode,flags", CASES)
def test_synthetic_parity(L, stride, faulty, payloadsz, mode, flags, hpath):
    umem, desc = D.synth_umem(3000, L, stride, faulty=faulty)
    cfg = D.RxConfig(payloadsz=payloadsz, mode=mode, flags=flags | hpath)
    ores, ocnt = compare(umem, desc, cfg, check_hist=D.histo_enabled(mode, flags))
    assert (ores["status"] == D.RX_OK).mean() > 0.9


FUSED_CASES = [c for c in CASES if c[4] != D.MODE_WAVEFORM and not (c[5] & D.F_NO_HISTO) and c[3] >= 16]


@pytest.mark.parametrize("L,stride,faulty,payloadsz,mode,flags", FUSED_CASES)
def test_fused_decode_parity(L, stride, faulty, payloadsz, mode, flags):
    """Partitioned batches without a record buffer and per-packet accounting
    take rx_decode_fused (keys bucketed in LDS, appended to per-XCD segments,
    checksum-failed frames taken back by the decode); batch-abort falls back to
    the records path.  Results, counters and the whole table vs the oracle."""
    umem, desc = D.synth_umem(6000, L, stride, faulty=faulty)
    cfg = D.RxConfig(payloadsz=payloadsz, mode=mode, flags=flags | D.F_HISTO_PARTITIONED)
    ores, ocnt = compare(umem, desc, cfg, check_hist=True, records=False)
    if faulty and flags & D.F_CSUM:
        assert (ores["status"] == D.RX_INVALID_UDP_CSUM).sum() > 0  # the decode has frames to take back


@pytest.mark.parametrize("records", [True, False], ids=["records", "fused"])
def test_fused_decode_hot_bins_overflow(records):
    """Peaked spectra: one L1 bucket gets most keys, so the fused decode's LDS
    stage and that bucket's segments overflow into the overflow list, which
    rx_part1 groups; the table is still exact."""
    _need_gpu()
    rng = np.random.default_rng(21)
    umem, desc = _peaked(20000, 0, rng)
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_HISTO_PARTITIONED)
    compare(umem, desc, cfg, check_hist=True, records=records)


@pytest.mark.parametrize("shift", [1, 2, 3, 5, 8, 10, 13, 15])
def test_unaligned_frames(shift):
    """Unaligned-chunk UMEM (src/dqdk.h:39): frames at any byte offset."""
    umem0, desc = D.synth_umem(1024, 1500, 4096, faulty=True)
    umem = np.zeros(umem0.size + 64, np.uint8)
    umem[shift:shift + umem0.size] = umem0
    desc = desc.copy()
    desc["addr"] += shift
    for flags in (0, D.F_CSUM | D.F_HISTO_PARTITIONED):
        compare(umem, desc, D.RxConfig(payloadsz=1458, flags=flags), check_hist=True)


def test_csum_writeback_mutates_umem_like_reference():
    umem, desc = D.synth_umem(512, 1500, 4096, faulty=True)
    compare(umem, desc, D.RxConfig(payloadsz=1458, flags=D.F_CSUM | D.F_CSUM_WRITEBACK))


def test_frames_at_umem_end_read_zero_past_size():
    umem, desc = D.synth_umem(64, 1500, 1504, faulty=False)
    desc = desc.copy()
    desc["addr"][-1] = umem.size - 1488  # frame runs past the UMEM end
    desc["addr"][-2] = umem.size + 4096  # entirely outside
    compare(umem, desc, D.RxConfig(payloadsz=1458, flags=D.F_CSUM), check_hist=True)


def test_prefilter_predicate():
    umem, desc = D.synth_umem(2048, 1500, 4096, faulty=True)
    rng = np.random.default_rng(7)
    f = umem.reshape(-1, 4096)
    sel = rng.random(len(desc)) < 0.1
    f[sel, 12] = 0x86                         # not IPv4 -> PASS
    sel = rng.random(len(desc)) < 0.1
    f[sel, 23] = 6                            # TCP -> PASS
    desc = desc.copy()
    sel = rng.random(len(desc)) < 0.05
    desc["len"][sel] = rng.choice([0, 10, 14, 30, 34, 40, 42], size=sel.sum())
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_PREFILTER | D.F_CSUM, port_start=5000, port_end=5000)
    ores, ocnt = compare(umem, desc, cfg, check_hist=True)
    assert ocnt["filtered_frames"] > 0


def test_random_bytes_fuzz():
    """Arbitrary bytes: every header field random, arbitrary lengths/addresses."""
    rng = np.random.default_rng(11)
    umem = rng.integers(0, 256, size=1 << 22, dtype=np.uint8)
    n = 8192
    desc = np.zeros(n, D.DESC_DTYPE)
    desc["addr"] = rng.integers(0, umem.size, size=n)
    desc["len"] = rng.integers(0, 4096, size=n)
    # a share of frames with consistent lengths so deeper branches are reached
    sel = rng.random(n) < 0.5
    for i in np.flatnonzero(sel):
        a, L = int(desc["addr"][i]), int(desc["len"][i])
        if a + 64 >= umem.size:
            continue
        ihl = int(rng.integers(0, 16)) if rng.random() < 0.2 else 5
        umem[a + 14] = 0x40 | ihl
        tot = (L - 14) & 0xFFFF
        umem[a + 16], umem[a + 17] = tot >> 8, tot & 0xFF
        u = a + 14 + ihl * 4
        ul = (tot - ihl * 4) & 0xFFFF
        if u + 8 < umem.size:
            umem[u + 4], umem[u + 5] = ul >> 8, ul & 0xFF
    for flags in (0, D.F_CSUM | D.F_HISTO_PARTITIONED, D.F_CSUM | D.F_BATCH_ABORT | D.F_HISTO_PARTITIONED):
        compare(umem, desc, D.RxConfig(payloadsz=200, flags=flags), check_hist=True)


@pytest.mark.parametrize("hpath", HPATHS, ids=["atomic", "partitioned"])
def test_skewed_histogram(hpath):
    """Real spectra are peaked: many events on few bins (LDS/atomic contention,
    counts far above 1 per bin) and whole buckets empty."""
    umem, desc = D.synth_umem(4096, 1500, 4096, faulty=False)
    f = umem.reshape(4096, 4096)
    rng = np.random.default_rng(5)
    ev = f[:, 42:42 + 91 * 16].reshape(4096, 91, 16)
    peaks = [(3, 1, 0x12, 0x34), (3, 1, 0x12, 0x35), (700, 4, 0xff, 0xff), (1511, 5, 0, 0)]
    pick = rng.integers(0, len(peaks) + 1, size=(4096, 91))
    for k, (chl, hc, e5, e6) in enumerate(peaks):
        m = pick == k
        ev[..., 2][m] = chl & 0xFF
        ev[..., 3][m] = chl >> 8
        ev[..., 5][m] = e5
        ev[..., 6][m] = e6
        ev[..., 8][m] = hc
    cfg = D.RxConfig(payloadsz=1458, flags=hpath)  # no checksum: payload edited
    _, _, okeys = O.rx_batch(umem.copy(), desc, 1458)
    per_slice = np.bincount((okeys[okeys != D.KEY_NONE] >> 14).astype(np.int64))
    assert per_slice.max() > 0xFFFF  # bins and slices far past the u16 range
    compare(umem, desc, cfg, check_hist=True)


def test_host_dropin_api_matches_device_api():
    """dqdk_gpu_rx_batch (host UMEM, zero-copy) == device-resident path."""
    _need_gpu()
    umem, desc = D.synth_umem(2048, 1500, 4096, faulty=True)
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM)
    ores, ocnt, _ = O.rx_batch(umem.copy(), desc, cfg.payloadsz, cfg.mode, cfg.flags)
    with D.RxQueue(0, cfg, 4096) as q:
        res, delta = q.process_batch(umem, desc)
        res2, delta2 = q.process_batch(umem, desc)
        total = q.counters()
    np.testing.assert_array_equal(res, ores)
    for k, v in ocnt.items():
        assert delta[k] == v and delta2[k] == v, k
    assert total["rcvd_pkts"] == 2 * ocnt["rcvd_pkts"]


def test_host_dropin_grown_umem_at_the_same_address():
    """A UMEM registered by a first batch, then a larger one at the same
    address (a grown view of one buffer): the second batch's frames past the
    first registration are read through a registration that covers them (the
    old one is replaced, not reused past its end), and both batches equal the
    oracle."""
    _need_gpu()
    umem, desc = D.synth_umem(2048, 1500, 4096, faulty=True)
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM)
    half = len(desc) // 2
    small, d_small = umem[: half * 4096], desc[:half]
    ores1, ocnt1, _ = O.rx_batch(small.copy(), d_small, cfg.payloadsz, cfg.mode, cfg.flags)
    ores2, ocnt2, _ = O.rx_batch(umem.copy(), desc, cfg.payloadsz, cfg.mode, cfg.flags)
    with D.RxQueue(0, cfg, 4096) as q:
        res1, delta1 = q.process_batch(small, d_small)
        res2, delta2 = q.process_batch(umem, desc)
        q.unregister_umem(umem)
    np.testing.assert_array_equal(res1, ores1)
    np.testing.assert_array_equal(res2, ores2)
    for k, v in ocnt1.items():
        assert delta1[k] == v, k
    for k, v in ocnt2.items():
        assert delta2[k] == v, k


def test_histogram_accumulates_across_batches_and_merges():
    _need_gpu()
    cfg = D.RxConfig(payloadsz=1458)
    acc = np.zeros(D.HISTO_ENTRIES, np.uint32)
    ref_keys = []
    with D.RxQueue(0, cfg, 1024) as q:
        for b in range(3):
            umem, desc = D.synth_umem(1024, 1500, 4096, faulty=True, first=b * 1024)
            run_gpu(umem, desc, cfg, keys=False, q=q)
            r, _, k = O.rx_batch(umem.copy(), desc, 1458)
            ok = r["status"] == 0
            kk = k.reshape(-1, 91)[ok].ravel()
            ref_keys.append(kk[kk != D.KEY_NONE])
        q.accumulate_histogram(acc)
    u, c = np.unique(np.concatenate(ref_keys), return_counts=True)
    nz = np.flatnonzero(acc)
    np.testing.assert_array_equal(nz, u)
    np.testing.assert_array_equal(acc[nz], c)


# ---- full BASELINE sizes: size-independent properties ----------------------

@pytest.mark.parametrize("L,stride,payloadsz", [(1500, 4096, 1458), (9000, 9216, 8958)])
def test_full_size_properties(L, stride, payloadsz):
    """1M-frame batches (BASELINE.json north star), records path: (1)
    counters are consistent with the per-frame results, (2) histogram mass ==
    accepted events == records, (3) every frame, record, counter and the
    whole table equal the oracle's (host threads), (4) batch order does not
    matter (permuted descriptors through the fused path give the oracle's
    table)."""
    _need_gpu()
    n = 1 << 20
    umem, desc = D.synth_umem(n, L, stride, faulty=True, threads=16)
    cfg = D.RxConfig(payloadsz=payloadsz, flags=D.F_CSUM)
    E = cfg.events
    res, cnt, keys, hist, _ = run_gpu(umem, desc, cfg, keys=True, histogram=True)
    st = res["status"]
    assert (st == D.RX_OK).mean() > 0.95
    assert cnt["rcvd_pkts"] == n and cnt["rcvd_frames"] == n
    assert cnt["total_events"] == E * int((st == D.RX_OK).sum())
    assert cnt["invalid_ip_pkts"] == int(((st == D.RX_INVALID_IP) | (st == D.RX_INVALID_IP_CSUM)).sum())
    assert cnt["rcvd_bytes"] == int(res["datalen"][st == D.RX_OK].astype(np.uint64).sum())
    mass = int(hist.astype(np.uint64).sum())
    kk = keys.reshape(n, E)[st == D.RX_OK]
    nrec = int((kk != D.KEY_NONE).sum())
    if nrec != cnt["total_events"] - cnt["oob_events"]:
        okf = np.flatnonzero(st == D.RX_OK)
        miss = okf[(keys.reshape(n, E)[okf] == D.KEY_NONE).sum(axis=1) > res["oob_events"][okf]]
        print("frames missing records:", len(miss), miss[:16], "tiles", np.unique(miss // 256)[:16],
              "slot%4", np.bincount(miss % 256 % 4, minlength=4))
        f = miss[0]
        print("frame", f, "NONE at", np.flatnonzero(keys.reshape(n, E)[f] == D.KEY_NONE)[:64])
    assert (mass, nrec) == (cnt["total_events"] - cnt["oob_events"],) * 2, (mass, nrec)
    # every frame, record, counter and the whole table vs the oracle (host threads)
    otable = np.zeros(D.HISTO_ENTRIES, np.uint32)
    ores, ocnt, okeys = O.rx_batch(umem, desc, payloadsz, flags=D.F_CSUM, hist=otable, threads=16)
    np.testing.assert_array_equal(res, ores)
    assert cnt == ocnt
    okk = ores["status"] == D.RX_OK
    np.testing.assert_array_equal(keys.reshape(n, E)[okk], okeys.reshape(n, E)[okk])
    assert np.array_equal(hist, otable)
    # batch order does not matter: permuted descriptors, fused path (no records), same table as the oracle's
    perm = np.random.default_rng(3).permutation(n)
    _, _, _, hist2, _ = run_gpu(umem, desc[perm], cfg, keys=False, histogram=True)
    assert np.array_equal(hist2, otable)


def test_configs1_parse_checksum_only_form():
    """BASELINE configs[1] exactly as bench.py measures it: 256K x 1500 B,
    IPv4 + UDP checksums, no histogram, NO record buffer (d_keys = NULL), so
    the decode does no event work; every frame against the oracle."""
    _need_gpu()
    n = 1 << 18
    umem, desc = D.synth_umem(n, 1500, 4096, faulty=True, threads=16)
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM | D.F_NO_HISTO)
    res, cnt, _, _, _ = run_gpu(umem, desc, cfg, keys=False)
    ores, ocnt, _ = O.rx_batch(umem, desc, cfg.payloadsz, cfg.mode, cfg.flags, want_keys=False)
    np.testing.assert_array_equal(res, ores)  # status, datalen, payload_off, oob_events (0: no histogram)
    assert cnt == ocnt
    assert ocnt["invalid_udp_pkts"] > 0 and ocnt["invalid_ip_pkts"] > 0 and ocnt["empty_pkts"] > 0


def test_configs2_jumbo_full_batch_vs_oracle():
    """BASELINE configs[2] at its own size: 256K x 9000 B, full path (IPv4 +
    UDP checksums, decode, histogram), every frame, record and bin against
    the oracle."""
    _need_gpu()
    n = 1 << 18
    umem, desc = D.synth_umem(n, 9000, 9216, faulty=True, threads=16)
    cfg = D.RxConfig(payloadsz=8958, flags=D.F_CSUM)
    res, cnt, keys, hist, _ = run_gpu(umem, desc, cfg, keys=True, histogram=True)
    table = np.zeros(D.HISTO_ENTRIES, np.uint32)
    ores, ocnt, okeys = O.rx_batch(umem, desc, cfg.payloadsz, cfg.mode, cfg.flags, hist=table, threads=16)
    np.testing.assert_array_equal(res, ores)
    assert cnt == ocnt
    ok = ores["status"] == D.RX_OK
    np.testing.assert_array_equal(keys.reshape(n, -1)[ok], okeys.reshape(n, -1)[ok])
    assert np.array_equal(hist, table)


@pytest.mark.parametrize("fold", [True, False], ids=["folded", "fold-off"])
@pytest.mark.parametrize("hpath,kernels", [
    (D.F_HISTO_ATOMIC, {"rx_decode", "rx_histo_atomic"}),
    (D.F_HISTO_PARTITIONED | D.F_HISTO_EAGER, {"rx_decode", "rx_part1", "rx_part2", "rx_slice_histo"})],
    ids=["atomic", "partitioned"])
def test_stage_timing_reports_every_kernel_once_per_batch(hpath, kernels, fold, monkeypatch):
    """The records path's kernels, each timed once per batch: the per-packet
    counters folded into rx_decode (default), or counted by rx_abort +
    rx_count launches (DQDK_GPU_FOLD=0, read at queue creation)."""
    _need_gpu()
    if not fold:
        monkeypatch.setenv("DQDK_GPU_FOLD", "0")
        kernels = kernels | {"rx_abort", "rx_count"}
    umem, desc = D.synth_umem(1024, 1500, 4096)
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM | hpath)
    q = D.RxQueue(0, cfg, len(desc))
    try:
        q.enable_timing(True)
        for _ in range(3):
            run_gpu(umem, desc, cfg, q=q)
        t = q.read_timing()
        assert {k for k, v in t.items() if v["launches"]} == kernels
        for k in kernels:
            assert t[k]["launches"] == 3 and t[k]["ms"] > 0
        assert all(v["launches"] == 0 for v in q.read_timing().values())  # read clears
    finally:
        q.close()


def _peaked(n, first, rng):
    """n clean 1500-B frames whose events pile onto 4 bins (counts >> 256)."""
    umem, desc = D.synth_umem(n, 1500, 4096, faulty=False, first=first)
    ev = umem.reshape(n, 4096)[:, 42:42 + 91 * 16].reshape(n, 91, 16)
    peaks = [(3, 1, 0x12, 0x34), (700, 4, 0xff, 0xff), (1511, 5, 0, 0), (0, 0, 0, 0)]
    pick = rng.integers(0, len(peaks) + 2, size=(n, 91))
    for k, (chl, hc, e5, e6) in enumerate(peaks):
        m = pick == k
        ev[..., 2][m] = chl & 0xFF
        ev[..., 3][m] = chl >> 8
        ev[..., 5][m] = e5
        ev[..., 6][m] = e6
        ev[..., 8][m] = hc
    return umem, desc


def test_auto_path_mixes_atomic_and_partitioned_batches_with_carries():
    """One queue, batches on both sides of the partition threshold: the atomic
    path adds to the table's base plane, the partitioned sweep to its low-byte
    plane with carries of 256; the table must equal the oracle's over all
    batches (hot bins pass many multiples of 256 within and across batches)."""
    _need_gpu()
    rng = np.random.default_rng(11)
    cfg = D.RxConfig(payloadsz=1458)  # auto path: partitioned at >= 4M events
    keys_all = []
    with D.RxQueue(0, cfg, 48000) as q:
        first = 0
        for n in (1024, 48000, 2048, 48000, 512):
            umem, desc = _peaked(n, first, rng)
            first += n
            run_gpu(umem, desc, cfg, keys=False, q=q)
            r, _, k = O.rx_batch(umem, desc, 1458)
            kk = k.reshape(-1, 91)[r["status"] == 0].ravel()
            keys_all.append(kk[kk != D.KEY_NONE])
        hist = q.histogram()
        assert q.histogram_nonzero() == int(np.count_nonzero(hist))
    u, c = np.unique(np.concatenate(keys_all), return_counts=True)
    assert c.max() > 100000
    nz = np.flatnonzero(hist)
    np.testing.assert_array_equal(nz, u)
    np.testing.assert_array_equal(hist[nz], c)


def test_staged_slice_pass_flush_and_reset():
    """Partitioned batches stage their events; the slice pass runs once per k
    staged batches and before any read.  k + 1 batches (one automatic pass +
    one pending at the read) sum like the oracle; reset drops the table with
    whatever is staged; the next batch alone is then in the table."""
    _need_gpu()
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM | D.F_HISTO_PARTITIONED)
    ref = []
    with D.RxQueue(0, cfg, 1024) as q:
        q.enable_timing(True)
        kp = q.histogram_batches_per_pass()
        assert kp > 1  # 1024 x 91 events: a few per slice
        for b in range(kp + 1):
            umem, desc = D.synth_umem(1024, 1500, 4096, faulty=True, first=b * 1024)
            run_gpu(umem, desc, cfg, keys=False, q=q)
            r, _, k = O.rx_batch(umem.copy(), desc, 1458, flags=D.F_CSUM)
            kk = k.reshape(-1, 91)[r["status"] == D.RX_OK].ravel()
            ref.append(kk[kk != D.KEY_NONE])
        assert q.read_timing()["rx_slice_histo"]["launches"] == 1  # after the k-th batch only
        hist = q.histogram()
        u, c = np.unique(np.concatenate(ref), return_counts=True)
        nz = np.flatnonzero(hist)
        np.testing.assert_array_equal(nz, u)
        np.testing.assert_array_equal(hist[nz], c)
        # staged batch, then reset: neither survives
        umem, desc = D.synth_umem(1024, 1500, 4096, faulty=True, first=9000)
        run_gpu(umem, desc, cfg, keys=False, q=q)
        q.reset_histogram()
        assert not q.histogram().any()
        run_gpu(umem, desc, cfg, keys=False, q=q)
        q.flush_histogram()
        hist = q.histogram()
    r, _, k = O.rx_batch(umem.copy(), desc, 1458, flags=D.F_CSUM)
    u, c = O.sparse_histogram(k, r, 91)
    nz = np.flatnonzero(hist)
    np.testing.assert_array_equal(nz, u)
    np.testing.assert_array_equal(hist[nz], c)


def test_launch_guard_refuses_umem_past_its_allocation():
    """Host-side launch guard: a UMEM image from dqdk_gpu_device_alloc whose
    stated umem_size runs past the allocation is refused with -EINVAL before
    any kernel reads past it (the kernels' buffer extents come from the
    caller's sizes)."""
    _need_gpu()
    umem, desc = D.synth_umem(256, 1500, 4096)
    with D.DeviceBuffer(0, umem.nbytes) as img, D.RxQueue(0, D.RxConfig(payloadsz=1458), 256) as q:
        img.tensor.copy_(torch.from_numpy(umem))
        d_desc = torch.from_numpy(desc.view(np.uint8)).cuda()
        d_res = torch.zeros(256 * 8, dtype=torch.uint8, device="cuda:0")
        q.set_stream(torch.cuda.current_stream().cuda_stream)
        with pytest.raises(D.DqdkError) as e:
            q.process_device(img.ptr, umem.nbytes + 4096, d_desc.data_ptr(), 256, d_res.data_ptr())
        assert e.value.errno == 22
        q.process_device(img.ptr, umem.nbytes, d_desc.data_ptr(), 256, d_res.data_ptr())  # exact: fine
        torch.cuda.synchronize()
        assert q.counters()["rcvd_pkts"] == 256


@pytest.mark.parametrize("flags", [D.F_CSUM, D.F_CSUM | D.F_BATCH_ABORT, D.F_PREFILTER])
@pytest.mark.parametrize("n", [1, 64, 255, 256])
def test_small_batches_single_launch(n, flags):
    """Batches of at most 256 frames (DQDK's default -b 64, src/tristan.c:393)
    run decode, abort and count in one launch (rx_small): results, records,
    counters and table equal the oracle's, for the device form and for the
    host drop-in (pinned descriptors / results, return at the last read of
    the caller's frames), under both accountings."""
    umem, desc = D.synth_umem(n, 1500, 4096, faulty=True, first=7 * n)
    cfg = D.RxConfig(payloadsz=1458, flags=flags | D.F_HISTO_ATOMIC, port_start=5000, port_end=5000)
    compare(umem, desc, cfg, check_hist=True)
    with D.RxQueue(0, cfg, 256) as q:
        q.enable_timing(True)
        res, delta = q.process_batch(umem, desc)
        t = q.read_timing()
        assert t["rx_decode"]["launches"] == 1 and t["rx_abort"]["launches"] == 0  # one launch for the three
        ores, ocnt, _ = O.rx_batch(umem.copy(), desc, cfg.payloadsz, cfg.mode, cfg.flags, cfg.port_start,
                                   cfg.port_end)
        np.testing.assert_array_equal(res, ores)
        for k in ("rcvd_pkts", "rcvd_bytes", "invalid_ip_pkts", "invalid_udp_pkts", "total_events", "total_bytes",
                  "oob_events", "first_abort_idx", "failing_batches"):
            assert delta[k] == ocnt[k], (k, delta[k], ocnt[k])
        q.unregister_umem(umem)
