"""fetch_xsk accounting (src/dqdk.c:252-322) in the oracle: per-packet vs
batch-abort semantics, -ENOBUFS on datalen 0, the udplen < 8 wrap, prefilter."""
import numpy as np

import dqdk_amd as D
from oracle import oracle as O


def batch(faulty=True, n=2048):
    return D.synth_umem(n, 1500, 4096, faulty=faulty)


def test_batch_abort_stops_at_first_failure():
    umem, desc = batch()
    res, c_pp, keys = O.rx_batch(umem.copy(), desc, 1458, flags=0)
    res2, c_ab, _ = O.rx_batch(umem.copy(), desc, 1458, flags=D.F_BATCH_ABORT)
    assert np.array_equal(res, res2)  # per-frame verdicts are the same
    a = c_ab["first_abort_idx"]
    assert a == c_pp["first_abort_idx"] < len(desc)
    assert res["status"][a] != 0 and (res["status"][:a] == 0).all()
    assert c_ab["rcvd_pkts"] == a + 1          # the failing frame is counted (dqdk.c:189)
    assert c_ab["rcvd_frames"] == len(desc)   # whole peeked batch (dqdk.c:289)
    assert c_ab["total_events"] == 91 * a
    assert c_ab["failing_batches"] == c_pp["failing_batches"] == 1
    assert c_pp["rcvd_pkts"] == len(desc)


def test_clean_batch_has_no_failure():
    umem, desc = batch(faulty=False)
    res, c, _ = O.rx_batch(umem.copy(), desc, 1458, flags=D.F_CSUM | D.F_BATCH_ABORT)
    assert (res["status"] == 0).all()
    assert c["failing_batches"] == 0 and c["first_abort_idx"] == len(desc)
    assert c["rcvd_bytes"] == 1458 * len(desc) and c["total_events"] == 91 * len(desc)


def test_empty_payload_is_enobufs_and_wrap_is_accepted():
    umem, desc = batch()
    res, c, _ = O.rx_batch(umem.copy(), desc, 1458)
    lens = desc["len"]
    assert (res["status"][lens == 42] == D.RX_EMPTY).all()      # udplen 8 -> datalen 0
    wrap = lens == 40                                           # udplen 6 -> datalen 0xFFFFFFFE
    assert wrap.any() and (res["status"][wrap] == D.RX_OK).all()
    assert (res["datalen"][wrap] == 0xFFFFFFFE).all()
    assert c["empty_pkts"] == int((lens == 42).sum())


def test_csum_config_catches_corrupted_checksums_only():
    umem, desc = batch()
    r0, c0, _ = O.rx_batch(umem.copy(), desc, 1458, flags=0)
    r1, c1, _ = O.rx_batch(umem.copy(), desc, 1458, flags=D.F_CSUM)
    bad = r1["status"] == D.RX_INVALID_UDP_CSUM
    assert bad.sum() > 0 and (r0["status"][bad] == 0).all()
    assert c1["invalid_udp_pkts"] == c0["invalid_udp_pkts"] + bad.sum()


def test_writeback_zeroes_udp_check_in_place():
    umem, desc = batch(faulty=False, n=64)
    u = umem.copy()
    O.rx_batch(u, desc, 1458, flags=D.F_CSUM | D.F_CSUM_WRITEBACK)
    f = u.reshape(64, 4096)
    assert (f[:, 40] == 0).all() and (f[:, 41] == 0).all()
    # and a second pass then skips the checksum (check == 0 -> valid, udp.c:12-14)
    res, c, _ = O.rx_batch(u, desc, 1458, flags=D.F_CSUM)
    assert (res["status"] == 0).all()


def test_prefilter_matches_forwarder_rules():
    lib = O.oracle()
    f = np.zeros(64, np.uint8)
    f[12], f[13], f[23], f[34], f[35] = 8, 0, 17, 0x13, 0x88  # sport 5000
    p = f.ctypes.data
    assert lib.or_prefilter(p, 0, 5000, 5000) == 0
    assert lib.or_prefilter(p, 14, 5000, 5000) == 0
    assert lib.or_prefilter(p, 34, 5000, 5000) == 0
    assert lib.or_prefilter(p, 42, 5000, 5000) == 0
    assert lib.or_prefilter(p, 43, 5000, 5000) == 2
    assert lib.or_prefilter(p, 43, 5001, 5002) == 1
    f[23] = 6
    assert lib.or_prefilter(p, 43, 5000, 5000) == 1
    assert lib.or_prefilter(p, 34, 5000, 5000) == 0  # length checked before protocol
    f[12] = 0x86
    assert lib.or_prefilter(p, 20, 5000, 5000) == 1  # not IPv4: PASS before the ip length check


def test_threaded_oracle_equals_sequential():
    """or_rx_batch_mt (the full-size GPU checks' oracle) == or_rx_batch:
    results, keys, counters and the table, faulty data, several threads."""
    umem, desc = D.synth_umem(6000, 1500, 4096, faulty=True)
    for flags in (0, D.F_CSUM, D.F_CSUM | D.F_PREFILTER):
        h1 = np.zeros(O.HISTO_ENTRIES, np.uint32)
        h8 = np.zeros(O.HISTO_ENTRIES, np.uint32)
        r1, c1, k1 = O.rx_batch(umem.copy(), desc, 1458, flags=flags, port_start=5000, port_end=5000, hist=h1)
        r8, c8, k8 = O.rx_batch(umem.copy(), desc, 1458, flags=flags, port_start=5000, port_end=5000, hist=h8,
                                threads=7)
        assert np.array_equal(r1, r8) and np.array_equal(k1, k8) and c1 == c8, (c1, c8)
        assert c1["failing_batches"] == 1 and c1["first_abort_idx"] < len(desc)
        nz = np.flatnonzero(h1)
        assert np.array_equal(nz, np.flatnonzero(h8)) and np.array_equal(h1[nz], h8[nz])


def test_peaked_synth_frames_stay_valid():
    """DQDK_SYNTH_PEAKED: 3/8 of the events on four hot bins, checksums
    still valid (computed after the events)."""
    umem, desc = D.synth_umem(512, 1500, 4096, peaked=True)
    res, c, keys = O.rx_batch(umem.copy(), desc, 1458, flags=D.F_CSUM)
    assert (res["status"] == D.RX_OK).all() and c["oob_events"] == 0
    u, cnt = np.unique(keys, return_counts=True)
    hot = cnt.argsort()[-4:]
    assert 0.3 < cnt[hot].sum() / keys.size < 0.45
    assert len(np.unique(u[hot] >> 21)) == 3  # three L1 buckets
