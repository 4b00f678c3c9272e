"""The fused decode's variants vs the oracle on frames built to hit every
edge of its geometry.  The shipped library holds policies 3 and 2 (whole-line
flushes / whole-word flushes, both with non-temporal frame loads: the
defaults from and below 128 events per frame); the first-line hand-off
(policy bit 2) and the other A/B variants are in a -DDQDK_AB_VARIANTS build
only, and their cases skip on the shipped one.

Phase A reads each frame's first 128 B for the headers; with the hand-off it
also decodes the events and sums the checksum bytes of that line, and the
stream starts at the chunk holding the line's end (frame_geo's a_end).  These
frames exercise every branch of that split: any byte offset (so the line ends
anywhere from 16 to 128 B past the 16-B aligned start), IP options (ihl 5..15
move the payload), datagrams that end inside the first line (nothing left to
stream when few events are decoded), odd lengths, out-of-bounds events in the
line, bad and absent UDP checksums (the fix-up takes A's keys back), and
frames whose first line runs past the UMEM end (no hand-off there).  Every
policy variant runs on the same frames: results, counters and the whole table
must equal the oracle's.
"""
import numpy as np
import pytest

import dqdk_amd as D
from oracle import oracle as O

from test_gpu_parity import compare, _need_gpu

pytestmark = pytest.mark.gpu


def _csum16(b: np.ndarray) -> int:
    """RFC 1071 one's complement sum of big-endian words (odd length: zero pad)."""
    if b.size & 1:
        b = np.concatenate([b, np.zeros(1, np.uint8)])
    w = b.reshape(-1, 2).astype(np.uint32)
    s = int(((w[:, 0] << 8) | w[:, 1]).sum())
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def build_frames(n: int, seed: int, slot: int = 2048):
    rng = np.random.default_rng(seed)
    umem = rng.integers(0, 256, size=n * slot + 512, dtype=np.uint8)
    desc = np.zeros(n, D.DESC_DTYPE)
    for i in range(n):
        a = i * slot + int(rng.integers(0, 256))
        ihl = 5 if rng.random() < 0.6 else int(rng.integers(5, 16))
        r = rng.random()
        dl = int(rng.integers(0, 90)) if r < 0.35 else int(rng.integers(90, 1459)) if r < 0.7 else 1458
        dl = min(dl, slot - 256 - 14 - 4 * ihl - 8)
        u = a + 14 + 4 * ihl
        L = 14 + 4 * ihl + 8 + dl
        f = umem[a:a + L + 1]
        f[12], f[13] = 0x08, 0x00
        f[14] = 0x40 | ihl
        tot = L - 14
        f[16], f[17] = tot >> 8, tot & 0xFF
        f[23] = 17
        f[24] = f[25] = 0
        # events: channels mostly in range, classes 0..7 (6, 7 out of range)
        nev = (L - (u - a) - 8) // 16
        for e in range(nev):
            p = u - a + 8 + 16 * e
            ch = int(rng.integers(0, 1600))
            f[p + 2], f[p + 3] = ch & 0xFF, ch >> 8
            f[p + 8] = int(rng.integers(0, 8))
        c = (~_csum16(f[14:14 + 4 * ihl])) & 0xFFFF
        f[24], f[25] = c >> 8, c & 0xFF
        ul = 8 + dl
        U = u - a
        f[U + 4], f[U + 5] = ul >> 8, ul & 0xFF
        f[U + 6] = f[U + 7] = 0
        if dl & 1 and rng.random() < 0.5:
            f[U + ul] = 0  # the byte past an odd datagram (read by the reference's sum)
        pseudo = np.concatenate([f[26:34], np.array([0, 17, ul >> 8, ul & 0xFF], np.uint8)])
        s = _csum16(np.concatenate([pseudo, f[U:U + ul]]))
        ck = (~s) & 0xFFFF or 0xFFFF
        r2 = rng.random()
        if r2 < 0.1:
            ck ^= 0x0101  # bad checksum
        elif r2 < 0.2:
            ck = 0  # no checksum
        f[U + 6], f[U + 7] = ck >> 8, ck & 0xFF
        desc["addr"][i] = a
        desc["len"][i] = L
    # the last frames' first lines run past the UMEM end (a0 + 128 > size)
    size = (int(desc["addr"][-1]) + 40 + 15) // 16 * 16  # (the ABI takes 16-B multiples)
    desc["len"][-1] = 40
    desc["addr"][-2] = size - 100
    desc["len"][-2] = 100
    return umem[:size].copy(), desc


FRAMES = {}


def frames(seed):
    if seed not in FRAMES:
        FRAMES[seed] = build_frames(3000, seed)
    return FRAMES[seed]


def _policy_or_skip(policy, monkeypatch):
    """Select a fused decode variant (read at queue creation); skip the case
    when this build does not hold it."""
    monkeypatch.setenv("DQDK_GPU_FUSED_POLICY", policy)
    try:  # (no histogram: nothing is allocated past the knob check)
        D.RxQueue(0, D.RxConfig(payloadsz=1458, flags=D.F_NO_HISTO), 1).close()
    except D.DqdkError as e:
        if "A/B variant" in str(e):
            pytest.skip(f"fused policy {policy} is not in this build (-DDQDK_AB_VARIANTS)")
        raise


@pytest.mark.parametrize("policy", ["3", "2", "6", "1", "4", "5", "7"])
@pytest.mark.parametrize("payloadsz", [1458, 48, 16])
@pytest.mark.parametrize("flags", [D.F_CSUM, 0], ids=["csum", "nocsum"])
def test_fused_first_line_handoff_vs_oracle(policy, payloadsz, flags, monkeypatch):
    _need_gpu()
    _policy_or_skip(policy, monkeypatch)
    umem, desc = frames(31)
    cfg = D.RxConfig(payloadsz=payloadsz, flags=flags | D.F_HISTO_PARTITIONED)
    ores, _ = compare(umem, desc, cfg, check_hist=True, records=False)
    st = ores["status"]
    assert (st == D.RX_OK).sum() > 1000
    if flags & D.F_CSUM:
        assert (st == D.RX_INVALID_UDP_CSUM).sum() > 50  # the fix-up takes staged keys back
    assert (ores["oob_events"] > 0).sum() > 100


def test_builder_frames_pass_the_oracle():
    """(CPU-side sanity of the builder above, run with the GPU tests.)"""
    umem, desc = frames(31)
    ores, _, _ = O.rx_batch(umem.copy(), desc, 1458, 3, D.F_CSUM)
    ok = ores["status"] == D.RX_OK
    assert ok.mean() > 0.6, np.unique(ores["status"], return_counts=True)


@pytest.mark.parametrize("fold", ["1", "0"])
@pytest.mark.parametrize("flags", [D.F_CSUM, D.F_CSUM | D.F_PREFILTER, 0], ids=["csum", "prefilter", "nocsum"])
def test_folded_counters_vs_oracle(fold, flags, monkeypatch):
    """The fused decode counts per-packet batches itself (per-block sums, the
    last block publishes; DQDK_GPU_FOLD=0: rx_abort + rx_count launches):
    every counter, cumulated over two batches, equals the oracle's."""
    _need_gpu()
    monkeypatch.setenv("DQDK_GPU_FOLD", fold)
    umem, desc = frames(31)
    cfg = D.RxConfig(payloadsz=1458, flags=flags | D.F_HISTO_PARTITIONED, port_start=0, port_end=65535)
    ores, ocnt, _ = O.rx_batch(umem.copy(), desc, cfg.payloadsz, cfg.mode, cfg.flags, cfg.port_start, cfg.port_end)
    q = D.RxQueue(0, cfg, len(desc))
    try:
        import torch
        d_umem = torch.from_numpy(umem).to("cuda:0")
        d_desc = torch.from_numpy(desc.view(np.uint8)).to("cuda:0")
        d_res = torch.empty(len(desc) * 8, dtype=torch.uint8, device="cuda:0")
        q.set_stream(torch.cuda.current_stream().cuda_stream)
        for _ in range(2):
            q.process_device(d_umem.data_ptr(), umem.nbytes, d_desc.data_ptr(), len(desc), d_res.data_ptr(), None)
        torch.cuda.synchronize()
        got = q.counters()
    finally:
        q.close()
    for k, v in ocnt.items():
        want = v if k == "first_abort_idx" else 2 * v
        assert got[k] == want, (k, got[k], want)
    assert ocnt["first_abort_idx"] < len(desc)
    if flags & D.F_CSUM:
        assert ocnt["invalid_udp_pkts"] > 0


@pytest.mark.parametrize("policy", ["2", "3", "1", "6"])
@pytest.mark.parametrize("fmap", ["1", "0"])
def test_frame_maps_vs_oracle(policy, fmap, monkeypatch):
    """Both frame maps of the fused decode (tile-major: a wave streams 64
    consecutive frames; interleaved: a block's waves stream 16 adjacent
    frames at a time), with the folded counters: results, counters (first
    failing frame included) and table equal the oracle's."""
    _need_gpu()
    _policy_or_skip(policy, monkeypatch)
    monkeypatch.setenv("DQDK_GPU_FRAME_MAP", fmap)
    umem, desc = frames(31)
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM | D.F_HISTO_PARTITIONED)
    ores, ocnt = compare(umem, desc, cfg, check_hist=True, records=False)
    assert ocnt["first_abort_idx"] < len(desc)


@pytest.mark.parametrize("flags", [D.F_CSUM, D.F_CSUM | D.F_CSUM_WRITEBACK, D.F_CSUM | D.F_PREFILTER],
                         ids=["csum", "writeback", "prefilter"])
@pytest.mark.parametrize("seed", [31, 47])
def test_decode_only_edge_frames_vs_oracle(flags, seed):
    """Decode-only batches (no histogram, no record buffer: BASELINE
    configs[1]'s form; the records-path decode streams every datagram for its
    checksum and decodes no event) on the edge frames above -- any byte
    offset, IP options, datagrams ending inside the first line, odd lengths,
    bad and absent checksums, first lines past the UMEM end: every result,
    every counter (and with writeback, every UMEM byte) equals the oracle's.
    (r06k: a first-line hand-off variant of this decode passed these too, and
    was slower.)"""
    _need_gpu()
    umem, desc = frames(seed)
    cfg = D.RxConfig(payloadsz=1458, flags=flags | D.F_NO_HISTO, port_start=0, port_end=65535)
    ores, ocnt = compare(umem, desc, cfg, check_hist=False, records=False)
    st = ores["status"]
    assert (st == D.RX_OK).sum() > 1000 and (st == D.RX_INVALID_UDP_CSUM).sum() > 50, np.unique(st, return_counts=True)
