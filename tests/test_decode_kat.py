"""Known-answer tests of the TRISTAN decode restatement.

src/tristan.c is unbuildable here (dqdk.h needs libbpf/libxdp headers), so the
decode is pinned by an INDEPENDENT restatement of `struct energy_evt`
(src/tristan.h:13-25, packed, little-endian, gcc bitfield order) written with
Python's struct module, plus hand-computed keys.
"""
import struct

import numpy as np

from oracle import oracle as O

CH, HC, BINS = 1512, 6, 65536


def pack_event(id_, channel, energy24, trigger, hist_class, reserved, mult, ts48):
    b8 = (hist_class & 7) | ((reserved & 0x1F) << 3)
    return (struct.pack("<HH", id_, channel) + (energy24 & 0xFFFFFF).to_bytes(3, "little")
            + bytes([trigger, b8, mult]) + (ts48 & ((1 << 48) - 1)).to_bytes(6, "little"))


def frame_with_events(events, extra=b""):
    payload = b"".join(events) + extra
    udplen = 8 + len(payload)
    tot = 20 + udplen
    f = bytearray(14 + tot)
    f[12:14] = b"\x08\x00"
    f[14] = 0x45
    f[16:18] = tot.to_bytes(2, "big")
    f[23] = 17
    f[34 + 4:34 + 6] = udplen.to_bytes(2, "big")
    f[42:] = payload
    return bytes(f)


def run(frames, payloadsz, mode=3):
    stride = 16384
    umem = np.zeros(stride * len(frames) + 65536, np.uint8)
    desc = np.zeros(len(frames), O.DESC_DTYPE)
    for i, f in enumerate(frames):
        umem[i * stride:i * stride + len(f)] = np.frombuffer(f, np.uint8)
        desc[i] = (i * stride, len(f), 0)
    hist = np.zeros(O.HISTO_ENTRIES, np.uint32)
    res, cnt, keys = O.rx_batch(umem, desc, payloadsz, mode, hist=hist)
    return res, cnt, keys, hist


def test_event_layout_is_16_bytes():
    assert len(pack_event(1, 2, 3, 4, 5, 6, 7, 8)) == 16


def test_keys_match_hand_computed_flat_index():
    evs = [
        pack_event(0, 0, 0x000000, 0, 0, 0, 0, 0),          # -> 0
        pack_event(1, 1511, 0xFFFFFF, 0xAA, 5, 31, 9, 1),    # last bin of last histogram
        pack_event(2, 7, 0x123456, 0, 3, 0, 0, 2),           # bin = energy >> 8 = 0x1234
        pack_event(3, 1512, 0x100, 0, 0, 0, 0, 3),           # channel OOB
        pack_event(4, 10, 0x100, 0, 6, 0, 0, 4),             # hist_class OOB
        pack_event(5, 10, 0x100, 0, 7, 31, 0, 5),            # hist_class OOB (reserved bits set)
        pack_event(6, 65535, 0xFFFFFF, 0xFF, 7, 31, 255, 6), # both OOB
        pack_event(7, 100, 0x0000FF, 0, 2, 31, 0, 7),        # low energy byte dropped -> bin 0
    ]
    res, cnt, keys, hist = run([frame_with_events(evs)], payloadsz=16 * len(evs))
    assert res["status"][0] == 0
    exp = [0, (1511 * HC + 5) * BINS + 0xFFFF, (7 * HC + 3) * BINS + 0x1234, 0xFFFFFFFF, 0xFFFFFFFF,
           0xFFFFFFFF, 0xFFFFFFFF, (100 * HC + 2) * BINS]
    assert list(keys) == exp
    assert cnt["oob_events"] == 4 and res["oob_events"][0] == 4
    assert cnt["total_events"] == 8  # tristan.c:328 counts OOB events too
    nz = np.flatnonzero(hist)
    assert sorted(nz.tolist()) == sorted(k for k in exp if k != 0xFFFFFFFF)
    assert hist[nz].sum() == 4


def test_E_comes_from_payloadsz_not_datalen():
    """tristan.c:311: nbEvents = payloadsz/16 even when the datagram is shorter."""
    evs = [pack_event(i, i, i << 8, 0, 0, 0, 0, i) for i in range(4)]
    f = frame_with_events(evs)
    res, cnt, keys, hist = run([f], payloadsz=16 * 6 + 15)  # E = 6 > 4 events present
    assert res["datalen"][0] == 64
    assert cnt["total_events"] == 6
    # events 4, 5 are read past the datagram: zero bytes -> key 0 (ch 0, hc 0, bin 0)
    assert list(keys[4:6]) == [0, 0]
    assert hist[0] == 1 + 2 and cnt["rcvd_bytes"] == 64


def test_listwave_and_waveform_decode_one_event():
    evs = [pack_event(i, 3, 0x200, 0, 1, 0, 0, i) for i in range(10)]
    f = frame_with_events(evs)
    res, cnt, keys, hist = run([f], payloadsz=160, mode=1)  # listwave: E = 1, histogram on
    assert cnt["total_events"] == 1 and hist.sum() == 1 and hist[(3 * HC + 1) * BINS + 2] == 1
    res, cnt, keys, hist = run([f], payloadsz=160, mode=0)  # waveform: E = 1, no histogram
    assert cnt["total_events"] == 1 and hist.sum() == 0


def test_counters_accumulate_u32_datalen():
    evs = [pack_event(0, 1, 0x100, 0, 0, 0, 0, 0)]
    f = frame_with_events(evs, extra=b"\x01" * 7)
    res, cnt, keys, hist = run([f, f, f], payloadsz=16)
    assert cnt["rcvd_bytes"] == 3 * 23 and cnt["total_bytes"] == 3 * 23
    assert hist[(1 * HC) * BINS + 1] == 3
