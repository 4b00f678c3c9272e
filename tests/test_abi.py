"""The C-ABI library loads, exports every symbol include/dqdk_gpu.h declares,
and refuses to run without a gfx950 device (no CPU fallback)."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

import dqdk_amd as D
from dqdk_amd import _lib as L

ROOT = Path(__file__).resolve().parents[1]


def declared_symbols():
    txt = (ROOT / "include" / "dqdk_gpu.h").read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dqdk_(?:gpu|synth)_\w+)\s*\(", txt)))


def test_header_symbols_exported():
    syms = declared_symbols()
    assert len(syms) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", str(L.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (\w+)", out))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    # and the Python binding covers every declared entry point
    assert set(syms) == set(L.SIGNATURES), set(syms) ^ set(L.SIGNATURES)


def test_library_loads_and_reports_abi():
    lib = L.lib()
    assert lib.dqdk_gpu_abi_version() == 1
    for name in L.SIGNATURES:
        assert hasattr(lib, name)


def test_struct_layouts_match_header():
    assert C.sizeof(L.Desc) == 16          # struct xdp_desc
    assert C.sizeof(L.RxResult) == 8
    assert C.sizeof(L.Counters) == 12 * 8
    assert C.sizeof(L.Cfg) == 16
    assert C.sizeof(L.SynthCfg) == 24
    assert C.sizeof(L.FpCfg) == 32
    assert L.HISTO_ENTRIES * 4 == 2_378_170_368  # sizeof(tristan_histo_t), SURVEY §2.1


def test_no_device_means_enodev():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(D.DqdkError) as e:
        D.RxQueue(0, D.RxConfig(), 16)
    assert e.value.errno == 19  # ENODEV: no CPU implementation behind the ABI


def test_bad_arguments_are_einval():
    lib = L.lib()
    h = C.c_void_p()
    assert lib.dqdk_gpu_queue_create(0, None, 16, C.byref(h)) == -22
    cfg = L.Cfg(3392, 9, 0, 0, 0)  # bad mode
    assert lib.dqdk_gpu_queue_create(0, C.byref(cfg), 16, C.byref(h)) == -22
    assert lib.dqdk_gpu_rx_batch_device(None, None, 0, None, 0, None, None) == -22
    assert lib.dqdk_gpu_queue_destroy(None) == -22


def test_synth_is_deterministic_and_seeded():
    u1, d1 = D.synth_umem(256, 1500, 4096, faulty=True, threads=1)
    u2, d2 = D.synth_umem(256, 1500, 4096, faulty=True, threads=7)
    assert np.array_equal(u1, u2) and np.array_equal(d1, d2)
    u3, _ = D.synth_umem(256, 1500, 4096, faulty=True, seed=1)
    assert not np.array_equal(u1, u3)
    u4, _ = D.synth_umem(256, 1500, 4096, queue=1)
    assert not np.array_equal(u1, u4)
    # frame layout: ethertype, ihl 5, ports 5000+q -> 5000
    f = u4.reshape(256, 4096)[0]
    assert f[12] == 8 and f[13] == 0 and f[14] == 0x45 and f[23] == 17
    assert (int(f[34]) << 8 | int(f[35])) == 5001 and (int(f[36]) << 8 | int(f[37])) == 5000


def test_summary_line_matches_tristan_fini_format():
    c = [{"total_events": 91, "total_bytes": 1458, "rcvd_pkts": 1},
         {"total_events": 182, "total_bytes": 2916, "rcvd_pkts": 2}]
    s = D.tristan_summary(c, [1_500_000, 2_250_000], "/data/run1")
    # src/tristan.c:186-189
    want = ("{ \"total_received_events\": %llu,\"total_received_bytes\": %llu, \"total_received_packets\": %llu, "
            "\"dqdk_runtime_ms\": %.2lf, \"directory\": \"%s\"}").replace("%llu", "%d").replace("%.2lf", "%.2f") % (
        273, 4374, 3, 2.25, "/data/run1")
    assert s == want


def test_frame_processor_plugin_refuses_without_setup_or_device():
    """dqdk_gpu_frame_processor (the dqdk_frame_processor_t of src/dqdk.h:85)
    fails like a processor error before dqdk_gpu_fp_init, and the plugin
    cannot be set up without a gfx950 device (no CPU path behind it)."""
    import torch
    lib = L.lib()
    worker = C.create_string_buffer(64)  # any dqdk_worker address: the plugin keys on the pointer
    payload = C.create_string_buffer(1458)
    assert lib.dqdk_gpu_frame_processor(C.addressof(worker), payload, 1458) == -22
    assert lib.dqdk_gpu_fp_fini(None, -1, None) == -22
    assert lib.dqdk_gpu_fp_flush(None) == -22
    assert lib.dqdk_gpu_fp_init(None) == -22
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    cfg = L.FpCfg(L.Cfg(1458, L.MODE_ENERGYHISTO, 0, 0, 0), 0, 0, 0, 0)
    assert lib.dqdk_gpu_fp_init(C.byref(cfg)) == -19  # ENODEV
