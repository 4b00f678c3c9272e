"""Probe: run 1500-B then 9000-B full-size batches in one process (the test's
order) and report frames whose records/results were not written."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np, torch
import dqdk_amd as D
from oracle import oracle as O

dev = torch.device("cuda:0")


def run(L, stride, pay, n=1 << 20):
    umem, desc = D.synth_umem(n, L, stride, faulty=True, threads=16)
    cfg = D.RxConfig(payloadsz=pay, flags=D.F_CSUM)
    E = cfg.events
    d_umem = torch.from_numpy(umem).to(dev)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    d_res = torch.full((n * 8,), 0xEE, dtype=torch.uint8, device=dev)  # poison: status 0xEE if unwritten
    d_keys = torch.full((n * E,), -1, dtype=torch.int32, device=dev)
    print("ptrs umem %x keys %x res %x" % (d_umem.data_ptr(), d_keys.data_ptr(), d_res.data_ptr()))
    with D.RxQueue(0, cfg, n) as q:
        q.set_stream(torch.cuda.current_stream().cuda_stream)
        q.process_device(d_umem.data_ptr(), umem.nbytes, d_desc.data_ptr(), n, d_res.data_ptr(), d_keys.data_ptr())
        torch.cuda.synchronize()
        h = q.histogram()
    res = d_res.cpu().numpy().view(D.RESULT_DTYPE)
    keys = d_keys.cpu().numpy().view(np.uint32).reshape(n, E)
    st = res["status"]
    unw = np.flatnonzero(st == 0xEE)
    ok = st == 0
    nrec = int((keys[ok] != D.KEY_NONE).sum())
    print(L, "unwritten results:", len(unw), "OK", int(ok.sum()), "records", nrec, "mass", int(h.astype(np.uint64).sum()))
    if len(unw):
        print("  first", unw[:16], "tiles", np.unique(unw // 256)[:10], "slot%4", np.bincount(unw % 256 % 4, minlength=4))
    part = ok & ((keys != D.KEY_NONE).sum(axis=1) < E - 40)
    pf = np.flatnonzero(part)
    print("  OK frames with many NONE records:", len(pf), pf[:10])
    if len(pf):
        f = pf[0]
        print("  frame", f, "NONE positions", np.flatnonzero(keys[f] == D.KEY_NONE)[:40])
        print("  tiles with such frames:", np.unique(pf // 256)[:20], "count tiles", len(np.unique(pf // 256)))
    sub = np.sort(np.random.default_rng(1).choice(n, 4096, replace=False))
    ores, _, okeys = O.rx_batch(umem, desc[sub], pay, flags=D.F_CSUM)
    print("  status mismatches in sample:", int((st[sub] != ores["status"]).sum()))
    del d_umem, d_keys, d_res, d_desc


run(1500, 4096, 1458)
run(9000, 9216, 8958)
run(9000, 9216, 8958)
