"""Probe: decoded records vs the oracle on a full-size faulty 9000-B batch."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np, torch
import dqdk_amd as D
from oracle import oracle as O

L, stride, pay = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
n = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 20
faulty = True
umem, desc = D.synth_umem(n, L, stride, faulty=faulty, threads=16)
cfg = D.RxConfig(payloadsz=pay, flags=D.F_CSUM)
E = cfg.events
dev = torch.device("cuda:0")
d_umem = torch.from_numpy(umem).to(dev)
d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
d_res = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
d_keys = torch.full((n * E,), -1, dtype=torch.int32, device=dev)
with D.RxQueue(0, cfg, n) as q:
    q.set_stream(torch.cuda.current_stream().cuda_stream)
    q.process_device(d_umem.data_ptr(), umem.nbytes, d_desc.data_ptr(), n, d_res.data_ptr(), d_keys.data_ptr())
    torch.cuda.synchronize()
res = d_res.cpu().numpy().view(D.RESULT_DTYPE)
keys = d_keys.cpu().numpy().view(np.uint32).reshape(n, E)
ok = res["status"] == 0
none_frac = np.zeros(n); none_frac[ok] = (keys[ok] == D.KEY_NONE).mean(axis=1)
print("OK frames", ok.sum(), "frames with >5% NONE records:", int((none_frac > 0.05).sum()))
hist = np.zeros(D.HISTO_ENTRIES, np.uint32)
with D.RxQueue(0, cfg, n) as q:
    pass
kk = keys[ok].ravel(); kk = kk[kk != D.KEY_NONE]
print("valid records", len(kk))
for hp in (0, D.F_HISTO_ATOMIC, D.F_HISTO_PARTITIONED, 0, D.F_HISTO_PARTITIONED):
    c2 = D.RxConfig(payloadsz=pay, flags=D.F_CSUM | hp)
    with D.RxQueue(0, c2, n) as q:
        q.set_stream(torch.cuda.current_stream().cuda_stream)
        q.process_device(d_umem.data_ptr(), umem.nbytes, d_desc.data_ptr(), n, d_res.data_ptr(), d_keys.data_ptr())
        torch.cuda.synchronize()
        h = q.histogram()
    print("path", hp, "mass", int(h.astype(np.uint64).sum()))
    if hp == D.F_HISTO_PARTITIONED:
        b = np.bincount(kk >> 21, minlength=284); hb = np.add.reduceat(h.astype(np.uint64), np.arange(0, 284 << 21, 1 << 21))
        d = np.flatnonzero(b != hb[:284])
        print("buckets with wrong mass:", len(d), d[:20], "expected", b[d[:5]], "got", hb[d[:5]])
sub = np.sort(np.random.default_rng(1).choice(n, 2048, replace=False))
ores, _, okeys = O.rx_batch(umem, desc[sub], pay, flags=D.F_CSUM)
okk = ores["status"] == 0
print("status mismatches in sample:", int((res["status"][sub] != ores["status"]).sum()))
mm = (keys[sub][okk] != okeys.reshape(-1, E)[okk]).any(axis=1)
print("key-mismatching sampled frames:", int(mm.sum()), "of", int(okk.sum()))
if mm.any():
    f = sub[okk][mm][0]
    kk = keys[f]; ok_ = okeys.reshape(-1, E)[okk][mm][0]
    diff = np.flatnonzero(kk != ok_)
    print("frame", f, "first diff events", diff[:10], "count", len(diff), "gpu", kk[diff[:5]], "ref", ok_[diff[:5]])
