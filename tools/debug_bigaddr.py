"""Probe: GPU verdicts for frames at UMEM offsets beyond 2 GiB."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np, torch
import dqdk_amd as D
from oracle import oracle as O

n = 1 << 20
umem, desc = D.synth_umem(n, 1500, 4096, faulty=False, threads=16)
dev = torch.device("cuda:0")
d_umem = torch.from_numpy(umem).to(dev)
# data integrity of the H2D copy
h = torch.from_numpy(umem[-(1 << 20):].copy()).to(dev)
print("tail equal:", bool(torch.equal(h, d_umem[-(1 << 20):])))
cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM)

def run(sub, base_ptr, size):
    d_desc = torch.from_numpy(sub.view(np.uint8).copy()).to(dev)
    m = len(sub)
    d_res = torch.zeros(m * 8, dtype=torch.uint8, device=dev)
    d_keys = torch.zeros(m * 91, dtype=torch.int32, device=dev)
    with D.RxQueue(0, cfg, m) as q:
        q.set_stream(torch.cuda.current_stream().cuda_stream)
        q.process_device(base_ptr, size, d_desc.data_ptr(), m, d_res.data_ptr(), d_keys.data_ptr())
        torch.cuda.synchronize()
    return d_res.cpu().numpy().view(D.RESULT_DTYPE)

res = run(desc, d_umem.data_ptr(), umem.nbytes)
bad = np.flatnonzero(res["status"] != 0)
print("bad frames:", len(bad), "first:", bad[:5], "addr of first:", desc["addr"][bad[:1]])
# same frames addressed relative to a base pointer 2 GiB in
off = 1 << 31
sub = desc[n // 2:].copy(); sub["addr"] -= off
res2 = run(sub, d_umem.data_ptr() + off, umem.nbytes - off)
print("rebased second half bad:", int((res2["status"] != 0).sum()))
# first-half frames but umem_size cut so remain < 2^31
sub = desc[:4096].copy()
res3 = run(sub, d_umem.data_ptr(), 1 << 30)
print("first frames with umem_size 1GiB bad:", int((res3["status"] != 0).sum()))
res4 = run(sub, d_umem.data_ptr(), (1 << 31) + 4096)
print("first frames with umem_size 2GiB+4K bad:", int((res4["status"] != 0).sum()))
res5 = run(sub, d_umem.data_ptr(), (1 << 31) - 4096)
print("first frames with umem_size 2GiB-4K bad:", int((res5["status"] != 0).sum()))
