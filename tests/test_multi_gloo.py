"""World-size-2 rehearsal of the queue-per-GPU scale-out on
CPU with the gloo backend: the same dqdk_amd.multi functions bench.py and
fini() use over RCCL, fed with per-rank oracle results of each rank's own
RX queue (synthetic queue = rank).  The merged counters and table must
equal one run over the union of both queues' frames.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import dqdk_amd as D
from dqdk_amd import multi
from oracle import oracle as O

M = 1 << 22             # reduced table (keys folded mod M): the reduce is size-agnostic
CHUNK = (1 << 20) + 3   # ragged chunks exercise the chunk loop


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _queue_result(queue: int):
    umem, desc = D.synth_umem(1024, 1500, 4096, queue=queue, faulty=True)
    res, cnt, keys = O.rx_batch(umem, desc, 1458, D.MODE_ENERGYHISTO, D.F_CSUM)
    u, c = O.sparse_histogram(keys, res, 1458 // 16, None)
    table = np.zeros(M, np.uint32)
    np.add.at(table, u % M, c.astype(np.uint32))
    table[[5, M - 1]] = 0xFFFFFFFF  # both ranks: wraps to 0xFFFFFFFE
    return cnt, table


def _worker(rank: int, world: int, port: int, out: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        queues = multi.shard(2, rank, world)
        assert list(queues) == [rank]
        cnt, table = _queue_result(rank)
        total = multi.reduce_counters(cnt)
        t = torch.from_numpy(table.view(np.int32).copy())
        multi.reduce_histogram(t, dst=0, chunk=CHUNK)
        if rank == 0:
            np.save(out + ".npy", t.numpy().view(np.uint32))
            with open(out + ".json", "w") as f:
                json.dump(total, f)
    finally:
        dist.destroy_process_group()


def test_shard_partitions_units():
    for count in (0, 1, 7, 8, 1 << 20):
        for world in (1, 2, 3, 8):
            got = [list(multi.shard(count, r, world)) for r in range(world)]
            flat = [i for g in got for i in g]
            assert flat == list(range(count))
            assert max(map(len, got)) - min(map(len, got)) <= 1


def test_gloo_world2_merge_equals_union(tmp_path):
    out = str(tmp_path / "merged")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    merged = np.load(out + ".npy")
    total = json.load(open(out + ".json"))
    c0, t0 = _queue_result(0)
    c1, t1 = _queue_result(1)
    np.testing.assert_array_equal(merged, t0 + t1)  # u32 wrap
    assert merged[5] == 0xFFFFFFFE and merged[M - 1] == 0xFFFFFFFE
    for f in D._lib.COUNTER_FIELDS:
        want = max(c0[f], c1[f]) if f == "first_abort_idx" else c0[f] + c1[f]
        assert total[f] == want, f
    s = D.tristan_summary([total], [0], "/tmp")
    assert f'"total_received_packets": {c0["rcvd_pkts"] + c1["rcvd_pkts"]}' in s


class _HostQueue:
    """The part of RxQueue that multi.fini touches, over one rank's oracle
    results (counters, an M-bin table) -- no GPU.  Its CSV is tristan_fini's
    format (src/tristan.c:197-216) of whatever table it holds at the time."""

    def __init__(self, queue: int):
        self.device = 0
        self.cfg = D.RxConfig(payloadsz=1458, mode=D.MODE_ENERGYHISTO, flags=D.F_CSUM)
        self._cnt, self._table = _queue_result(queue)
        self.csv_calls = 0

    def counters(self):
        return dict(self._cnt)

    def histogram(self):
        return self._table.copy()

    def load_histogram(self, table):
        self._table = table.copy()

    def write_histogram_csv(self, fd):
        self.csv_calls += 1
        text = _csv(self._table).encode()
        os.write(fd, text)
        return len(text)


def _csv(table: np.ndarray) -> str:
    nz = np.flatnonzero(table)
    out = ["Channel,Histo,Energy,Freq\n"]
    for k in nz.tolist():
        ch, rest = divmod(k, 6 * 65536)
        h, e = divmod(rest, 65536)
        out.append("%d,%d,%u,%u\n" % (ch, h, e, int(table[k])))
    return "".join(out)


def _fini_worker(rank: int, world: int, port: int, out: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q = _HostQueue(rank)
        line = multi.fini(q, runtime_ns=1_000_000 * (rank + 1), directory="/data/run",
                          histo_path=out + ".csv" if rank == 0 else out + f".rank{rank}.csv")
        with open(out + f".r{rank}.json", "w") as f:
            json.dump({"line": line, "csv_calls": q.csv_calls}, f)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_fini_writes_the_union(tmp_path):
    """multi.fini over gloo, world 2, histo_path set on both ranks: the
    counters are summed (first_abort_idx: max), the runtime is the longest
    rank's, the tables are SUM-reduced into rank 0's queue, and only rank 0
    writes the CSV and returns the controller line.  The CSV equals the file
    of the union of both queues' frames; the line carries the union's totals."""
    out = str(tmp_path / "fini")
    mp.start_processes(_fini_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    r0 = json.load(open(out + ".r0.json"))
    r1 = json.load(open(out + ".r1.json"))
    assert r1["line"] is None and r1["csv_calls"] == 0 and not os.path.exists(out + ".rank1.csv")
    assert r0["csv_calls"] == 1
    c0, t0 = _queue_result(0)
    c1, t1 = _queue_result(1)
    assert open(out + ".csv").read() == _csv(t0 + t1)
    total = {f: (max(c0[f], c1[f]) if f == "first_abort_idx" else c0[f] + c1[f]) for f in D._lib.COUNTER_FIELDS}
    assert r0["line"] == D.tristan_summary([total], [2_000_000], "/data/run")
    assert f'"total_received_packets": {c0["rcvd_pkts"] + c1["rcvd_pkts"]}' in r0["line"]
