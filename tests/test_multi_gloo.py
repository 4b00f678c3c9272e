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
