"""Queue-per-GPU scale-out: one process per GPU, no collective
on the data path, one merge at end of run.

The reference runs one worker pthread per RX queue (src/dqdk.c:517-620),
all of them incrementing ONE shared tristan_histo_t with relaxed atomics
(src/tristan.c:243) and summing per-worker dqdk_stats_t at exit
(src/tristan.c:177-183, src/dqdk.c dqdk_dump_stats).  Here each rank owns
its RX queues and a private device table; the only exchange is at fini:

* :func:`reduce_counters` -- sum of the per-rank counters (max for the
  per-batch diagnostic ``first_abort_idx``), like the per-worker stats sum;
* :func:`reduce_histogram` -- an integer SUM reduce of the per-rank tables to
  one rank, in chunks (u32 addition is the same bit pattern as int32
  wrap-around addition, so the merged table equals the shared atomic table);
* :func:`merge_queue_histogram` / :func:`fini` -- the same for a live
  :class:`~dqdk_amd.rx.RxQueue` on its GPU (RCCL over xGMI), then the
  tristan_fini outputs (JSON status line + histogram CSV) on the root rank.

The functions take torch tensors and use whatever backend the process
group has (``nccl`` = RCCL on GPU tensors, ``gloo`` on CPU tensors), so the
same code is exercised by the world_size-2 gloo tests on CPU.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import _lib as L

# 256 MB per collective: large enough to run xGMI links at bandwidth, small
# enough to bound the extra staging next to a 2.38 GB table.
REDUCE_CHUNK_ENTRIES = 64 << 20


def shard(count: int, rank: int, world: int) -> range:
    """Contiguous share of `count` independent units (queues, frames) for `rank`."""
    base, extra = divmod(count, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def reduce_counters(counters: dict, device: torch.device | str = "cpu", group=None) -> dict:
    """All-reduce one rank's counter dict (L.COUNTER_FIELDS) into the job total."""
    vals = [int(counters.get(f, 0)) for f in L.COUNTER_FIELDS]
    t = torch.tensor(vals, dtype=torch.int64, device=device)
    i_abort = L.COUNTER_FIELDS.index("first_abort_idx")
    mx = t[i_abort : i_abort + 1].clone()
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    t[i_abort] = mx[0]
    return {f: int(v) for f, v in zip(L.COUNTER_FIELDS, t.tolist())}


def reduce_histogram(table: torch.Tensor, dst: int = 0, group=None, chunk: int = REDUCE_CHUNK_ENTRIES) -> None:
    """In-place SUM reduce of an int32 view of a u32 table to rank `dst`, chunked."""
    if table.dtype != torch.int32 or not table.is_contiguous() or table.dim() != 1:
        raise ValueError("reduce_histogram needs a contiguous 1-D int32 view of the u32 table")
    for o in range(0, table.numel(), chunk):
        dist.reduce(table[o : o + chunk], dst=dst, op=dist.ReduceOp.SUM, group=group)


def merge_queue_histogram(q, dst: int = 0, group=None, buf: torch.Tensor | None = None) -> torch.Tensor:
    """Reduce every rank's queue table into rank `dst`'s queue table (RCCL).

    The queue's table is copied into a device buffer on the queue stream,
    reduced, and on `dst` written back (reset + add) so the queue's egress
    functions (histogram CSV) see the job-wide table.  Returns the buffer.
    """
    dev = torch.device("cuda", q.device)
    if buf is None:
        buf = torch.empty(L.HISTO_ENTRIES, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    prev = L.lib().dqdk_gpu_queue_stream(q.handle)
    q.sync()  # the queue's batches and staged slice passes are complete before the copy
    q.set_stream(s.cuda_stream)
    try:
        q.histogram_copy(buf.data_ptr())
        reduce_histogram(buf, dst=dst, group=group)
        if dist.get_rank(group) == dst:
            q.reset_histogram()
            q.histogram_add(buf.data_ptr())
        torch.cuda.synchronize(dev)
    finally:
        q.set_stream(prev or 0)
    return buf


def merge_queue_histogram_host(q, dst: int = 0, group=None) -> None:
    """merge_queue_histogram for a host-side process group (gloo): the table
    goes through host memory (``q.histogram()``), is SUM-reduced as an int32
    CPU tensor, and ``dst``'s queue takes the job-wide table back
    (``q.load_histogram``)."""
    import numpy as np

    t = torch.from_numpy(q.histogram().view(np.int32))
    reduce_histogram(t, dst=dst, group=group)
    if dist.get_rank(group) == dst:
        q.load_histogram(t.numpy().view(np.uint32))


def fini(q, runtime_ns: int, directory: str, histo_path: str | None = None, dst: int = 0, group=None) -> str | None:
    """tristan_fini across ranks (src/tristan.c:162-233): merged counters
    (sum; first_abort_idx max), the longest runtime, the merged histogram,
    the controller JSON line and the histogram CSV on `dst`.  Returns the
    JSON line on `dst`, None elsewhere.  The reductions run where the group's
    backend does: on the queue's GPU over RCCL (``nccl``), in host memory
    over ``gloo``."""
    from .rx import histo_enabled, tristan_summary

    on_gpu = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", q.device) if on_gpu else torch.device("cpu")
    total = reduce_counters(q.counters(), device=dev, group=group)
    rt = torch.tensor([runtime_ns], dtype=torch.int64, device=dev)
    dist.all_reduce(rt, op=dist.ReduceOp.MAX, group=group)
    has_histo = histo_enabled(q.cfg.mode, q.cfg.flags)  # is_store_histo (no table materialised)
    if has_histo:
        if on_gpu:
            merge_queue_histogram(q, dst=dst, group=group)
        else:
            merge_queue_histogram_host(q, dst=dst, group=group)
    if dist.get_rank(group) != dst:
        return None
    if has_histo and histo_path:
        fd = os.open(histo_path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        try:
            q.write_histogram_csv(fd)
            os.fsync(fd)
        finally:
            os.close(fd)
    return tristan_summary([total], [int(rt.item())], directory)
