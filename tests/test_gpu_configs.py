"""BASELINE configs[3] and configs[4] on the device, against the oracle.

configs[3]: 4 RX queues sharded 1:1 to GPUs with mixed 1500/9000 B frames.
Each queue is a dqdk_gpu_queue with its own synthetic traffic (UDP source
port 5000 + q), its own counters and its own table (the per-worker state of
src/dqdk.c:517-620); the reference's one shared atomic table
(src/tristan.c:243) and per-worker stats sum (src/tristan.c:171-189) are the
end-of-run merge: histogram_copy / histogram_add (dqdk_amd.multi's RCCL
merge does the same per GPU) and multi's counter reduction.  Here the four
queues share the test box's one GPU; the code path per queue is the one a
4-GPU run takes.

configs[4]: the PCIe-inclusive replay (dqdk_amd.pipeline.E2EPipeline):
pinned host UMEM -> H2D on a side stream -> the full path -> D2H of the
per-frame results on a third stream, three slots in flight; every batch's
results as they land in host memory, and the final table, vs the oracle.
"""
import numpy as np
import pytest

import dqdk_amd as D
from oracle import oracle as O
from test_gpu_parity import _need_gpu

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

HOST_THREADS = 16


def merge_counters(per_queue: list[dict]) -> dict:
    """dqdk_amd.multi.reduce_counters' rule (sum; max of the per-batch
    diagnostic first_abort_idx) on host dicts."""
    out = {}
    for k in per_queue[0]:
        vals = [c[k] for c in per_queue]
        out[k] = max(vals) if k == "first_abort_idx" else sum(vals)
    return out


@pytest.mark.parametrize("records", [False, True], ids=["fused", "records"])
def test_configs3_four_queues_mixed_sizes_merged(records):
    _need_gpu()
    n, stride = 1 << 16, 9216  # 64K mixed frames per queue: 6M events, the partitioned path
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM)
    E = cfg.events
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    queues, gres, gcnt = [], [], []
    otable = np.zeros(D.HISTO_ENTRIES, np.uint32)  # the reference's one shared table
    ocnts = []
    try:
        for qid in range(4):
            umem, desc = D.synth_umem(n, 0, stride, queue=qid, faulty=True, threads=HOST_THREADS)
            assert len(np.unique(desc["len"])) >= 3  # 1500, 9000 and the short faulty frames
            q = D.RxQueue(0, cfg, n)
            queues.append(q)
            q.set_stream(s)
            d_umem = torch.from_numpy(umem).to(dev)
            d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
            d_res = torch.full((n * 8,), 0xEE, dtype=torch.uint8, device=dev)
            d_keys = torch.empty(n * E, dtype=torch.int32, device=dev) if records else None
            q.enable_timing(True)
            q.process_device(d_umem.data_ptr(), umem.nbytes, d_desc.data_ptr(), n, d_res.data_ptr(),
                             d_keys.data_ptr() if records else None)
            torch.cuda.synchronize()
            launched = {k for k, v in q.read_timing().items() if v["launches"]}
            # fused (no records): no rx_part1 (the decode takes back failed frames and adds its
            # overflow keys itself, or lists them for rx_fixup's grouping); records: rx_part1
            assert ("rx_part1" in launched) == records and "rx_part2" in launched, launched
            gres.append(d_res.cpu().numpy().view(D.RESULT_DTYPE))
            gcnt.append(q.counters())
            ores, ocnt, _ = O.rx_batch(umem, desc, cfg.payloadsz, cfg.mode, cfg.flags, want_keys=False, hist=otable,
                                       threads=HOST_THREADS)
            np.testing.assert_array_equal(gres[-1], ores)
            assert gcnt[-1] == ocnt, (qid, gcnt[-1], ocnt)
            ocnts.append(ocnt)
            del d_umem, d_desc, d_keys
        # end-of-run merge into queue 0's table
        buf = torch.empty(D.HISTO_ENTRIES, dtype=torch.int32, device=dev)
        for q in queues[1:]:
            q.histogram_copy(buf.data_ptr())
            queues[0].histogram_add(buf.data_ptr())
        torch.cuda.synchronize()
        del buf
        table = queues[0].histogram()
        assert np.array_equal(table, otable)
        total = merge_counters(gcnt)
        assert total == merge_counters(ocnts)
        line = D.tristan_summary(gcnt, [10**9] * 4, "/tmp")
        assert f'"total_received_packets": {total["rcvd_pkts"]}' in line
        assert f'"total_received_events": {total["total_events"]}' in line
    finally:
        for q in queues:
            q.close()


@pytest.mark.parametrize("records", [False, True], ids=["fused", "records"])
def test_configs4_e2e_pipeline_vs_oracle(records):
    """3 slots in flight, 9 batches of faulty frames replayed from 2 pinned
    host images: every batch's results (and records) as they reach host
    memory, the counters, and the table after the run == the oracle."""
    _need_gpu()
    from dqdk_amd.pipeline import E2EPipeline

    n, L, stride = 1 << 16, 1500, 4096  # 6M events per batch: the partitioned path
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM)
    E = cfg.events
    pl = E2EPipeline(0, cfg, n, L, stride, depth=3, images=2, records=records, faulty=True)
    try:
        expect = []
        for k in range(2):
            umem, desc = pl.image(k)
            ores, ocnt, okeys = O.rx_batch(umem, desc, cfg.payloadsz, cfg.mode, cfg.flags, threads=HOST_THREADS)
            expect.append((ores, ocnt, okeys))
        seen = []

        def on_result(b, res, keys):
            ores, _, okeys = expect[b % 2]
            np.testing.assert_array_equal(res, ores)
            if records:
                ok = ores["status"] == D.RX_OK
                np.testing.assert_array_equal(keys.reshape(n, E)[ok], okeys.reshape(n, E)[ok])
            seen.append(b)

        nb = 9
        r = pl.run(nb, on_result=on_result)
        assert seen == list(range(nb))
        assert r["packets"] == nb * n
        cnt = pl.q.counters()
        want = merge_counters([expect[b % 2][1] for b in range(nb)])
        want["first_abort_idx"] = expect[(nb - 1) % 2][1]["first_abort_idx"]  # the last batch's
        assert cnt == want, (cnt, want)
        table = pl.q.histogram()
        otable = np.zeros(D.HISTO_ENTRIES, np.uint64)
        for b in range(nb):
            ores, _, okeys = expect[b % 2]
            u, c = O.sparse_histogram(okeys, ores, E)
            otable[u] += c
        assert np.array_equal(table, otable.astype(np.uint32))
    finally:
        pl.close()


def test_configs4_eight_queues_paced_vs_oracle_of_union():
    """configs[4] short of 8 GPUs: eight E2EPipelines (RX queues 0..7, UDP
    source ports 5000..5007) share the box's one GPU, each on its own host
    thread (the reference's one worker pthread per queue, src/dqdk.c:491-515),
    replaying faulty 1500 B traffic paced at 100 Gbit/s aggregate
    (12.5 GB/s / 8 per queue).  Every batch's results as they land in host
    memory equal the oracle's; the eight per-queue tables merged
    (histogram_copy / histogram_add, the fini merge) equal the oracle of the
    union; the counters sum.  Prints the per-queue p99 batch latency."""
    _need_gpu()
    import json
    import threading

    from dqdk_amd.pipeline import E2EPipeline

    nq, n, L, stride, nb = 8, 1 << 16, 1500, 4096, 4  # 6M events per batch: the partitioned (fused) path
    cfg = D.RxConfig(payloadsz=1458, flags=D.F_CSUM)
    E = cfg.events
    pls, expect = [], []
    try:
        for q in range(nq):
            pl = E2EPipeline(0, cfg, n, L, stride, queue=q, depth=3, images=2, faulty=True)
            pls.append(pl)
            ex = []
            for k in range(2):
                umem, desc = pl.image(k)
                ores, ocnt, okeys = O.rx_batch(umem, desc, cfg.payloadsz, cfg.mode, cfg.flags, threads=HOST_THREADS)
                ex.append((ores, ocnt, okeys))
            expect.append(ex)
        rate = 100e9 / 8 / nq  # bytes per second per queue
        out, errs = [None] * nq, []

        def worker(q):
            seen = []

            def on_result(b, res, _keys):
                np.testing.assert_array_equal(res, expect[q][b % 2][0])
                seen.append(b)
            try:
                r = pls[q].run(nb, rate, on_result=on_result)
                assert seen == list(range(nb)), seen
                out[q] = r
            except BaseException as e:  # re-raised on the main thread
                errs.append((q, e))
        th = [threading.Thread(target=worker, args=(q,)) for q in range(nq)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        assert not any(t.is_alive() for t in th), "a queue thread hung"
        if errs:
            raise errs[0][1]
        # counters per queue, then summed (tristan_fini's totals)
        gcnt = [pl.q.counters() for pl in pls]
        for q in range(nq):
            want = merge_counters([expect[q][b % 2][1] for b in range(nb)])
            want["first_abort_idx"] = expect[q][(nb - 1) % 2][1]["first_abort_idx"]
            assert gcnt[q] == want, (q, gcnt[q], want)
        # the eight tables merged into queue 0's == the oracle of the union
        dev = torch.device("cuda:0")
        buf = torch.empty(D.HISTO_ENTRIES, dtype=torch.int32, device=dev)
        for pl in pls[1:]:
            pl.q.histogram_copy(buf.data_ptr())
            pl.q.sync()
            pls[0].q.histogram_add(buf.data_ptr())
            pls[0].q.sync()
        del buf
        table = pls[0].q.histogram()
        otable = np.zeros(D.HISTO_ENTRIES, np.uint64)
        for q in range(nq):
            for b in range(nb):
                ores, _, okeys = expect[q][b % 2]
                u, c = O.sparse_histogram(okeys, ores, E)
                otable[u] += c
        assert np.array_equal(table, otable.astype(np.uint32))
        p99 = [round(r["batch_latency_ms"]["p99"], 3) for r in out]
        print("configs4_8q " + json.dumps({
            "queues": nq, "frames_per_batch": n, "batches_per_queue": nb, "offered_Gbit_s": 100,
            "p99_batch_latency_ms": p99, "p50_batch_latency_ms": [round(r["batch_latency_ms"]["p50"], 3) for r in out],
            "Mpkt_s_per_queue": [round(r["Mpkt_s"], 3) for r in out]}), flush=True)
        assert max(p99) < 1000.0, p99
    finally:
        for pl in pls:
            pl.close()
