"""Data-parallel reducer (yolox_amd.dp) on CPU with gloo, world size 2.

Checks the bucket layout, that buckets launch in index order no matter in which order
the reverse pass finishes parameters, that the result is the mean over ranks, and the
DDP-constructor broadcast of rank 0's parameters.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from yolox_amd.dp import DistributedDataParallel, GradReducer
        from yolox_amd.train import GradBuffer
        torch.manual_seed(rank)
        params = [nn.Parameter(torch.randn(n)) for n in (300, 5000, 70, 2000, 900, 10)]
        gb = GradBuffer(params, "cpu")
        red = GradReducer(gb.flat, gb.params, gb.offsets, bucket_mb=1000 * 4 / 2**20)
        # each rank writes rank-dependent gradients, finishing parameters out of order
        for p in gb.params:
            gb.of(p).fill_(float(rank + 1) * (1 + gb.offsets[id(p)] % 7))
        order = list(range(len(gb.params)))[::-1]
        for i in order:
            red.ready(gb.params[i])
        red.finish()
        # DDP-style wrapper: broadcast of rank 0's parameters at construction
        m = nn.Linear(4, 3)
        with torch.no_grad():
            m.weight.fill_(rank)
        DistributedDataParallel(m)
        q.put((rank, red.buckets, red.launch_order, gb.flat.tolist(), float(m.weight[0, 0])))
    finally:
        dist.destroy_process_group()


def test_grad_reducer_gloo_world2():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "pixeltable-yolox_amd"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, b0, o0, f0, w0), (_, b1, o1, f1, w1) = res
    assert b0 == b1 and len(b0) >= 3  # several contiguous buckets over the flat buffer
    assert all(b0[i][1] == b0[i + 1][0] for i in range(len(b0) - 1)) and b0[0][0] == 0
    assert o0 == o1 == sorted(o0)  # launched strictly in index order on both ranks
    f0, f1 = torch.tensor(f0), torch.tensor(f1)
    torch.testing.assert_close(f0, f1)
    # mean over ranks: (1 + 2) / 2 = 1.5 times the per-offset pattern
    assert torch.allclose(f0 / 1.5, torch.round(f0 / 1.5))
    assert w0 == w1 == 0.0


# ------------------------------------------------ stream ordering (production semantics, mocked)
class _Log:
    """Records what GradReducer issues per stream; NCCL semantics: ``work.wait()`` only makes
    the current stream wait (enqueues), it never blocks the host."""

    def __init__(self):
        self.ops = []  # (stream, kind, payload)
        self.cur = "main"
        self.nev = 0

    def emit(self, stream, kind, payload=None):
        self.ops.append((stream, kind, payload))
        return len(self.ops) - 1


class _FakeOps:
    def __init__(self, log):
        self.log = log

    def current(self, device):
        return self.log.cur

    def new_stream(self, device):
        return "rccl"

    def record(self, stream):
        self.log.nev += 1
        ev = ("ev", self.log.nev)
        self.log.emit(stream, "record", ev)
        return ev

    def wait(self, stream, ev):
        self.log.emit(stream, "wait", ev)

    def all_reduce(self, t, stream, group):
        log = self.log
        idx = log.emit(stream, "allreduce", (t.storage_offset(), t.storage_offset() + t.numel()))

        class _Work:
            def wait(self_inner):
                log.emit(log.cur, "wait_work", idx)
        return _Work()

    def scale(self, t, v):
        self.log.emit(self.log.cur, "scale", v)


def _happens_before(ops):
    """Transitive happens-before over the logged ops: program order per stream, record ->
    wait on events, all-reduce -> work wait."""
    n = len(ops)
    preds = [set() for _ in range(n)]
    last = {}
    rec = {}
    for i, (s, kind, pay) in enumerate(ops):
        if s in last:
            preds[i].add(last[s])
        last[s] = i
        if kind == "record":
            rec[pay] = i
        elif kind == "wait":
            preds[i].add(rec[pay])
        elif kind == "wait_work":
            preds[i].add(pay)
    before = [set() for _ in range(n)]
    for i in range(n):
        for p in preds[i]:
            before[i] |= before[p] | {p}
    return before


@pytest.mark.parametrize("bucket_elems", [1, 40, 150, 10 ** 6])
def test_grad_reducer_orders_allreduce_after_every_writer_stream(bucket_elems):
    """conv weights are written (and reported ready) on the weight-gradient side
    stream, BN / head parameters on the compute stream.  Whatever the bucket cuts, every
    bucket's all-reduce must come after every write into it on either stream, and the final
    1/world scaling after every all-reduce -- with ``work.wait()`` that only enqueues."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "pixeltable-yolox_amd"))
    from yolox_amd.dp import GradReducer
    from yolox_amd.train import GradBuffer
    # registration order per layer: conv.weight, bn.weight, bn.bias (the reverse pass finishes
    # bn first on the main stream, then issues the conv's weight gradient on the side stream)
    layers = [(64, 8), (36, 4), (128, 16), (9, 3), (300, 12)]
    params, kinds = [], {}
    for cw, cb in layers:
        for n, kind in ((cw, "wside"), (cb, "main"), (cb, "main")):
            p = nn.Parameter(torch.zeros(n))
            params.append(p)
            kinds[id(p)] = kind
    gb = GradBuffer(params, "cpu")
    log = _Log()
    red = GradReducer(gb.flat, gb.params, gb.offsets, bucket_mb=bucket_elems * 4 / 2 ** 20, world=2,
                      ops=_FakeOps(log))
    red.reset()
    mixed = False
    # reverse pass: layers last-to-first; per layer bn params (main) then the conv weight (side)
    for cw_i in range(len(layers) - 1, -1, -1):
        conv_w, bn_w, bn_b = params[3 * cw_i:3 * cw_i + 3]
        for p in (bn_w, bn_b, conv_w):
            s = kinds[id(p)]
            off = gb.offsets[id(p)]
            log.emit(s, "write", (off, off + p.numel()))
            log.cur = s
            red.ready(p)
            log.cur = "main"
    # backward end (train.py): the compute stream joins the side stream, then the reducer finishes
    log.cur = "wside"
    ev = _FakeOps(log).record("wside")
    log.cur = "main"
    log.emit("main", "wait", ev)
    red.finish()
    hb = _happens_before(log.ops)
    writes = [(i, pay) for i, (s, k, pay) in enumerate(log.ops) if k == "write"]
    reduces = [(i, pay) for i, (s, k, pay) in enumerate(log.ops) if k == "allreduce"]
    assert len(reduces) == len(red.buckets)
    for ri, (s, e) in reduces:
        streams = set()
        for wi, (ws, we) in writes:
            if ws < e and s < we:
                assert wi in hb[ri], f"all-reduce of [{s},{e}) may read the write [{ws},{we}) early"
                streams.add(log.ops[wi][0])
        mixed |= len(streams) > 1
    scale = [i for i, (s, k, _) in enumerate(log.ops) if k == "scale"]
    assert len(scale) == 1 and log.ops[scale[0]][0] == "main"
    assert all(ri in hb[scale[0]] for ri, _ in reduces)
    assert all(wi in hb[scale[0]] for wi, _ in writes)
    if bucket_elems < 10 ** 6:
        assert mixed or bucket_elems == 1  # the cuts put both streams' writes into one bucket
