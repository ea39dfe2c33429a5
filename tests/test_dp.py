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
