"""Data-parallel training: bucketed gradient all-reduce overlapped with the HIP reverse pass.

Replaces ``DDP(model, device_ids=[local_rank], broadcast_buffers=False)``
(reference core/trainer.py:168-169) and the process topology of core/launch.py:37-145:
one process per GPU, ``torch.distributed`` with the "nccl" backend (RCCL on ROCm) over
xGMI.

The reverse pass (yolox_amd.train) writes every parameter gradient into one flat fp32
buffer, parameters in reverse registration order.  ``GradReducer`` cuts that buffer into
contiguous buckets; as soon as the last gradient of a bucket has been *enqueued* on the
compute stream, an event is recorded there and the bucket's all-reduce is issued from a
side stream that waits on the event -- the collective runs on RCCL's stream while the
compute stream continues with the next layers' gradients.  Buckets are launched strictly
in index order, which is the same on every rank because every rank replays the same tape,
so the collective sequence matches across ranks.  ``finish`` makes the compute stream wait
for the collectives and scales by 1/world (the mean of DDP).

Semantics kept from the reference: per-rank ``num_fg`` normalisation of the loss (no
all-reduce of num_fg), ``broadcast_buffers=False`` (BN running statistics stay
rank-local), parameters broadcast from rank 0 at wrap time (DDP's constructor does).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn


class _CudaOps:
    """The stream operations GradReducer issues (tests substitute a recording fake)."""

    def current(self, device):
        return torch.cuda.current_stream(device)

    def new_stream(self, device):
        return torch.cuda.Stream(device)

    def record(self, stream):
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev

    def wait(self, stream, ev) -> None:
        stream.wait_event(ev)

    def all_reduce(self, t: torch.Tensor, stream, group):
        with torch.cuda.stream(stream):
            return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True)

    def scale(self, t: torch.Tensor, v: float) -> None:
        t.mul_(v)


class GradReducer:
    """Bucketed all-reduce over a flat gradient buffer.

    flat: 1-D fp32 tensor; params_in_order: the parameters laid out in ``flat`` (each a
    contiguous slice, in order); offsets: id(param) -> element offset.

    Ordering: a parameter is reported ready from the stream that wrote its gradient (the
    compute stream for BN / head parameters, the weight-gradient side stream for conv
    weights, yolox_amd.train).  Each ``ready`` records an event on the CURRENT stream for
    the parameter's bucket (one live event per (bucket, stream): a later record on the same
    stream covers the earlier writes), and a bucket's all-reduce waits on every one of them,
    so it never reads a gradient another stream is still writing -- wherever the bucket
    boundaries fall.
    """

    def __init__(self, flat: torch.Tensor, params_in_order, offsets: dict, bucket_mb: float = 8.0,
                 group=None, world: Optional[int] = None, ops=None):
        self.flat = flat
        self.group = group
        self.world = world if world is not None else dist.get_world_size(group)
        cap = max(1, int(bucket_mb * 1024 * 1024 / flat.element_size()))
        self.buckets: list[tuple[int, int]] = []
        self.bucket_of: dict[int, int] = {}
        sizes: list[int] = []
        start = cur = 0
        n_in = 0
        for p in params_in_order:
            off = offsets[id(p)]
            assert off == cur, "parameters must tile the flat buffer in order"
            if cur - start >= cap and n_in:
                self.buckets.append((start, cur))
                sizes.append(n_in)
                start, n_in = cur, 0
            self.bucket_of[id(p)] = len(self.buckets)
            n_in += 1
            cur += p.numel()
        if cur > start:
            self.buckets.append((start, cur))
            sizes.append(n_in)
        self.sizes = sizes
        self.ops = ops if ops is not None else (_CudaOps() if flat.is_cuda else None)
        self.side = self.ops.new_stream(flat.device) if self.ops is not None else None
        self.reset()

    def reset(self) -> None:
        self.pending = list(self.sizes)
        self.next = 0
        self.works: list = []
        self.launch_order: list[int] = []
        self.events: list[dict] = [{} for _ in self.buckets]  # bucket -> {stream: latest event}

    def ready(self, p: nn.Parameter) -> None:
        k = self.bucket_of.get(id(p))
        if k is None:
            return
        if self.ops is not None:
            s = self.ops.current(self.flat.device)
            self.events[k][s] = self.ops.record(s)
        self.pending[k] -= 1
        while self.next < len(self.buckets) and self.pending[self.next] <= 0:
            self._launch(self.next)
            self.next += 1

    def _launch(self, k: int) -> None:
        s, e = self.buckets[k]
        t = self.flat[s:e]
        if self.ops is not None:
            if not self.events[k]:  # finish() of a bucket nobody reported: order after the caller
                cur = self.ops.current(self.flat.device)
                self.events[k][cur] = self.ops.record(cur)
            for ev in self.events[k].values():
                self.ops.wait(self.side, ev)
            w = self.ops.all_reduce(t, self.side, self.group)
        else:
            w = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self.works.append(w)
        self.launch_order.append(k)

    def finish(self) -> None:
        """Launch what is left (in order), make the compute stream wait, average."""
        while self.next < len(self.buckets):
            self._launch(self.next)
            self.next += 1
        for w in self.works:
            w.wait()  # NCCL: the current stream waits on RCCL's stream; gloo: blocks
        if self.world > 1:
            if self.ops is not None:
                self.ops.scale(self.flat, 1.0 / self.world)
            else:
                self.flat.mul_(1.0 / self.world)


class DistributedDataParallel(nn.Module):
    """Drop-in for ``torch.nn.parallel.DistributedDataParallel`` around a YoloxModule
    (trainer.py:168-169): same constructor arguments, ``.module`` attribute, forward
    passthrough; gradients are averaged over the process group during the HIP
    reverse pass (bucketed, overlapped)."""

    def __init__(self, module: nn.Module, device_ids=None, broadcast_buffers: bool = False,
                 bucket_cap_mb: float = 8.0, process_group=None, **_ignored):
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.bucket_cap_mb = bucket_cap_mb
        self.broadcast_buffers = broadcast_buffers
        # DDP's constructor: every rank starts from rank 0's parameters (and buffers)
        with torch.no_grad():
            for p in module.parameters():
                dist.broadcast(p.data, 0, group=process_group)
            for b in module.buffers():
                dist.broadcast(b.data, 0, group=process_group)
        self._reducer: Optional[GradReducer] = None
        self._graph_id = None

    def forward(self, *args, **kwargs):
        out = self.module(*args, **kwargs)
        if self.module.training:
            g = self.module._train_graph
            if self._reducer is None or self._graph_id != id(g):
                gb = g.grads
                self._reducer = GradReducer(gb.flat, gb.params, gb.offsets, self.bucket_cap_mb, self.process_group)
                self._graph_id = id(g)
            red = self._reducer
            red.reset()
            g.on_param_ready = red.ready
            g.on_backward_end = red.finish
        return out
