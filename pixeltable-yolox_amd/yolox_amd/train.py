"""Training step of YoloxModule on libyoloxhip.

Reference: ``YoloxModule.forward(x, targets)`` in train mode (yolox/models/yolox.py:72-92)
-> backbone (darknet.py:95-177, yolo_pafpn.py:83-116) -> ``YoloxHead.forward`` training
branch (yolo_head.py:161-182, get_output_and_grid :213-231) -> ``get_losses`` (:253-411)
and ``loss.backward()`` (trainer.py:112).

Every BaseConv runs as conv (MFMA, raw output) -> BatchNorm2d batch statistics
(yxh_bn_stats, running stats updated like torch) -> BN+act apply (+ Bottleneck
residual); the head's preds write raw rows of [B, A, 5+C]; decode, SimOTA and the losses
run on the device without a host sync.  The forward records a tape of backward
closures; ``backward`` replays it in reverse:

* act + BN backward (yxh_bn_act_bwd) -> dgamma / dbeta straight into the gradient
  buffer, conv-output gradient in the compute dtype;
* weight gradient (yxh_conv_wgrad, MFMA, split over pixels);
* data gradient = a forward conv with transposed, flipped weights
  (yxh_pack_dgrad_weight; stride 2 via a zero-dilated source) accumulating into the
  fp32 gradient of each input view; nearest-x2 sources through yxh_upsample_bwd;
* SPP max-pool backward (yxh_spp_bwd), residuals as plain adds;
* DWConv (yolox_nano): the depthwise conv forward on yxh_conv2d (groups = channels), its
  gradients on yxh_dw_wgrad / yxh_dw_dgrad.

Parameter gradients land in one flat fp32 buffer (``GradBuffer``) whose slices become
``param.grad``; a data-parallel reducer (yolox_amd.dp) can all-reduce it in buckets as
the reverse pass completes them (``on_param_ready``).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Callable, Optional, Sequence

import torch
import torch.nn as nn

from . import _native as N
from .models.losses import LOSS_KEYS
from .models.network import (BaseConv, Bottleneck, CspDarknet, CspLayer, DWConv, Focus, SPPBottleneck,
                             YoloPafpn, YoloxHead)

MAX_CHANNELS = 4096  # reduction workspace sizing (yolox_x: 1280)
WGRAD_WS_BYTES = 64 << 20  # = the launchers' largest cap on per-split partials (16 Mi floats, tiles 25-28)
DW_WS_BYTES = 16 << 20  # depthwise weight-gradient partials per stream (yolox_nano 640 batch 64: < 1 MiB)


class Act:
    """An NHWC activation: channels [coff, coff + ch) of storage ``t`` [B, h, w, Ct]."""

    __slots__ = ("t", "coff", "ch", "h", "w", "grad", "needs_grad")

    def __init__(self, t: torch.Tensor, coff: int, ch: int, needs_grad: bool = True):
        self.t, self.coff, self.ch = t, coff, ch
        self.h, self.w = t.shape[1], t.shape[2]
        self.grad: Optional[torch.Tensor] = None
        self.needs_grad = needs_grad

    def src(self, up: int = 0) -> N.Src:
        s = N.Src()
        s.ptr = self.t.data_ptr() + self.coff * self.t.element_size()
        s.channels, s.cstride = self.ch, self.t.shape[3]
        s.bstride = self.h * self.w * self.t.shape[3]
        s.h, s.w, s.upsample = self.h, self.w, up
        return s

    def ensure_grad(self) -> torch.Tensor:
        if self.grad is None:
            self.grad = torch.zeros(self.t.shape[0], self.h, self.w, self.ch, dtype=torch.float32,
                                    device=self.t.device)
        return self.grad

    def grad_target(self) -> tuple:
        """(gradient buffer, accumulate?) for a writer that covers every element: the first
        writer of the reverse pass stores into uninitialised memory instead of a zero fill +
        accumulate."""
        if self.grad is None:
            self.grad = torch.empty(self.t.shape[0], self.h, self.w, self.ch, dtype=torch.float32,
                                    device=self.t.device)
            return self.grad, False
        return self.grad, True


def dense_src(t: torch.Tensor, up: int = 0) -> N.Src:
    """View of a dense [B, h, w, C] tensor."""
    s = N.Src()
    s.ptr = t.data_ptr()
    s.channels = s.cstride = t.shape[3]
    s.bstride = t.shape[1] * t.shape[2] * t.shape[3]
    s.h, s.w, s.upsample = t.shape[1], t.shape[2], up
    return s


class GradBuffer:
    """One flat fp32 buffer holding every parameter gradient, parameters in reverse
    registration order (roughly the order the reverse pass finishes them)."""

    def __init__(self, params: Sequence[nn.Parameter], device):
        self.params = list(params)[::-1]
        self.offsets = {}
        off = 0
        for p in self.params:
            self.offsets[id(p)] = off
            off += p.numel()
        self.numel = off
        self.flat = torch.zeros(off, dtype=torch.float32, device=device)
        self.views = {id(p): self.flat[self.offsets[id(p)]:self.offsets[id(p)] + p.numel()].view_as(p)
                      for p in self.params}

    def of(self, p: nn.Parameter) -> torch.Tensor:
        return self.views[id(p)]

    def begin(self) -> Optional[torch.Tensor]:
        """Zero the buffer for a new reverse pass; returns what param.grad held if the
        gradients already live here (torch accumulates across backward calls)."""
        held = any(p.grad is not None and p.grad.data_ptr() == self.views[id(p)].data_ptr() for p in self.params)
        prev = self.flat.clone() if held else None
        self.flat.zero_()
        return prev

    def publish(self, prev: Optional[torch.Tensor]) -> None:
        if prev is not None:
            self.flat.add_(prev)
        for p in self.params:
            g = self.views[id(p)]
            if p.grad is None:
                p.grad = g
            elif p.grad.data_ptr() != g.data_ptr():
                p.grad.add_(g)


# Tiles of the training convolutions, picked on the device the first time a shape runs
# (HIP events around each candidate, outputs redirected to scratch) and cached for the
# process.  Forward/data-gradient convs: the conv_igemm, conv_glds and conv_rows
# families, plus the conv_r3h tiles on fp32 (tile codes as engine.TILE_CANDIDATES); weight
# gradients: yxh_wgrad_desc
# tiles 1-10.  YOLOX_AMD_TRAIN_TUNE=0 keeps the by-shape defaults.
_BASE_TILES = [2 * i + k for i in list(range(1, 10)) + list(range(17, 26)) + list(range(33, 52)) for k in (0, 1)]
# 16-bit (autocast) steps also try the inference path's 16-bit kernels for the forward convs: dense
# 1x1 conv_pwf (97-104), weight-stationary 3x3 conv_ws (161-190, 261-280: yolox_x / yolox_l widths) and
# 1x1 conv_ws1 (201-210); of those conv_ws's fp32-gradient tiles (281-288, stride-1 3x3s) and conv_pwf
# (1x1s, round 5) take the data gradient's fp32-accumulating form; stride-2 3x3 data gradients also try the
# parity-class tiles (217-220, dgrad_s2h: 1/2/2/4 taps instead of 9 over a zero-dilated dy)
CONV_TUNE_TILES = _BASE_TILES + ([] if os.environ.get("YOLOX_AMD_TRAIN_TILES16") == "base" else
                                 [2 * i for i in list(range(97, 105)) + list(range(161, 191)) + list(range(201, 211))
                                  + list(range(261, 290)) + list(range(217, 221))])
CONV_TUNE_TILES_F32 = _BASE_TILES + [2 * (112 + i) for i in (29, 30, 31, 32, 33, 38, 39, 40)] + [2 * i for i in range(211, 217)]
WGRAD_TUNE_TILES = list(range(1, 11)) + list(range(11, 17)) + list(range(17, 25)) + list(range(25, 31))
_TRAIN_TILES: dict = {}
# YOLOX_AMD_TUNE_CHECK_DET=1 (tests): every applicable candidate also runs twice into a zeroed sink and
# must write the same bytes both times; (shape key, tile) pairs that do not are collected here
_CHECK_DET = os.environ.get("YOLOX_AMD_TUNE_CHECK_DET", "0") == "1"
TUNE_DET_FAILURES: list = []
TUNE_DET_CHECKED = [0]
# diagnostic (tools/train_shapes.py): every conv / wgrad launch of the training step, in order
_LAUNCH_LOG: Optional[list] = [] if os.environ.get("YOLOX_AMD_TRAIN_LOG") else None


def _src_key(s: N.Src) -> tuple:
    return (s.channels, s.cstride, s.h, s.w, s.upsample)


class TrainGraph:
    """Executes one training forward (recording the tape) and its backward."""

    def __init__(self, model, dtype: torch.dtype):
        if dtype not in (torch.float32, torch.bfloat16, torch.float16):
            raise ValueError(f"compute dtype {dtype} not supported")
        self.model = model
        self.dtype = dtype
        self.dcode = N.DTYPE_CODE[dtype]
        self.device = model.device
        self.lib = N.lib()
        self.esize = torch.empty((), dtype=dtype).element_size()
        self.grads = GradBuffer(model.parameters(), self.device)
        self.ws = torch.empty(int(self.lib.yxh_reduce_workspace_bytes(MAX_CHANNELS)), dtype=torch.uint8,
                              device=self.device)
        self.zero_bias = torch.zeros(MAX_CHANNELS, dtype=torch.float32, device=self.device)
        self.tape: list[Callable[[], None]] = []
        self.on_param_ready: Optional[Callable[[nn.Parameter], None]] = None
        self.on_backward_end: Optional[Callable[[], None]] = None  # e.g. GradReducer.finish
        self._fwd_w: dict = {}
        self.grad_total = torch.ones((), dtype=torch.float32, device=self.device)
        self.tune = os.environ.get("YOLOX_AMD_TRAIN_TUNE", "1") != "0"
        self._scratch = torch.empty(0, dtype=torch.uint8, device=self.device)
        # weight gradients run on a side stream beside the data-gradient chain (YOLOX_AMD_WGRAD_STREAM=0: inline)
        self._wside = (torch.cuda.Stream(self.device) if os.environ.get("YOLOX_AMD_WGRAD_STREAM", "1") != "0"
                       and self.device.type == "cuda" else None)
        # per-split partial weight gradients of the fp32 wgrad tiles (summed in a fixed order); the
        # launcher uses at most 16 MiB of partials, 64 MiB for the 16-bit nine-tap tiles 25-28
        # (csrc/train.hip ws_cap_splits; a weight too large
        # for one split falls back to fp32 atomics).  One workspace per stream that issues
        # weight gradients (head preds: main stream; BaseConvs: the side stream), so work in
        # flight on one stream never shares partials with the other.
        self.wg_ws = torch.empty(WGRAD_WS_BYTES, dtype=torch.uint8, device=self.device)
        self.wg_ws_side = (torch.empty(WGRAD_WS_BYTES, dtype=torch.uint8, device=self.device)
                           if self._wside is not None else self.wg_ws)
        self._scratch_side = torch.empty(0, dtype=torch.uint8, device=self.device)
        self._wpending: list = []
        self._segcap = None  # CapturedTrainStep's segment recorder while it captures
        # weight-gradient convs per side-stream fork (YOLOX_AMD_WGRAD_GROUP; round 6: 3 -- the captured configs[2]
        # step 535-536 -> 543-546 img/s over three alternating A/Bs (fewer cross-stream edges), configs[4] neutral)
        self.wgrad_group = max(1, int(os.environ.get("YOLOX_AMD_WGRAD_GROUP", "3")))
        # weight repacks: the first step launches one pack per conv (forward layout) and per
        # data-gradient input slice, recording each as a yxh_pack_job; later steps repack
        # everything in ONE yxh_pack_weights_batch launch at the start of the forward
        self._dgrad_w: dict = {}
        self._dgrad_ptrs: set = set()  # data pointers of the dgrad weight buffers (launch log only)
        self._pack_jobs: dict = {}  # key -> (PackJob, (weight, bias) tensors it reads)
        self._pack_table = None     # (device job table, njobs, total blocks, signature)
        self._batched = False       # this step's repacks were done by the batch launch
        self.batch_pack = os.environ.get("YOLOX_AMD_BATCH_PACK", "1") != "0"

    # ------------------------------------------------------------ helpers
    @property
    def stream(self) -> int:
        return N.stream_ptr(self.device)

    def _chk(self, rc, what):
        N.check(rc, what)

    def _ready(self, *params) -> None:
        if self.on_param_ready is not None:
            for p in params:
                self.on_param_ready(p)

    def _fwd_weight(self, conv: nn.Conv2d, cin_pad: int):
        """conv.weight -> [cout][kh][kw][cin_pad] compute dtype (+ fp32 bias)."""
        kh, kw = conv.kernel_size
        w = self._fwd_w.get(id(conv))
        if w is None:
            w = (torch.empty(conv.out_channels * kh * kw * cin_pad, dtype=self.dtype, device=self.device),
                 torch.empty(conv.out_channels, dtype=torch.float32, device=self.device))
            self._fwd_w[id(conv)] = w
        key = ("fwd", id(conv))
        if self._batched and key in self._pack_jobs:
            return w
        wt = conv.weight.detach()
        if wt.dtype != torch.float32:
            raise ValueError("training keeps fp32 master weights; the compute dtype comes from autocast")
        b = conv.bias.detach() if conv.bias is not None else None
        self._chk(self.lib.yxh_fold_bn_pack(
            wt.data_ptr(), b.data_ptr() if b is not None else None, None, None, None, None, 0.0,
            conv.out_channels, conv.in_channels // conv.groups, kh, kw, cin_pad, self.dcode, w[0].data_ptr(),
            w[1].data_ptr(), self.stream), "pack weights")
        job = N.PackJob(wt.data_ptr(), b.data_ptr() if b is not None else None, w[0].data_ptr(), w[1].data_ptr(),
                        N.PACK_FWD, conv.out_channels, conv.in_channels // conv.groups, kh, kw, cin_pad, 0, 0)
        self._pack_jobs[key] = (job, conv.out_channels * kh * kw * cin_pad, (conv.weight, conv.bias))
        self._pack_table = None  # a job the table lacks: rebuild it after this step
        return w

    # ------------------------------------------------------------ batched repacks
    def _pack_signature(self) -> tuple:
        return tuple((p.data_ptr() if p is not None else 0) for _, _, ts in self._pack_jobs.values() for p in ts)

    def _build_pack_table(self) -> None:
        """After a step that launched its repacks one by one: the job table for later steps."""
        jobs, block = [], 0
        for job, elems, _ in self._pack_jobs.values():
            job.block0 = block
            block += (elems + 255) // 256
            jobs.append(job)
        raw = (N.PackJob * len(jobs))(*jobs)
        table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        self._pack_table = (table, len(jobs), block, self._pack_signature())

    def _pack_all(self) -> None:
        """One launch for every repack of this step, when the recorded table still matches
        the parameters' storage; otherwise this step packs per conv (and re-records)."""
        self._batched = False
        t = self._pack_table
        if not self.batch_pack or t is None:
            return
        if t[3] != self._pack_signature():
            self._pack_table = None
            self._pack_jobs = {}
            return
        self._chk(self.lib.yxh_pack_weights_batch(t[0].data_ptr(), t[1], t[2], self.dcode, self.stream),
                  "pack weights (batch)")
        self._batched = True

    def _conv(self, srcs: list, cin: int, cout: int, k: int, stride: int, pad: int, weight: int, bias: int,
              dst: int, dst_f32: bool, dst_cs: int, dst_bs: int, in_h: int, in_w: int, out_h: int, out_w: int,
              batch: int, accumulate: bool = False, groups: int = 1) -> None:
        d = N.ConvDesc()
        d.dtype, d.batch = self.dcode, batch
        d.in_h, d.in_w, d.out_h, d.out_w = in_h, in_w, out_h, out_w
        d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups = cin, cout, k, k, stride, pad, groups
        d.nsrc = len(srcs)
        for j, s in enumerate(srcs):
            d.src[j] = s
        d.weight, d.bias = weight, bias
        d.dst = dst
        d.dst_dtype = N.F32 if dst_f32 else self.dcode
        d.dst_cstride, d.dst_bstride = dst_cs, dst_bs
        d.act = N.ACT_NONE
        d.flags = N.CONV_ACCUMULATE if accumulate else 0
        key = ("conv", self.dcode, batch, in_h, in_w, out_h, out_w, cin, cout, k, stride, pad, int(dst_f32),
               dst_cs, d.flags) + tuple(_src_key(q) for q in srcs)
        # depthwise convs have one kernel (dwconv): nothing to tune
        d.tile = 0 if groups != 1 else self._tile(key, d, self.lib.yxh_conv2d, "dst",
                                                  batch * dst_bs * (4 if dst_f32 else self.esize),
                                                  CONV_TUNE_TILES_F32 if self.dtype == torch.float32 else CONV_TUNE_TILES)
        self._chk(self.lib.yxh_conv2d(C.byref(d), self.stream), "conv")
        if _LAUNCH_LOG is not None:
            _LAUNCH_LOG.append(("dgrad" if weight in self._dgrad_ptrs else "conv", k, stride, cin, cout, in_h, in_w,
                                out_h, out_w, batch, d.tile, len(srcs), int(srcs[0].upsample), int(accumulate)))

    def _wgrad(self, srcs: list, cin: int, cin_store: int, cout: int, k: int, stride: int, pad: int, dy: N.Src,
               dw: torch.Tensor, in_h: int, in_w: int, out_h: int, out_w: int, batch: int) -> None:
        d = N.WgradDesc()
        d.dtype, d.batch = self.dcode, batch
        d.in_h, d.in_w, d.out_h, d.out_w = in_h, in_w, out_h, out_w
        d.cin, d.cout, d.kh, d.kw, d.stride, d.pad = cin, cout, k, k, stride, pad
        d.nsrc, d.cin_store = len(srcs), cin_store
        for j, s in enumerate(srcs):
            d.src[j] = s
        d.dy = dy
        d.dw = dw.data_ptr()
        side = self._wside is not None and torch.cuda.current_stream(self.device) == self._wside
        wsb = self.wg_ws_side if side else self.wg_ws
        d.workspace, d.workspace_bytes = wsb.data_ptr(), wsb.numel()
        key = ("wgrad", self.dcode, batch, in_h, in_w, out_h, out_w, cin, cin_store, cout, k, stride, pad,
               _src_key(dy)) + tuple(_src_key(q) for q in srcs)
        d.tile = self._tile(key, d, self.lib.yxh_conv_wgrad, "dw", cout * cin_store * k * k * 4, WGRAD_TUNE_TILES)
        self._chk(self.lib.yxh_conv_wgrad(C.byref(d), self.stream), "wgrad")
        if _LAUNCH_LOG is not None:
            _LAUNCH_LOG.append(("wgrad", k, stride, cin, cout, in_h, in_w, out_h, out_w, batch, d.tile, len(srcs),
                                int(srcs[0].upsample), 0))

    def _dw_wgrad(self, x: N.Src, dy: N.Src, C_: int, stride: int, out_h: int, out_w: int, batch: int,
                  dw: torch.Tensor) -> None:
        """Depthwise weight gradient (yxh_dw_wgrad): WRITTEN (not added) into the gradient buffer --
        safe because one reverse pass replays one tape, in which each depthwise weight is used by
        exactly one conv (GradBuffer.begin zeroes and publish adds what param.grad held, so torch's
        accumulation over backward calls still holds); its per-block partials go to a workspace of
        the issuing stream."""
        need = int(self.lib.yxh_dw_wgrad_workspace_bytes(batch, out_h, out_w, C_, 3))
        side = self._wside is not None and torch.cuda.current_stream(self.device) == self._wside
        name = "_dw_ws_side" if side else "_dw_ws"
        ws = getattr(self, name, None)
        if ws is None:  # one fixed workspace per stream (never re-allocated under pending work)
            ws = torch.empty(DW_WS_BYTES, dtype=torch.uint8, device=self.device)
            setattr(self, name, ws)
        if need > ws.numel():
            raise NotImplementedError(f"depthwise weight gradient needs {need} B of partials (> {DW_WS_BYTES})")
        self._chk(self.lib.yxh_dw_wgrad(self.dcode, batch, C.byref(x), C.byref(dy), C_, 3, stride, 1, out_h, out_w,
                                        dw.data_ptr(), ws.data_ptr(), ws.numel(), self.stream), "dw wgrad")

    def _side_wgrad(self, launch: Callable[[], None], dy: torch.Tensor, param: nn.Parameter) -> None:
        """A conv's weight gradient on the side stream: it needs only dy and the forward's input
        (both final by now) and nothing on the main stream reads dW before the backward ends, so
        it overlaps the data-gradient chain (the critical path) instead of sitting in it."""
        if self._wside is None:
            launch()
            self._ready(param)
            return
        self._wpending.append((launch, dy, param))
        if len(self._wpending) >= self.wgrad_group:
            self._flush_wgrad()

    def _flush_wgrad(self) -> None:
        """Issue the pending weight gradients on the side stream behind ONE fork from the main
        stream (YOLOX_AMD_WGRAD_GROUP convs per fork: fewer cross-stream edges in a captured step)."""
        if not self._wpending:
            return
        if self._segcap is not None:  # CapturedTrainStep: a side-stream graph segment of its own
            self._segcap.side(self._wpending)
            self._wpending = []
            return
        self._wside.wait_stream(torch.cuda.current_stream(self.device))  # dy written, dW zeroed
        with torch.cuda.stream(self._wside):
            for launch, _, param in self._wpending:
                launch()
                self._ready(param)  # DP: the bucket's event is recorded on this stream
        for _, dy, _ in self._wpending:
            dy.record_stream(self._wside)
        self._wpending = []

    def _tile(self, key: tuple, d, fn, out_field: str, out_bytes: int, candidates: list, reps: int = 3) -> int:
        """The cached tile for this shape, or the fastest candidate timed now (writing to
        scratch instead of ``out_field``); 0 (by shape) when tuning is off."""
        t = _TRAIN_TILES.get(key)
        if t is not None:
            return t
        if not self.tune or torch.cuda.is_current_stream_capturing():  # no timing inside a capture
            return 0
        stream = torch.cuda.current_stream(self.device)
        side = self._wside is not None and stream == self._wside  # each stream tunes into its own sink
        scratch = self._scratch_side if side else self._scratch
        if scratch.numel() < out_bytes:
            scratch = torch.empty(out_bytes, dtype=torch.uint8, device=self.device)
            if side:
                self._scratch_side = scratch
            else:
                self._scratch = scratch
        real = getattr(d, out_field)
        setattr(d, out_field, scratch.data_ptr())
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st, ref = self.stream, C.byref(d)
        best = (float("inf"), 0)
        try:
            for tile in candidates:
                d.tile = tile
                if fn(ref, st) != N.OK:  # variant not applicable to this shape
                    continue
                ev0.record(stream)
                for _ in range(reps):
                    fn(ref, st)
                ev1.record(stream)
                ev1.synchronize()
                ms = ev0.elapsed_time(ev1) / reps
                if ms < best[0]:
                    best = (ms, tile)
                if _CHECK_DET:
                    sink = scratch[:out_bytes]
                    sink.zero_()
                    fn(ref, st)
                    first = sink.clone()
                    sink.zero_()
                    fn(ref, st)
                    if not torch.equal(first, sink):
                        TUNE_DET_FAILURES.append((key, tile))
                    TUNE_DET_CHECKED[0] += 1
        finally:
            setattr(d, out_field, real)
        _TRAIN_TILES[key] = best[1]
        return best[1]

    def _dgrad(self, conv: nn.Conv2d, dy_t: torch.Tensor, cout_pad: int, inputs: list, batch: int) -> None:
        """Accumulate the data gradient of every input view that needs one.
        inputs: [(Act, upsample, channel offset in the conv's cin)]."""
        kh = conv.kernel_size[0]
        s = conv.stride[0]
        if s not in (1, 2):
            raise NotImplementedError("stride > 2")
        pad = kh - 1 - conv.padding[0]
        dy = dense_src(dy_t, up=2 if s == 2 else 0)
        for act, up, cb in inputs:
            if not act.needs_grad:
                continue
            cs = act.ch
            key = ("dgrad", id(conv), cb, cs, cout_pad)
            wt = self._dgrad_w.get(key)
            if wt is None:
                wt = torch.empty(cs * kh * kh * cout_pad, dtype=self.dtype, device=self.device)
                self._dgrad_w[key] = wt
                self._dgrad_ptrs.add(wt.data_ptr())
            if not (self._batched and key in self._pack_jobs):
                self._chk(self.lib.yxh_pack_dgrad_weight(
                    conv.weight.detach().data_ptr(), conv.out_channels, conv.in_channels, kh, kh, cb, cs, cout_pad,
                    self.dcode, wt.data_ptr(), self.stream), "pack dgrad")
                job = N.PackJob(conv.weight.detach().data_ptr(), None, wt.data_ptr(), None, N.PACK_DGRAD,
                                conv.out_channels, conv.in_channels, kh, kh, cout_pad, cb, cs)
                self._pack_jobs[key] = (job, cs * kh * kh * cout_pad, (conv.weight,))
                self._pack_table = None
            in_h, in_w = act.h << up, act.w << up  # the conv's logical input size
            if up:  # the conv writes every element of the temporary; upsample_bwd accumulates
                dst, acc = torch.empty(batch, in_h, in_w, cs, dtype=torch.float32, device=self.device), False
            else:
                dst, acc = act.grad_target()
            self._conv([dy], cout_pad, cs, kh, 1, pad, wt.data_ptr(), self.zero_bias.data_ptr(), dst.data_ptr(),
                       True, cs, in_h * in_w * cs, in_h, in_w, in_h, in_w, batch, accumulate=acc)
            if up:
                g = act.ensure_grad()
                self._chk(self.lib.yxh_upsample_bwd(dst.data_ptr(), batch, act.h, act.w, cs, g.data_ptr(),
                                                    self.stream), "upsample bwd")

    # ------------------------------------------------------------ layers
    def base_conv(self, m: BaseConv, inputs: list, out: Optional[Act] = None, residual: Optional[Act] = None,
                  cin_store: Optional[int] = None) -> Act:
        """BaseConv.forward (network_blocks.py:48-49) in train mode; inputs: [(Act,
        upsample)] concatenated along channels (torch.cat order).  A DWConv (:55-74, yolox_nano)
        is its depthwise BaseConv (groups = channels) then its pointwise one."""
        if isinstance(m, DWConv):
            t = self.base_conv(m.dconv, inputs)
            return self.base_conv(m.pconv, [(t, 0)], out=out, residual=residual)
        conv, bn = m.conv, m.bn
        B = inputs[0][0].t.shape[0]
        cin = sum(a.ch for a, _ in inputs)
        k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        in_h, in_w = inputs[0][0].h << inputs[0][1], inputs[0][0].w << inputs[0][1]
        oh, ow = (in_h + 2 * p - k) // s + 1, (in_w + 2 * p - k) // s + 1
        cout = conv.out_channels
        dw = conv.groups != 1  # depthwise: groups == cin == cout, one un-upsampled source
        if dw and not (conv.groups == cin == cout and len(inputs) == 1 and inputs[0][1] == 0 and k == 3 and p == 1):
            raise NotImplementedError("grouped convs other than a 3x3 depthwise conv over one source")
        if dw and (cout * self.esize) % 16:
            # yxh_dw_dgrad reads dy as 16-byte pixel rows (train_dw.hip dw_dgrad_launch); the yolox_nano /
            # yolox_tiny widths all meet this
            raise NotImplementedError(f"depthwise conv training needs channels % {16 // self.esize} == 0 "
                                      f"(16-byte gradient rows), got {cout}")
        w, _ = self._fwd_weight(conv, 1 if dw else cin)
        srcs = [a.src(up) for a, up in inputs]
        y = torch.empty(B, oh, ow, cout, dtype=self.dtype, device=self.device)
        self._conv(srcs, cin, cout, k, s, p, w.data_ptr(), self.zero_bias.data_ptr(), y.data_ptr(), False, cout,
                   oh * ow * cout, in_h, in_w, oh, ow, B, groups=conv.groups)
        stats = torch.empty(4, cout, dtype=torch.float32, device=self.device)
        ys = dense_src(y)
        self._chk(self.lib.yxh_bn_stats(
            self.dcode, B, C.byref(ys), bn.weight.detach().data_ptr(), bn.bias.detach().data_ptr(),
            bn.running_mean.data_ptr(), bn.running_var.data_ptr(), float(bn.eps), float(bn.momentum),
            stats.data_ptr(), self.ws.data_ptr(), self.ws.numel(), self.stream), "bn stats")
        self._bn_counters.append(bn.num_batches_tracked)  # += 1 for all BNs in one launch (forward end)
        if out is None:
            out = Act(torch.empty(B, oh, ow, cout, dtype=self.dtype, device=self.device), 0, cout)
        os_ = out.src()
        rs = residual.src() if residual is not None else None
        act = N.ACT_CODE[getattr(m, "act_name", "silu")]
        self._chk(self.lib.yxh_bn_act_fwd(self.dcode, B, C.byref(ys), stats.data_ptr(), act,
                                          C.byref(rs) if rs is not None else None, C.byref(os_), self.stream),
                  "bn act fwd")
        cin_store = cin_store or cin

        def backward():
            if out.grad is None:  # output unused by the loss
                return
            assert y.data_ptr() == ys.ptr  # the closure holds y: ys is a raw pointer into it
            dy = torch.empty(B, oh, ow, cout, dtype=self.dtype, device=self.device)
            go = dense_src(out.grad)
            gb = self.grads
            self._chk(self.lib.yxh_bn_act_bwd(
                self.dcode, B, C.byref(ys), C.byref(go), stats.data_ptr(), bn.weight.detach().data_ptr(), act,
                gb.of(bn.weight).data_ptr(), gb.of(bn.bias).data_ptr(), dy.data_ptr(), self.ws.data_ptr(),
                self.ws.numel(), self.stream), "bn act bwd")
            self._ready(bn.weight, bn.bias)
            if residual is not None and residual.needs_grad:
                if residual.grad is None:  # first writer: take over out.grad (consumed above)
                    residual.grad = out.grad
                else:
                    residual.grad.add_(out.grad)
            if dw:  # depthwise gradients: yxh_dw_wgrad (side stream) and yxh_dw_dgrad
                self._side_wgrad(lambda: self._dw_wgrad(srcs[0], dense_src(dy), cout, s, oh, ow, B,
                                                        gb.of(conv.weight)), dy, conv.weight)
                a = inputs[0][0]
                if a.needs_grad:
                    g, acc = a.grad_target()
                    self._chk(self.lib.yxh_dw_dgrad(self.dcode, B, C.byref(dense_src(dy)), w.data_ptr(), cout, k, s, p,
                                                    in_h, in_w, g.data_ptr(), a.ch, in_h * in_w * a.ch, int(acc),
                                                    self.stream), "dw dgrad")
                return
            self._side_wgrad(lambda: self._wgrad(srcs, cin, cin_store, cout, k, s, p, dense_src(dy), gb.of(conv.weight),
                                                 in_h, in_w, oh, ow, B), dy, conv.weight)
            off, ins = 0, []
            for a, up in inputs:
                ins.append((a, up, off))
                off += a.ch
            self._dgrad(conv, dy, cout, ins, B)

        self.tape.append(backward)
        return out

    def bottleneck(self, b: Bottleneck, x: Act) -> Act:
        # network_blocks.py:95-99
        t = self.base_conv(b.conv1, [(x, 0)])
        return self.base_conv(b.conv2, [(t, 0)], residual=x if b.use_add else None)

    def csp(self, m: CspLayer, inputs: list) -> Act:
        # network_blocks.py:176-183
        x1 = self.base_conv(m.conv1, inputs)
        x2 = self.base_conv(m.conv2, inputs)
        for b in m.m:
            x1 = self.bottleneck(b, x1)
        return self.base_conv(m.conv3, [(x1, 0), (x2, 0)])

    def spp(self, m: SPPBottleneck, inputs: list) -> Act:
        # network_blocks.py:137-142: x -> cat[x, mp5(x), mp9(x), mp13(x)] in one buffer
        x0 = inputs[0][0]
        B = x0.t.shape[0]
        c = m.conv1.conv.out_channels
        h, w = x0.h << inputs[0][1], x0.w << inputs[0][1]
        cat = torch.empty(B, h, w, 4 * c, dtype=self.dtype, device=self.device)
        x = self.base_conv(m.conv1, inputs, out=Act(cat, 0, c))
        self._chk(self.lib.yxh_spp_maxpool(cat.data_ptr(), self.dcode, B, h, w, c, 4 * c, h * w * 4 * c,
                                           self.stream), "spp")
        cat_act = Act(cat, 0, 4 * c)

        def backward():
            if cat_act.grad is None:
                return
            xs = cat_act.src()
            g = x.ensure_grad()
            self._chk(self.lib.yxh_spp_bwd(self.dcode, B, C.byref(xs), c, cat_act.grad.data_ptr(), g.data_ptr(),
                                           self.stream), "spp bwd")

        self.tape.append(backward)
        return self.base_conv(m.conv2, [(cat_act, 0)])

    def focus(self, m: Focus, images: torch.Tensor) -> Act:
        # network_blocks.py:193-208: space-to-depth into 16 NHWC channels (12 used)
        B, _, H, W = images.shape
        packed = torch.empty(B, H // 2, W // 2, 16, dtype=self.dtype, device=self.device)
        self._chk(self.lib.yxh_focus_pack(images.data_ptr(), N.NCHW, N.DTYPE_CODE[images.dtype], B, H, W,
                                          packed.data_ptr(), self.dcode, self.stream), "focus")
        return self.base_conv(m.conv, [(Act(packed, 0, 16, needs_grad=False), 0)], cin_store=12)

    def darknet(self, m: CspDarknet, images: torch.Tensor):
        # darknet.py:165-177
        outs = self.darknet_all(m, images)
        return outs["dark3"], outs["dark4"], outs["dark5"]

    def darknet_all(self, m: CspDarknet, images: torch.Tensor) -> dict:
        x = self.focus(m.stem, images)
        outs = {"stem": x}
        for name, stage in (("dark2", m.dark2), ("dark3", m.dark3), ("dark4", m.dark4), ("dark5", m.dark5)):
            x = self.base_conv(stage[0], [(x, 0)])
            for blk in list(stage)[1:]:
                x = self.spp(blk, [(x, 0)]) if isinstance(blk, SPPBottleneck) else self.csp(blk, [(x, 0)])
            outs[name] = x
        return outs

    def pafpn(self, m: YoloPafpn, images: torch.Tensor):
        # yolo_pafpn.py:83-116
        x2, x1, x0 = self.darknet(m.backbone, images)
        fpn_out0 = self.base_conv(m.lateral_conv0, [(x0, 0)])
        f_out0 = self.csp(m.C3_p4, [(fpn_out0, 1), (x1, 0)])
        fpn_out1 = self.base_conv(m.reduce_conv1, [(f_out0, 0)])
        pan_out2 = self.csp(m.C3_p3, [(fpn_out1, 1), (x2, 0)])
        p_out1 = self.base_conv(m.bu_conv2, [(pan_out2, 0)])
        pan_out1 = self.csp(m.C3_n3, [(p_out1, 0), (fpn_out1, 0)])
        p_out0 = self.base_conv(m.bu_conv1, [(pan_out1, 0)])
        pan_out0 = self.csp(m.C3_n4, [(p_out0, 0), (fpn_out0, 0)])
        return pan_out2, pan_out1, pan_out0

    def head(self, head: YoloxHead, feats, labels: torch.Tensor) -> dict:
        # yolo_head.py:140-182 (training branch), 213-231, 253-411
        B = feats[0].t.shape[0]
        nc = head.num_classes
        D = 5 + nc
        hw = [(f.h, f.w) for f in feats]
        A = sum(h * w for h, w in hw)
        raw = torch.empty(B, A, D, dtype=torch.float32, device=self.device)
        levels = []
        a_off = 0
        for k, x in enumerate(feats):
            s = self.base_conv(head.stems[k], [(x, 0)])
            c = self.base_conv(head.cls_convs[k][0], [(s, 0)])
            c = self.base_conv(head.cls_convs[k][1], [(c, 0)])
            r = self.base_conv(head.reg_convs[k][0], [(s, 0)])
            r = self.base_conv(head.reg_convs[k][1], [(r, 0)])
            h, w = x.h, x.w
            # reg | obj preds stacked (5 rows, both read reg_feat, :155-159) and the cls
            # preds write raw rows of [B, A, 5+C] (the cat of :164 in anchor order)
            w_ro = torch.cat([head.reg_preds[k].weight.detach().reshape(4, -1),
                              head.obj_preds[k].weight.detach().reshape(1, -1)]).contiguous()
            b_ro = torch.cat([head.reg_preds[k].bias.detach(), head.obj_preds[k].bias.detach()]).contiguous()
            pk_ro = torch.empty(5 * r.ch, dtype=self.dtype, device=self.device)
            pk_rob = torch.empty(5, dtype=torch.float32, device=self.device)
            self._chk(self.lib.yxh_fold_bn_pack(w_ro.data_ptr(), b_ro.data_ptr(), None, None, None, None, 0.0, 5,
                                                r.ch, 1, 1, r.ch, self.dcode, pk_ro.data_ptr(), pk_rob.data_ptr(),
                                                self.stream), "pack preds")
            wc, bc = self._fwd_weight(head.cls_preds[k], c.ch)
            base = raw.data_ptr() + a_off * D * 4
            self._conv([r.src()], r.ch, 5, 1, 1, 0, pk_ro.data_ptr(), pk_rob.data_ptr(), base, True, D, A * D,
                       h, w, h, w, B)
            self._conv([c.src()], c.ch, nc, 1, 1, 0, wc.data_ptr(), bc.data_ptr(), base + 5 * 4, True, D, A * D,
                       h, w, h, w, B)
            levels.append((k, r, c, w_ro, a_off, h, w))
            a_off += h * w
        preds = torch.empty_like(raw)
        lhw = (C.c_int32 * (2 * len(hw)))(*[v for t in hw for v in t])
        strides = (C.c_int32 * len(hw))(*head.strides[:len(hw)])
        self._chk(self.lib.yxh_head_decode_train(raw.data_ptr(), B, A, nc, lhw, strides, len(hw), preds.data_ptr(),
                                                 self.stream), "decode")
        L = labels.shape[1]
        use_l1 = bool(head.use_l1)
        origin = raw[..., :4].contiguous() if use_l1 else None
        fg = torch.empty(B, A, dtype=torch.uint8, device=self.device)
        matched = torch.empty(B, A, dtype=torch.int32, device=self.device)
        piou = torch.empty(B, A, dtype=torch.float32, device=self.device)
        num_fg = torch.empty(B, dtype=torch.int32, device=self.device)
        losses = torch.empty(6, dtype=torch.float32, device=self.device)
        ws = torch.empty(int(self.lib.yxh_yolox_loss_workspace_bytes(B, A, L)), dtype=torch.uint8,
                         device=self.device)
        self._chk(self.lib.yxh_yolox_loss(
            preds.data_ptr(), origin.data_ptr() if origin is not None else None, labels.data_ptr(), B, A, nc, L,
            lhw, strides, len(hw), fg.data_ptr(), matched.data_ptr(), piou.data_ptr(), num_fg.data_ptr(),
            losses.data_ptr(), ws.data_ptr(), ws.numel(), self.stream), "yolox loss")
        self.assign = {"fg_mask": fg, "matched_gt_inds": matched, "pred_ious": piou, "num_fg": num_fg}
        self.outputs = preds

        def backward():
            g_ro = torch.empty(B, A, 8, dtype=self.dtype, device=self.device)
            g_cls = torch.empty(B, A, nc, dtype=self.dtype, device=self.device)
            self._chk(self.lib.yxh_yolox_loss_bwd(
                preds.data_ptr(), raw.data_ptr(), labels.data_ptr(), B, A, nc, L, lhw, strides, len(hw),
                fg.data_ptr(), matched.data_ptr(), piou.data_ptr(), num_fg.data_ptr(), self.grad_total.data_ptr(),
                int(use_l1), self.dcode, g_ro.data_ptr(), g_cls.data_ptr(), self.stream), "loss bwd")
            gb = self.grads
            for k, r, c, w_ro, a0, h, w in reversed(levels):
                for g_all, ch, feat, wmat, convs in (
                        (g_ro, 8, r, w_ro, (head.reg_preds[k], head.obj_preds[k])),
                        (g_cls, nc, c, head.cls_preds[k].weight.detach().reshape(nc, -1), (head.cls_preds[k],))):
                    cout = sum(cv.out_channels for cv in convs)
                    dys = N.Src()
                    dys.ptr = g_all.data_ptr() + a0 * ch * self.esize
                    dys.channels, dys.cstride, dys.bstride = ch, ch, A * ch
                    dys.h, dys.w, dys.upsample = h, w, 0
                    # weight gradient (stacked rows) and bias sums
                    dw = torch.zeros(cout, feat.ch, dtype=torch.float32, device=self.device)
                    self._wgrad([feat.src()], feat.ch, feat.ch, cout, 1, 1, 0, dys, dw, h, w, h, w, B)
                    bsum = torch.empty(ch, dtype=torch.float32, device=self.device)
                    self._chk(self.lib.yxh_channel_sum(self.dcode, B, C.byref(dys), bsum.data_ptr(),
                                                       self.ws.data_ptr(), self.ws.numel(), self.stream), "bias sum")
                    row = 0
                    for cv in convs:
                        n = cv.out_channels
                        gb.of(cv.weight).copy_(dw[row:row + n].view_as(cv.weight))
                        gb.of(cv.bias).copy_(bsum[row:row + n])
                        row += n
                        self._ready(cv.weight, cv.bias)
                    # data gradient: 1x1 conv with the transposed pred weights (K padded to `ch`)
                    wt = torch.empty(feat.ch * ch, dtype=self.dtype, device=self.device)
                    wm = wmat.contiguous()
                    self._chk(self.lib.yxh_pack_dgrad_weight(
                        wm.data_ptr(), cout, feat.ch, 1, 1, 0, feat.ch, ch, self.dcode, wt.data_ptr(), self.stream),
                        "pack pred dgrad")
                    g, acc = feat.grad_target()
                    self._conv([dys], ch, feat.ch, 1, 1, 0, wt.data_ptr(), self.zero_bias.data_ptr(), g.data_ptr(),
                               True, feat.ch, h * w * feat.ch, h, w, h, w, B, accumulate=acc)

        self.tape.append(backward)
        return {k: losses[i] for i, k in enumerate(LOSS_KEYS)}

    # ------------------------------------------------------------ entry points
    def forward(self, images: torch.Tensor, labels: torch.Tensor) -> dict:
        self.tape = []
        if images.dim() != 4 or images.shape[1] != 3:
            raise ValueError(f"expected [B, 3, H, W] images, got {tuple(images.shape)}")
        if images.shape[2] % 32 or images.shape[3] % 32:
            raise ValueError("input size must be multiples of 32")
        images = images.to(self.device)
        if images.dtype not in (torch.float32, torch.bfloat16, torch.float16, torch.uint8):
            images = images.float()
        images = images.contiguous()
        labels = labels.to(self.device, torch.float32).contiguous()
        self._keep = (images, labels)
        self._bn_counters = []
        self._pack_all()
        feats = self.pafpn(self.model.backbone, images)
        out = self.head(self.model.head, feats, labels)
        if self._bn_counters:
            torch._foreach_add_(self._bn_counters, 1)
        return out

    def backward(self, grad_total: Optional[torch.Tensor] = None) -> None:
        if not self.tape:
            raise RuntimeError("backward without a recorded training forward (or called twice)")
        if grad_total is not None:
            self.grad_total.copy_(grad_total.reshape(()).to(torch.float32))
        prev = self.grads.begin()
        for fn in reversed(self.tape):
            fn()
        if self._wside is not None:  # every weight gradient is in before the reducer / optimizer
            self._flush_wgrad()
            if self._segcap is None:
                torch.cuda.current_stream(self.device).wait_stream(self._wside)
        self.tape = []
        self._keep = None
        if self.batch_pack and self._pack_table is None and self._pack_jobs:
            self._build_pack_table()
        if self.on_backward_end is not None:
            self.on_backward_end()
        self.grads.publish(prev)


class CapturedTrainStep:
    """One training forward + reverse pass captured as hipGraph segments (torch.cuda.CUDAGraph
    objects sharing one memory pool: the main stream's work between two weight-gradient forks,
    and each fork's weight gradients for the side stream) and replayed for every batch of the
    same shape: the step's ~850 launches cost the host a few graph launches and events instead
    of the ctypes issue of every kernel (bench.py reports the eager ``host_issue_ms_per_step``).

    Each call copies the batch into the static input buffers and replays; the loss dict, the
    SimOTA assignment and the flat gradient buffer are rewritten in place, and ``param.grad``
    views are (re)published, as after ``optimizer.zero_grad(set_to_none=True)`` +
    ``loss.backward()`` (trainer.py:104-112).  The weight repacks, the BN running statistics
    and ``num_batches_tracked`` are inside the graph and read the fp32 master weights through
    their fixed storage, so in-place optimizer steps between replays are seen.  ``grad_scale``
    (a one-element fp32 device tensor, e.g. ``GradScaler._scale``) is read by every replay.

    Data parallel (round 6): when the model runs under ``yolox_amd.dp.DistributedDataParallel``
    (the reducer's hooks are installed on the TrainGraph by an eager DDP step), the capture records
    in which segment -- and so on which stream, at which point of it -- every parameter's
    gradient is reported ready, instead of issuing collectives inside the capture.  A replay then
    resets the reducer, reports the same parameters right after replaying that segment on that
    segment's stream (the eager step's exact event placement: the reducer's bucketed RCCL
    all-reduces are issued between segments, overlapping the later segments), and finishes the
    reducer behind the last segment (1/world mean on the compute stream), as the eager backward does.

    Requirements: the step ran eagerly once for this shape (tiles tuned, the repack table
    recorded), and the parameters keep their storage (``model.to`` / re-created tensors need a new
    capture)."""

    def __init__(self, model, images: torch.Tensor, targets: torch.Tensor, dtype: Optional[torch.dtype] = None,
                 grad_scale: Optional[torch.Tensor] = None):
        g = getattr(model, "_train_graph", None)
        dtype = dtype or compute_dtype_from_autocast()
        if g is None or g.dtype != dtype or g.device != model.device:
            raise RuntimeError("CapturedTrainStep: run one eager training step of this shape first")
        # data-parallel hooks (DistributedDataParallel.forward installs them): reported between the
        # replayed segments, never captured
        self.on_ready, self.on_end = g.on_param_ready, g.on_backward_end
        self.reducer = getattr(self.on_ready, "__self__", None)
        if g.batch_pack and g._pack_table is None:
            raise RuntimeError("CapturedTrainStep: the repack table is not recorded yet (run an eager step)")
        self.model, self.g, self.dev = model, g, model.device
        self.images = images.to(model.device).clone()
        self.targets = targets.to(model.device).clone()
        self.grad_scale = grad_scale
        if grad_scale is None:
            g.grad_total.fill_(1.0)
        for p in g.grads.params:  # the graph overwrites the gradients (no carry-over of held ones)
            p.grad = None
        # segments: the main stream's work between two weight-gradient forks is one graph, each
        # fork's weight gradients another, replayed on the side stream behind an event -- the
        # concurrency of the eager step.  (One multi-stream capture lets the runtime re-assign
        # nodes to its own queues, which serialised the weight gradients with the data-gradient
        # chain on MI355X: profiles/r03/train_graph.txt.)
        self.pool = None  # the first segment's private pool, shared by the later segments (CUDAGraph.pool())
        self.plan: list = []  # ("main" | "side", CUDAGraph or None (an empty main segment), [ready params])
        self._ready_cur: list = []  # parameters reported ready in the main segment being captured
        self._empty: list = []  # captured main segments with no launch (kept alive, not replayed)
        self._keep: list = []  # conv-output gradients read by side segments: alive for the whole step
        # YOLOX_AMD_MAIN_PRIORITY=1: the main segments replay on a high-priority stream, so the
        # data-gradient chain (the step's critical path) is dispatched ahead of the side stream's
        # weight gradients when both have workgroups waiting for CUs
        prio = -1 if os.environ.get("YOLOX_AMD_MAIN_PRIORITY", "0") == "1" else 0
        self.main = torch.cuda.Stream(self.dev, priority=prio)
        self.side_stream = g._wside
        self._dbg = os.environ.get("YOLOX_AMD_CAP_DEBUG", "")
        if "torch" in self._dbg:  # diagnostic: one torch.cuda.graph capture (side stream forked inside it)
            self.single = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.single):
                self.out = g.forward(self.images, self.targets)
                g.backward(grad_scale)
            return
        self.single = None
        torch.cuda.synchronize(self.dev)
        if "gc" in self._dbg:
            import gc
            gc.collect()
            torch.cuda.empty_cache()
        with torch.cuda.stream(self.main):
            self._begin()
            g._segcap = self if self.side_stream is not None else None
            g.on_param_ready, g.on_backward_end = self._ready_cur.append, None
            try:
                self.out = g.forward(self.images, self.targets)
                g.backward(grad_scale)  # begin(): p.grad is None here, nothing to carry over
            finally:
                g._segcap = None
                g.on_param_ready, g.on_backward_end = self.on_ready, self.on_end
                self._end()
        self.events = [torch.cuda.Event() for _ in self.plan]

    def _begin(self) -> None:
        self._cur = torch.cuda.CUDAGraph()
        self._cur.capture_begin(pool=self.pool, capture_error_mode="global" if "global" in self._dbg else "thread_local")

    def _end(self) -> None:
        # a main segment between two weight-gradient flushes (or after the last one) may hold no
        # launch at all: torch reports it empty; it is kept only as the pool owner, not replayed
        import warnings
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            self._cur.capture_end()
        empty = any("Graph is empty" in str(w.message) for w in caught)
        for w in caught:
            if "Graph is empty" not in str(w.message):
                warnings.warn_explicit(w.message, w.category, w.filename, w.lineno)
        if self.pool is None:
            self.pool = self._cur.pool()
        if empty:  # kept as the pool owner; its readiness reports stay at this point of the main stream
            self._empty.append(self._cur)
            if self._ready_cur:
                self.plan.append(("main", None, self._ready_cur))
        else:
            self.plan.append(("main", self._cur, self._ready_cur))
        self._ready_cur = []
        self._cur = None

    def side(self, pending: list) -> None:
        """TrainGraph._flush_wgrad while capturing: close the main segment, capture the
        pending weight gradients as a side segment, open the next main segment."""
        self._end()
        gs = torch.cuda.CUDAGraph()
        with torch.cuda.stream(self.side_stream):
            gs.capture_begin(pool=self.pool, capture_error_mode="thread_local")
            for launch, dy, _ in pending:
                launch()
                self._keep.append(dy)
            gs.capture_end()
        self.plan.append(("side", gs, [param for _, _, param in pending]))
        self._begin()

    def _replay(self) -> None:
        caller = torch.cuda.current_stream(self.dev)
        self.main.wait_stream(caller)
        fork = torch.cuda.Event()  # a side segment ahead of every (non-empty) main one forks here
        fork.record(self.main)
        ready = self.on_ready
        if ready is not None and self.reducer is not None and hasattr(self.reducer, "reset"):
            self.reducer.reset()  # what DistributedDataParallel.forward does before an eager step
        with torch.cuda.stream(self.main):
            for (kind, gr, params), ev in zip(self.plan, self.events):
                if kind == "main":
                    if gr is not None:
                        gr.replay()
                    if ready is not None:
                        for p in params:  # events on the main stream, right behind this segment
                            ready(p)
                    fork = ev
                    ev.record(self.main)
                else:
                    self.side_stream.wait_event(fork)
                    with torch.cuda.stream(self.side_stream):
                        gr.replay()
                        if ready is not None:
                            for p in params:  # events on the side stream, behind its segment
                                ready(p)
            if self.side_stream is not None:
                self.main.wait_stream(self.side_stream)
            if self.on_end is not None:
                self.on_end()  # the reducer's remaining buckets, the wait for them and the 1/world mean
        caller.wait_stream(self.main)

    def __call__(self, images: torch.Tensor, targets: torch.Tensor) -> dict:
        if images.shape != self.images.shape or targets.shape != self.targets.shape:
            raise ValueError("CapturedTrainStep: batch shape differs from the captured one")
        if images.data_ptr() != self.images.data_ptr():
            self.images.copy_(images, non_blocking=True)
        if targets.data_ptr() != self.targets.data_ptr():
            self.targets.copy_(targets, non_blocking=True)
        if self.single is not None:
            self.single.replay()
        else:
            self._replay()
        self.g.grads.publish(None)
        if hasattr(self.model, "weights_changed"):  # BN running statistics were updated in place
            self.model.weights_changed()
        return dict(self.out)


class _LossFn(torch.autograd.Function):
    """Hooks the HIP reverse pass into ``loss.backward()`` (trainer.py:112)."""

    @staticmethod
    def forward(ctx, anchor, total, graph):
        ctx.graph = graph
        return total.clone()

    @staticmethod
    def backward(ctx, g):
        ctx.graph.backward(g)
        return None, None, None


def compute_dtype_from_autocast() -> torch.dtype:
    """The reference trains under torch.cuda.amp.autocast when --fp16 (trainer.py:103-104):
    autocast selects the compute dtype of the HIP path; fp32 otherwise."""
    if torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return torch.float32


def train_forward(model, images: torch.Tensor, targets: torch.Tensor, dtype: Optional[torch.dtype] = None) -> dict:
    """YoloxModule.forward(x, targets) in train mode: the reference's loss dict with
    ``total_loss`` differentiable through the HIP reverse pass."""
    dtype = dtype or compute_dtype_from_autocast()
    g = getattr(model, "_train_graph", None)
    if g is None or g.dtype != dtype or g.device != model.device:
        g = TrainGraph(model, dtype)
        model._train_graph = g
    out = g.forward(images, targets)
    if hasattr(model, "weights_changed"):  # BN running statistics were updated in place
        model.weights_changed()
    anchor = torch.zeros((), device=model.device, requires_grad=True)
    out["total_loss"] = _LossFn.apply(anchor, out["total_loss"], g)
    return out


# ------------------------------------------------------------------ standalone blocks, train mode
class _BlockOwner:
    """What TrainGraph needs of its model for one building block: parameters and device."""

    def __init__(self, block: nn.Module):
        self.block = block

    def parameters(self):
        return self.block.parameters()

    @property
    def device(self) -> torch.device:
        return next(self.block.parameters()).device


class _BlockFn(torch.autograd.Function):
    """A block's train-mode forward recorded on its TrainGraph tape; backward replays the tape
    from the output gradients (parameter gradients published as in the model's step) and
    returns the input's gradient."""

    @staticmethod
    def forward(ctx, anchor, x, graph, run):
        outs, acts, in_act = run()
        ctx.graph, ctx.acts, ctx.in_act, ctx.x_dtype = graph, acts, in_act, x.dtype
        # this call's tape and the tensors it reads belong to this autograd node: a block called
        # again before backward (a shared module on two inputs) records a tape of its own
        ctx.tape, ctx.keep = graph.tape, graph._keep
        graph.tape, graph._keep = [], None
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        if ctx.tape is None:
            raise RuntimeError("block backward called twice on one forward (retain_graph is not supported)")
        for a, go in zip(ctx.acts, gouts):
            if go is not None:
                a.grad = go.permute(0, 2, 3, 1).to(torch.float32).contiguous()
        ctx.graph.tape, ctx.graph._keep = ctx.tape, ctx.keep
        ctx.tape = ctx.keep = None
        ctx.graph.backward(None)
        a = ctx.in_act
        gx = None
        if a is not None and a.grad is not None:
            gx = a.grad.permute(0, 3, 1, 2).to(ctx.x_dtype).contiguous()
        return None, gx, None, None


def block_train_forward(block: nn.Module, x: torch.Tensor, dtype: Optional[torch.dtype] = None) -> list:
    """A building block's forward in training mode (network_blocks.py:27-208, darknet.py:95-177
    called standalone on a train-mode module, as the reference's eager modules allow): BatchNorm
    with batch statistics (running statistics and num_batches_tracked updated like torch), the
    HIP kernels of the model's train step, and autograd through its reverse pass.  Returns the
    block's output maps as NCHW tensors (CspDarknet: dark3, dark4, dark5)."""
    from .models.network import BaseConv, Bottleneck, CspDarknet, CspLayer, DWConv, Focus, SPPBottleneck
    dtype = dtype or compute_dtype_from_autocast()
    owner = _BlockOwner(block)
    g = block.__dict__.get("_train_graph_block")
    if g is None or g.dtype != dtype or g.device != owner.device:
        g = TrainGraph(owner, dtype)
        block.__dict__["_train_graph_block"] = g
    dev = owner.device
    x = x.to(dev)

    def run():
        g.tape = []
        g._bn_counters = []
        g._pack_all()
        in_act = None
        if isinstance(block, (Focus, CspDarknet)):
            images = x.contiguous() if x.dtype in (torch.float32, torch.bfloat16, torch.float16, torch.uint8) \
                else x.float().contiguous()
            g._keep = (images,)
            if isinstance(block, Focus):
                outs = [g.focus(block, images)]
            else:
                allm = g.darknet_all(block, images)
                outs = [allm[k] for k in block._names()]
        else:
            t = x.detach().to(dtype).permute(0, 2, 3, 1).contiguous()
            in_act = Act(t, 0, t.shape[3], needs_grad=x.requires_grad)
            g._keep = (t,)
            if isinstance(block, (BaseConv, DWConv)):
                outs = [g.base_conv(block, [(in_act, 0)])]
            elif isinstance(block, Bottleneck):
                outs = [g.bottleneck(block, in_act)]
            elif isinstance(block, CspLayer):
                outs = [g.csp(block, [(in_act, 0)])]
            elif isinstance(block, SPPBottleneck):
                outs = [g.spp(block, [(in_act, 0)])]
            else:
                raise NotImplementedError(f"{type(block).__name__} has no train-mode block forward")
        if g._bn_counters:
            torch._foreach_add_(g._bn_counters, 1)
        maps = [a.t[..., a.coff:a.coff + a.ch].permute(0, 3, 1, 2).contiguous() for a in outs]
        return maps, outs, in_act

    anchor = torch.zeros((), device=dev, requires_grad=True)
    return list(_BlockFn.apply(anchor, x, g, run))
