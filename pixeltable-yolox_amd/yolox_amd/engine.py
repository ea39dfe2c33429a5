"""Planner + executor: turns a YoloxModule into a fixed libyoloxhip op list.

A plan is built once per (model, batch, input size, compute dtype, input format):

* every activation is an NHWC buffer in ONE device arena (bump-allocated, 256-B
  aligned); concatenations are buffers whose channel slices are written directly by
  the producing convs, nearest-x2 upsampling is a strided read flag -- nothing is
  copied between layers;
* every conv has its BN folded into packed ``[cout][kh][kw][cin]`` weights in a
  second arena (yxh_fold_bn_pack, re-run whenever parameters change);
* the head's 1x1 preds write decoded fp32 rows into the [B, A, 5+C] output.

The op list runs eagerly (one ctypes call, ``yxh_run_ops``) or as a captured
hipGraph (``capture()`` / ``replay()``).
"""
from __future__ import annotations

import ctypes as C
import os
import statistics
import sys
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn

from . import _native as N

ALIGN = 256


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass(eq=False)
class Buffer:
    h: int
    w: int
    c: int
    esize: int
    offset: int = -1

    @property
    def nelem_image(self) -> int:
        return self.h * self.w * self.c

    def full(self) -> "View":
        return View(self, 0, self.c)

    def slice(self, coff: int, ch: int) -> "View":
        if coff < 0 or coff + ch > self.c:
            raise ValueError(f"slice [{coff}, {coff + ch}) outside buffer of {self.c} channels")
        return View(self, coff, ch)


@dataclass(eq=False)
class View:
    buf: Buffer
    coff: int
    ch: int
    up: int = 0

    @property
    def lh(self) -> int:
        return self.buf.h << self.up

    @property
    def lw(self) -> int:
        return self.buf.w << self.up

    def upsampled(self) -> "View":
        return View(self.buf, self.coff, self.ch, self.up + 1)

    def same_storage(self, other: "View") -> bool:
        return self.buf is other.buf and self.coff == other.coff and self.ch == other.ch


@dataclass(eq=False)
class WeightSpec:
    convs: list  # [(nn.Conv2d, nn.BatchNorm2d | None)], stacked along cout
    cout: int
    cin_g: int
    kh: int
    kw: int
    cin_pad: int
    stem: bool = False  # fused Focus+stem layout [round16(cout)][6][32] (yxh_stem_pack)
    w_off: int = -1  # bytes into weight arena
    b_off: int = -1  # bytes into bias arena
    f_off: int = -1  # bytes into the fragment-major copy (yxh_pack_frag), -1 = none


@dataclass(eq=False)
class ImageRef:
    """The plan's input image (bound at run time): what Focus plans from."""
    h: int
    w: int


@dataclass(eq=False)
class OpRec:
    kind: int
    args: dict = field(default_factory=dict)
    lane: int = 0  # graph branch (yxh_graph_create_lanes); 0 = backbone / neck


# Bottleneck fusion is opt-in (Plan(fuse_bottleneck=True) or YOLOX_AMD_FUSE_BOTTLENECK=1): in one
# process on one box (tools/ab_fuse.py) the two-launch form is 1.8 % faster (2.001 vs 2.038 ms per
# yolox_s bs32 forward) -- the fused kernel's 1x1-on-the-halo phase is not overlapped with MFMAs
_FUSE_BOTTLENECK = os.environ.get("YOLOX_AMD_FUSE_BOTTLENECK", "0") == "1"
# 1x1 convs folded into the launch that produces their input (YOLOX_AMD_CSP_FUSION=0: separate launches)
_CSP_FUSION = os.environ.get("YOLOX_AMD_CSP_FUSION", "1") != "0"
# head levels whose preds ride in the cls_convs[k][1] | reg_convs[k][1] launch (conv_ws head form),
# YOLOX_AMD_HEAD_FUSION="0,1,2" / "2" / ...; default none: measured on MI355X (round 4, one box,
# profiles/r04/head_fusion_ab.txt) the bench forward is 1.693 ms with all three levels fused,
# 1.681 with levels 0 + 2, 1.679 with level 2 and 1.678 with none -- the head-form tile runs its
# conv ~45 us slower at level 0 than the plain two-group tile, which eats the head_pred launch
_HEAD_FUSION = {int(v) for v in os.environ.get("YOLOX_AMD_HEAD_FUSION", "").split(",") if v.strip()}
# fragment-major weight copies for the weight-stationary tiles (YOLOX_AMD_WFRAG=0: row layout only)
_WFRAG = os.environ.get("YOLOX_AMD_WFRAG", "1") != "0"


class PlanCtx:
    def __init__(self, batch: int, dtype: torch.dtype, device: torch.device, fuse_stem: bool = True,
                 fuse_bottleneck: bool = _FUSE_BOTTLENECK, fuse_stem_s2: bool = True, csp_fusion: Optional[bool] = None):
        if dtype not in (torch.float32, torch.bfloat16, torch.float16):
            raise ValueError(f"compute dtype {dtype} not supported (float32, bfloat16, float16)")
        self.batch = batch
        self.dtype = dtype
        self.dcode = N.DTYPE_CODE[dtype]
        self.esize = torch.empty((), dtype=dtype).element_size()
        self.epc = 16 // self.esize
        self.device = device
        self.fuse_stem = fuse_stem
        self.fuse_stem_s2 = fuse_stem_s2  # Focus stem + dark2[0] as one yxh_stem_s2 launch
        # 1x1 convs folded into a neighbouring launch (stem_s2's CSP form; YOLOX_AMD_CSP_FUSION=0: off)
        self.csp_fusion = (_CSP_FUSION if csp_fusion is None else csp_fusion) and dtype != torch.float32
        # the image the plan reads (set by Plan): the fused stem + stride-2 conv needs NHWC
        self.input_layout = N.NHWC
        self.input_dtype = torch.uint8
        # Bottleneck conv1 (1x1) folded into conv2's 3x3 (conv_ws fused tiles): 16-bit only
        self.fuse_bottleneck = fuse_bottleneck and dtype != torch.float32
        self.buffers: list[Buffer] = []
        self.weights: list[WeightSpec] = []
        self.ops: list[OpRec] = []
        self.flops = 0.0  # algorithmic multiply-adds x2 of the recorded convs

    # ---------------------------------------------------------------- buffers
    def buffer(self, h: int, w: int, c: int) -> Buffer:
        if c % self.epc:
            raise ValueError(f"channel count {c} not a multiple of {self.epc}")
        b = Buffer(h, w, c, self.esize)
        self.buffers.append(b)
        return b

    # ---------------------------------------------------------------- ops
    def image(self, h: int, w: int) -> ImageRef:
        return ImageRef(h, w)

    def stem_fusable(self, m) -> bool:
        c = m.conv
        return (self.fuse_stem and c.in_channels == 12 and c.groups == 1 and c.kernel_size == (3, 3)
                and c.stride == (1, 1) and c.padding == (1, 1) and c.out_channels <= 80
                and (c.out_channels * self.esize) % 16 == 0)

    def stem(self, m, img: ImageRef) -> View:
        """Focus + its BaseConv (3x3 s1 on 12 channels) as one 6x6 s2 conv on the image."""
        conv = m.conv
        out = self.buffer(img.h // 2, img.w // 2, conv.out_channels)
        spec = WeightSpec([(conv, m.bn)], conv.out_channels, 12, 3, 3, 12, stem=True)
        self.weights.append(spec)
        self.ops.append(OpRec(N.OP_STEM, dict(dst=out.full(), h=img.h, w=img.w, spec=spec,
                                              act=N.ACT_CODE[getattr(m, "act_name", "silu")])))
        self.flops += 2.0 * self.batch * out.h * out.w * conv.out_channels * 9 * 12
        return out.full()

    def stem_s2_fusable(self, stem, conv) -> bool:
        """Focus stem + dark2[0] as one yxh_stem_s2 launch: 16-bit compute, an NHWC
        u8/bf16/f16 image, 12 -> 32 stem channels, BaseConv 32 -> 64 3x3 s2, SiLU both."""
        c1 = stem.conv
        c2 = getattr(conv, "conv", None)
        return (self.fuse_stem and self.fuse_stem_s2 and self.dtype != torch.float32 and self.input_layout == N.NHWC
                and self.input_dtype in (torch.uint8, torch.bfloat16, torch.float16) and c2 is not None
                and self.stem_fusable(stem) and c1.out_channels == 32 and c2.in_channels == 32
                and c2.out_channels == 64 and c2.kernel_size == (3, 3) and c2.stride == (2, 2)
                and c2.padding == (1, 1) and c2.groups == 1
                and getattr(stem, "act_name", "silu") == getattr(conv, "act_name", "silu") == "silu")

    def stem_s2(self, stem, conv, img: ImageRef) -> View:
        """Focus + stem BaseConv + dark2[0] (darknet.py:112-123) as ONE launch: the stem map
        exists only per tile in LDS (csrc/stem_s2.hip)."""
        return self._stem_s2(stem, conv, img)[0]

    def stem_s2_csp_fusable(self, csp) -> bool:
        """dark2's CspLayer conv1 | conv2 (1x1 64 -> 2 x 32) and its first Bottleneck's conv1
        (1x1 32 -> 32) can ride in the stem_s2 launch (yxh_stem2_desc.w3 / w4)."""
        if not (self.csp_fusion and not self.fuse_bottleneck and hasattr(csp, "conv1") and len(csp.m) >= 1):
            return False
        b0 = csp.m[0]
        k1, k2, kb = csp.conv1.conv, csp.conv2.conv, getattr(b0.conv1, "conv", None)
        ok = kb is not None and all(k.kernel_size == (1, 1) and k.groups == 1 and k.stride == (1, 1) for k in (k1, k2, kb))
        return (ok and k1.in_channels == 64 and k1.out_channels == 32 and k2.out_channels == 32
                and kb.in_channels == 32 and kb.out_channels == 32
                and {getattr(m, "act_name", "silu") for m in (csp.conv1, csp.conv2, b0.conv1)} == {"silu"})

    def stem_s2_csp(self, stem, conv, csp, img: ImageRef) -> tuple:
        """stem_s2 + dark2's CspLayer conv1 | conv2 + its first Bottleneck conv1 as ONE launch:
        returns (the [x_1 | x_2] concat buffer, the Bottleneck's hidden map t)."""
        _, cat, t = self._stem_s2(stem, conv, img, csp)
        return cat, t

    def _stem_s2(self, stem, conv, img: ImageRef, csp=None) -> tuple:
        if img.h % 4 or img.w % 4:
            raise ValueError("stem_s2 needs image sides that are multiples of 4")
        oh1, ow1 = img.h // 2, img.w // 2
        oh, ow = (oh1 - 1) // 2 + 1, (ow1 - 1) // 2 + 1
        c1, c2 = stem.conv.out_channels, conv.conv.out_channels
        s1 = WeightSpec([(stem.conv, stem.bn)], c1, 12, 3, 3, 12, stem=True)
        self.weights.append(s1)
        s2 = self._weights([(conv.conv, conv.bn)], c1)
        args = dict(h=img.h, w=img.w, spec1=s1, spec2=s2, c1=c1, c2=c2, act=N.ACT_SILU)
        self.flops += 2.0 * self.batch * oh1 * ow1 * c1 * 9 * 12 + 2.0 * self.batch * oh * ow * c2 * 9 * c1
        if csp is None:
            out = self.buffer(oh, ow, c2)
            self.ops.append(OpRec(N.OP_STEM2, dict(dst=out.full(), **args)))
            return out.full(), None, None
        hidden = csp.conv1.conv.out_channels
        b0 = csp.m[0]
        cat = self.buffer(oh, ow, 2 * hidden)
        t = self.buffer(oh, ow, hidden)
        s3 = self._weights([(csp.conv1.conv, csp.conv1.bn), (csp.conv2.conv, csp.conv2.bn)], c2)
        s4 = self._weights([(b0.conv1.conv, b0.conv1.bn)], hidden)
        self.ops.append(OpRec(N.OP_STEM2, dict(dst=None, dst3=cat.full(), dst4=t.full(), spec3=s3, spec4=s4, **args)))
        self.flops += 2.0 * self.batch * oh * ow * (2 * hidden * c2 + hidden * hidden)
        return None, cat, t.full()

    def focus(self, h: int, w: int) -> View:
        packed = self.buffer(h // 2, w // 2, 16)
        self.ops.append(OpRec(N.OP_FOCUS, dict(dst=packed.full(), h=h, w=w)))
        return packed.full()

    def _weights(self, convs, cin_pad: int) -> WeightSpec:
        c0 = convs[0][0]
        spec = WeightSpec(convs, sum(c.out_channels for c, _ in convs), c0.in_channels // c0.groups,
                          c0.kernel_size[0], c0.kernel_size[1], cin_pad)
        self.weights.append(spec)
        return spec

    def conv(self, m, srcs: list[View], out: Optional[View] = None, residual: Optional[View] = None) -> View:
        """A BaseConv (conv + BN + act) over 1-2 channel-concatenated sources."""
        return self.conv_multi([m], srcs, out=out, residual=residual)

    def conv_multi(self, ms, srcs: list[View], out: Optional[View] = None,
                   residual: Optional[View] = None) -> View:
        """Several BaseConvs with the same input and geometry as ONE conv whose output
        channels are the concatenation of theirs (weights stacked along cout): e.g.
        CspLayer.conv1 | conv2 writing the whole concat buffer in one pass over x."""
        convs = [m.conv for m in ms]
        conv: nn.Conv2d = convs[0]
        acts = {getattr(m, "act_name", "silu") for m in ms}
        if len(acts) != 1 or any((c.kernel_size, c.stride, c.padding, c.groups, c.in_channels)
                                 != (conv.kernel_size, conv.stride, conv.padding, conv.groups, conv.in_channels)
                                 for c in convs):
            raise ValueError("stacked convs must share geometry and activation")
        cout = sum(c.out_channels for c in convs)
        cin = sum(s.ch for s in srcs)
        lh, lw = srcs[0].lh, srcs[0].lw
        if any(s.lh != lh or s.lw != lw for s in srcs):
            raise ValueError("concatenated sources differ in spatial size")
        groups = conv.groups
        if groups == 1:
            if conv.in_channels != cin and not (conv.in_channels == 12 and cin == 16):
                raise ValueError(f"conv expects {conv.in_channels} channels, got {cin}")
        elif len(convs) > 1 or groups != cin or conv.out_channels != cin:
            raise NotImplementedError("only single depthwise grouped convs are supported")
        kh, kw = conv.kernel_size
        sh, sw_ = conv.stride
        ph, pw = conv.padding
        if kh != kw or sh != sw_ or ph != pw:
            raise NotImplementedError("square kernels/strides/padding only")
        oh = (lh + 2 * ph - kh) // sh + 1
        ow = (lw + 2 * pw - kw) // sw_ + 1
        if out is None:
            out = self.buffer(oh, ow, cout).full()
        if out.ch != cout or out.lh != oh or out.lw != ow or out.up:
            raise ValueError("output view does not match the conv")
        spec = self._weights([(c, m.bn) for c, m in zip(convs, ms)], cin if groups == 1 else 1)
        self.ops.append(OpRec(N.OP_CONV, dict(
            srcs=list(srcs), out=out, residual=residual, spec=spec, cin=cin, cout=cout, k=kh,
            stride=sh, pad=ph, groups=groups, in_h=lh, in_w=lw, out_h=oh, out_w=ow,
            act=N.ACT_CODE[acts.pop()], dst_f32=False)))
        self.flops += 2.0 * self.batch * oh * ow * cout * kh * kw * (conv.in_channels // groups)
        return out

    # (main conv cin, stride, post_src channels, post cout) shapes the conv_ws post tiles are built for
    # (cin, stride, post_src channels, post cout): dark2 / dark3 / C3_p3 conv3 over [y | x_2], a stage's
    # stride-2 conv + conv1 | conv2, and the Bottleneck chain (3x3 + shortcut, stored, + the next conv1)
    POST_SHAPES = {(32, 1, 32, 64), (64, 1, 64, 128), (64, 2, 0, 128), (64, 1, 0, 64), (128, 1, 0, 128)}

    def post_fusable(self, m, post_ms, post_src_ch: int) -> bool:
        """BaseConv ``m`` (3x3) followed by the 1x1 BaseConvs ``post_ms`` (stacked along cout)
        over [m's output | a post_src of ``post_src_ch`` channels] as one conv_ws post launch."""
        if not (self.csp_fusion and not self.fuse_bottleneck and hasattr(m, "conv")
                and all(hasattr(q, "conv") for q in post_ms)):
            return False
        k = m.conv
        pk = [q.conv for q in post_ms]
        cout_post = sum(q.out_channels for q in pk)
        acts = {getattr(q, "act_name", "silu") for q in [m] + list(post_ms)}
        return (acts == {"silu"} and k.kernel_size == (3, 3) and k.padding == (1, 1) and k.groups == 1
                and (k.out_channels == k.in_channels if k.stride == (1, 1) else k.out_channels == 2 * k.in_channels)
                and (k.in_channels, k.stride[0], post_src_ch, cout_post) in self.POST_SHAPES
                and all(q.kernel_size == (1, 1) and q.groups == 1 and q.stride == (1, 1)
                        and q.in_channels == k.out_channels + post_src_ch for q in pk))

    def conv_post(self, m, srcs: list, post_ms, post_src: Optional[View], post_out: View,
                  residual: Optional[View] = None, out: Optional[View] = None) -> View:
        """conv ``m`` + the 1x1 post conv (``post_ms`` stacked) over [m's output | post_src] as
        ONE launch (yxh_conv_desc.post_*): m's output never leaves the block's LDS -- unless
        ``out`` is given (YXH_CONV_POST_STORE: the Bottleneck chain), then it is stored there too."""
        k = m.conv
        lh, lw = srcs[0].lh, srcs[0].lw
        s = k.stride[0]
        oh, ow = (lh + 2 - 3) // s + 1, (lw + 2 - 3) // s + 1
        cout_post = sum(q.conv.out_channels for q in post_ms)
        if post_out.ch != cout_post or post_out.lh != oh or post_out.lw != ow:
            raise ValueError("post conv output view does not match")
        spec = self._weights([(k, m.bn)], k.in_channels)
        pspec = self._weights([(q.conv, q.bn) for q in post_ms], k.out_channels + (post_src.ch if post_src else 0))
        self.ops.append(OpRec(N.OP_CONV, dict(
            srcs=list(srcs), out=None, residual=residual, spec=spec, cin=k.in_channels, cout=k.out_channels, k=3,
            stride=s, pad=1, groups=1, in_h=lh, in_w=lw, out_h=oh, out_w=ow, act=N.ACT_CODE["silu"], dst_f32=False,
            post_spec=pspec, post_src=post_src, post_out=post_out, post_store_out=out)))
        self.flops += 2.0 * self.batch * oh * ow * (k.out_channels * 9 * k.in_channels + cout_post * pspec.cin_pad)
        return post_out

    def bottleneck_fusable(self, b) -> bool:
        c1, c2 = b.conv1, b.conv2
        if not (self.fuse_bottleneck and hasattr(c1, "conv") and hasattr(c2, "conv")):
            return False
        k1, k3 = c1.conv, c2.conv
        ch = k1.in_channels
        return (ch in (32, 64, 128) and k1.out_channels == ch and k3.in_channels == ch and k3.out_channels == ch
                and k1.kernel_size == (1, 1) and k1.groups == 1 and k3.kernel_size == (3, 3)
                and k3.stride == (1, 1) and k3.padding == (1, 1) and k3.groups == 1
                and getattr(c1, "act_name", "silu") == getattr(c2, "act_name", "silu") == "silu")

    def bottleneck(self, b, x: View, out: View) -> View:
        """Bottleneck (network_blocks.py:77-99) as ONE conv: conv1's 1x1 is computed per tile
        on the 3x3's halo in LDS (yxh_conv_desc.pre_weight) -- the hidden map never reaches
        HBM.  ``out`` must not alias ``x`` (neighbouring tiles read x's halo)."""
        k1, k3 = b.conv1.conv, b.conv2.conv
        ch = k1.in_channels
        if out.buf is x.buf and out.coff < x.coff + x.ch and x.coff < out.coff + out.ch:
            raise ValueError("fused Bottleneck output aliases its input")
        spec = self._weights([(k3, b.conv2.bn)], ch)
        pre = self._weights([(k1, b.conv1.bn)], ch)
        self.ops.append(OpRec(N.OP_CONV, dict(
            srcs=[x], out=out, residual=x if b.use_add else None, spec=spec, pre_spec=pre, cin=ch, cout=ch, k=3,
            stride=1, pad=1, groups=1, in_h=x.lh, in_w=x.lw, out_h=x.lh, out_w=x.lw,
            act=N.ACT_CODE["silu"], dst_f32=False)))
        self.flops += 2.0 * self.batch * x.lh * x.lw * ch * ch * 10  # 1x1 + 3x3
        return out

    def grouped2_fusable(self, a, b, src: View) -> bool:
        if self.dtype == torch.float32 or not (hasattr(a, "conv") and hasattr(b, "conv")):
            return False
        ka, kb = a.conv, b.conv
        same = all(getattr(ka, f) == getattr(kb, f) for f in ("in_channels", "out_channels", "kernel_size",
                                                              "stride", "padding", "groups"))
        return (same and ka.kernel_size == (3, 3) and ka.stride == (1, 1) and ka.groups == 1
                and ka.in_channels in (128, 256) and src.ch == 2 * ka.in_channels and ka.out_channels % 64 == 0
                and getattr(a, "act_name", "silu") == getattr(b, "act_name", "silu") == "silu")

    def conv_grouped2(self, ms, src: View) -> View:
        """Two same-shaped 3x3 BaseConvs over the two halves of one source (a head level's
        cls_convs[k][1] | reg_convs[k][1] over [cls | reg], yolo_head.py:160-161) as ONE launch
        (YXH_CONV_GROUPS2); the output buffer is [a | b]."""
        ka, kb = ms[0].conv, ms[1].conv
        cin, half = ka.in_channels, ka.out_channels
        out = self.buffer(src.lh, src.lw, 2 * half).full()
        spec = self._weights([(ka, ms[0].bn), (kb, ms[1].bn)], cin)
        self.ops.append(OpRec(N.OP_CONV, dict(
            srcs=[src], out=out, residual=None, spec=spec, cin=cin, cout=2 * half, k=3, stride=1, pad=1, groups=1,
            in_h=src.lh, in_w=src.lw, out_h=src.lh, out_w=src.lw, act=N.ACT_CODE["silu"], dst_f32=False,
            grouped2=True)))
        self.flops += 2.0 * self.batch * src.lh * src.lw * 2 * half * 9 * cin
        return out

    def grouped2_head_fusable(self, head, src: View, train: bool, level: int = 0) -> bool:
        """cls_convs[k][1] | reg_convs[k][1] + the level's preds + decode as ONE conv_ws head-form
        launch (yxh_conv_desc.post_weight / post_weight2): eval, 16-bit, 128 channels per group,
        65-80 classes, 16-byte level rows."""
        return (self.csp_fusion and int(train) == self.HEAD_EVAL and self.dtype != torch.float32 and src.ch == 256
                and 65 <= head.num_classes <= 80 and level in _HEAD_FUSION)

    def conv_grouped2_head(self, ms, src: View, head, k: int, out: "OutBuffer", a_off: int, stride: int) -> None:
        """The two-group 3x3 (cls | reg, yolo_head.py:160-161) whose blocks keep their 128-channel
        tiles in LDS and write the level's decoded rows (reg_preds | obj_preds over reg,
        cls_preds over cls, :149-159, :185-187, :233-251) -- the [cls | reg] map never leaves the
        CU and the separate pred launch disappears."""
        ka, kb = ms[0].conv, ms[1].conv
        cin, half = ka.in_channels, ka.out_channels
        spec = self._weights([(ka, ms[0].bn), (kb, ms[1].bn)], cin)
        ro = self._weights([(head.reg_preds[k], None), (head.obj_preds[k], None)], half)
        cl = self._weights([(head.cls_preds[k], None)], half)
        self.ops.append(OpRec(N.OP_CONV, dict(
            srcs=[src], out=None, residual=None, spec=spec, cin=cin, cout=2 * half, k=3, stride=1, pad=1, groups=1,
            in_h=src.lh, in_w=src.lw, out_h=src.lh, out_w=src.lw, act=N.ACT_CODE["silu"], dst_f32=False,
            grouped2=True, head_post=dict(cls=cl, ro=ro, out=out, a_off=a_off, stride=float(stride),
                                          num_classes=head.num_classes))))
        hw = src.lh * src.lw
        self.flops += 2.0 * self.batch * hw * 2 * half * 9 * cin + 2.0 * self.batch * hw * (5 + head.num_classes) * half

    def spp(self, cat: Buffer, hidden: int) -> None:
        self.ops.append(OpRec(N.OP_SPP, dict(buf=cat, c=hidden)))

    # head output modes: eval rows (decode_outputs), train rows (get_output_and_grid), eval rows
    # without the box decode (decode_in_inference = False, yolo_head.py:208-211)
    HEAD_EVAL, HEAD_TRAIN, HEAD_RAW = 0, 1, 2

    def head_preds(self, k: int, head, cls_feat: View, reg_feat: View, out: "OutBuffer", a_off: int,
                   stride: int, train) -> None:
        """``train``: False / True, or a HEAD_* mode (yxh_head_desc.train)."""
        mode = int(train)
        act = (N.ACT_DECODE, N.ACT_DECODE_TRAIN, N.ACT_DECODE_RAW)[mode]
        train = mode
        h, w = cls_feat.lh, cls_feat.lw
        C = head.num_classes
        if (self.dtype != torch.float32 and cls_feat.ch == reg_feat.ch and cls_feat.ch in (64, 128, 256)
                and 65 <= C <= 80 and (h * w) % 4 == 0 and a_off % 4 == 0 and out.anchors % 4 == 0
                and not cls_feat.up and not reg_feat.up):
            # the three preds + cat + sigmoid + decode of the level as one launch (head.hip)
            ro = self._weights([(head.reg_preds[k], None), (head.obj_preds[k], None)], reg_feat.ch)
            cl = self._weights([(head.cls_preds[k], None)], cls_feat.ch)
            self.ops.append(OpRec(N.OP_HEAD, dict(reg=reg_feat, cls=cls_feat, spec_ro=ro, spec_cls=cl,
                                                  head_out=(out, a_off, 0), h=h, w=w, cin=cls_feat.ch,
                                                  num_classes=C, stride=float(stride), train=int(train))))
            self.flops += 2.0 * self.batch * h * w * (5 + C) * cls_feat.ch
            return
        for convs, feat, coff in (([(head.reg_preds[k], None), (head.obj_preds[k], None)], reg_feat, 0),
                                  ([(head.cls_preds[k], None)], cls_feat, 5)):
            spec = self._weights(convs, feat.ch)
            cout = spec.cout
            self.ops.append(OpRec(N.OP_CONV, dict(
                srcs=[feat], out=None, head_out=(out, a_off, coff), residual=None, spec=spec, cin=feat.ch,
                cout=cout, k=1, stride=1, pad=0, groups=1, in_h=h, in_w=w, out_h=h, out_w=w, act=act,
                decode_stride=float(stride), decode_coff=coff, dst_f32=True)))
            self.flops += 2.0 * self.batch * h * w * cout * feat.ch


@dataclass(eq=False)
class OutBuffer:
    anchors: int
    row: int  # 5 + C


# tile codes (2 * id + slabs - 1); ids 1-9 register-staged conv_igemm, 17-25 the same
# tiles on the LDS-DMA conv_glds kernel, 33-51 the row-tiled 3x3 conv_rows kernel,
# 65-70 the persistent streaming 1x1 conv_pw kernel, 81-82 the register-operand 1x1
# conv_pwr kernel, 97-104 the dense 1x1 conv_pwf kernel, 113-150 the 3x3 conv_r3 kernel
# (yoloxhip.h yxh_conv_desc.tile); for the weight-stationary 1x1 conv_ws1 (201-210, 241-258) the slab bit
# selects the 16-byte-store epilogue instead (round 6)
TILE_CANDIDATES = [2 * i + k for i in list(range(1, 10)) + list(range(17, 26)) + list(range(33, 52))
                   + list(range(65, 71)) for k in (0, 1)] + [2 * 81, 2 * 82] + [2 * i for i in range(97, 105)] + [2 * i for i in range(113, 153)] + [2 * i for i in range(161, 197)] + [2 * i + k for i in range(201, 211) for k in (0, 1)] + [2 * i for i in range(221, 237)] + [2 * i + k for i in range(241, 259) for k in (0, 1)] + [2 * i for i in range(261, 281)]
# 16-bit plans: the families that win on MI355X (profiles/r03/final/tune_r3fa_*.json: yolox_s picks only
# conv_pwf / conv_ws / conv_ws1; yolox_l fp16 also conv_igemm and conv_r3 once or twice); the LDS-DMA
# conv_glds, row-tiled conv_rows and the round-1 pointwise kernels never do and are tried only with
# YOLOX_AMD_TUNE_ALL_FAMILIES=1 (fp32 plans always try every family)
TILE_CANDIDATES_16 = [t for t in TILE_CANDIDATES if (t >> 1) < 17 or (t >> 1) > 96]
_TUNE_ALL_FAMILIES = os.environ.get("YOLOX_AMD_TUNE_ALL_FAMILIES", "0") == "1"
# CUs a graph lane's persistent conv grids may occupy ("lane:cus,..."; yxh_conv_desc.grid_cap): a head
# level forked early (YOLOX_AMD_GRAPH=streams) leaves the rest of the chip to the neck it runs beside
_LANE_CUS = {int(k): int(v) for k, v in (e.split(":") for e in os.environ.get("YOLOX_AMD_LANE_CUS", "").split(",") if e)}
_TUNE_CACHE: dict = {}
_TUNE_TIMES: dict = {}  # shape key -> [(isolated ms, tile)] of every applicable candidate, fastest first
_TUNE_ALL = os.environ.get("YOLOX_AMD_TUNE_ALL", "0") == "1"  # print every variant's time


def save_tune_cache(path: str) -> None:
    """Write the per-shape tile choices (JSON) so another process can skip tuning."""
    import json
    with open(path, "w") as f:
        json.dump([[list(k), v] for k, v in _TUNE_CACHE.items()], f)


def load_tune_cache(path: str) -> int:
    import json
    with open(path) as f:
        for k, v in json.load(f):
            _TUNE_CACHE[tuple(k)] = int(v)
    return len(_TUNE_CACHE)


def _tune_key(d) -> tuple:
    return (d.dtype, d.batch, d.in_h, d.in_w, d.out_h, d.out_w, d.cin, d.cout, d.kh, d.stride, d.nsrc,
            d.src[0].channels, d.src[0].upsample, d.src[1].upsample if d.nsrc > 1 else 0,
            bool(d.residual), d.dst_dtype, d.dst_cstride == d.cout, d.act >= N.ACT_DECODE, bool(d.pre_weight),
            d.flags, d.post_cout, d.post_src.channels, d.post_cout2)


def op_buffers(r: OpRec) -> tuple:
    """(buffers read, buffers written) by one op; the input image and the [B, A, 5+C]
    output rows (disjoint anchor ranges per level, written once) are not tracked."""
    a = r.args
    if r.kind == N.OP_SPP:
        return [a["buf"]], [a["buf"]]
    if r.kind == N.OP_STEM2 and a.get("dst") is None:
        return [], [a["dst3"].buf, a["dst4"].buf]
    if r.kind in (N.OP_FOCUS, N.OP_STEM, N.OP_STEM2):
        return [], [a["dst"].buf]
    if r.kind == N.OP_HEAD:
        return [a["reg"].buf, a["cls"].buf], []
    if a.get("head_post") is not None:  # decoded rows (untracked, like OP_HEAD)
        return [v.buf for v in a["srcs"]], []
    reads = [v.buf for v in a["srcs"]]
    if a.get("residual") is not None:
        reads.append(a["residual"].buf)
    if a.get("post_src") is not None:
        reads.append(a["post_src"].buf)
    writes = [a["out"].buf] if a.get("out") is not None else []
    if a.get("post_out") is not None:
        writes.append(a["post_out"].buf)
    if a.get("post_store_out") is not None:
        writes.append(a["post_store_out"].buf)
    return reads, writes


def dependencies_rw(rw: list) -> list:
    """Per op, the earlier ops it must wait for, from (read keys, write keys) per op:
    read-after-write, write-after-write and write-after-read edges."""
    last_w: dict = {}
    readers: dict = {}
    deps = []
    for i, (reads, writes) in enumerate(rw):
        d = set()
        for b in list(reads) + list(writes):
            if b in last_w:
                d.add(last_w[b])
        for b in writes:
            d.update(readers.get(b, ()))
        d.discard(i)
        for b in reads:
            readers.setdefault(b, []).append(i)
        for b in writes:
            last_w[b] = i
            readers[b] = []
        deps.append(sorted(d))
    return deps


def hoist_lanes(ops) -> list:
    """The op list reordered so that every graph-lane op (a head level, ``OpRec.lane`` > 0)
    directly follows the last op it depends on, instead of the whole neck: the op order is the
    capture order of the lanes graph, and the runtime dispatches a branch's nodes in that order,
    so a level planned after the neck (yolo_head.py:140-211 runs after yolo_pafpn.py:71-112)
    otherwise queues behind the other levels' work although its input (the 80x80 PAN output)
    is ready long before them.  Lane-0 order and each lane's own order are kept; the result is a
    topological order of the same dataflow DAG (``op_dependencies``)."""
    deps = op_dependencies(ops)
    placed = [False] * len(ops)
    order = []
    pending = [i for i, r in enumerate(ops) if r.lane != 0]
    for i, r in enumerate(ops):
        if r.lane != 0:
            continue
        order.append(i)
        placed[i] = True
        grew = True
        while grew:
            grew = False
            for j in pending:
                if not placed[j] and all(placed[k] for k in deps[j]):
                    order.append(j)
                    placed[j] = True
                    grew = True
    order += [j for j in pending if not placed[j]]
    return [ops[i] for i in order]


def op_dependencies(ops) -> list:
    """Per op, the earlier ops it must wait for, from the buffers it reads and writes
    (read-after-write, write-after-write, write-after-read).  Arena buffers never alias
    (bump allocation)."""
    rw = []
    for r in ops:
        reads, writes = op_buffers(r)
        rw.append(([id(b) for b in reads], [id(b) for b in writes]))
    return dependencies_rw(rw)


class Plan:
    """A finalised op list with its arenas.  ``run(x)`` executes one forward pass.

    ``chunk``: the op list is planned for ``chunk`` images and executed batch/chunk
    times (input and output pointers advance per chunk).  By default the chunks share
    one activation arena and run back to back (each layer's output is still in the
    MI355X Infinity Cache when the next layer reads it); with ``parallel_chunks`` every
    chunk gets an arena of its own, so in the captured dataflow graph the chunks are
    independent chains that the device runs side by side (one chunk's small layers and
    kernel boundaries overlap the other's work).  The result is identical to an
    unchunked plan either way."""

    def __init__(self, model, batch: int, height: int, width: int, dtype: torch.dtype, device,
                 input_layout: int = N.NCHW, input_dtype: torch.dtype = torch.float32, train: bool = False,
                 fuse_stem: bool = True, chunk: Optional[int] = None, fuse_bottleneck: bool = _FUSE_BOTTLENECK,
                 parallel_chunks: bool = False, fuse_stem_s2: bool = True, stage: str = "full",
                 head_inputs: Optional[list] = None, csp_fusion: Optional[bool] = None, block=None):
        """``stage``: "full" (image -> decoded rows), "features" (image -> the three PAFPN
        maps: YoloPafpn.forward), "head" (three feature maps of ``head_inputs`` shapes
        [(C, H, W)] -> decoded rows: YoloxHead.forward) or "block" (one building block of the
        module tree -- ``block.plan_block`` -- over one NCHW map of ``head_inputs[0]``'s shape, or
        over the image when ``block.takes_image``: the blocks' standalone forward)."""
        if stage not in ("full", "features", "head", "block"):
            raise ValueError(f"unknown plan stage {stage!r}")
        self.stage = stage
        if stage == "block":
            if block is None or (not block.takes_image and (not head_inputs or len(head_inputs) != 1)):
                raise ValueError("a block plan takes the block and its one input shape")
            if block.takes_image and (height % 2 or width % 2):
                raise ValueError("the Focus stem needs an even input size")
        elif height % 32 or width % 32:
            raise ValueError("input size must be multiples of 32")
        chunk = chunk or batch
        if chunk <= 0 or batch % chunk:
            raise ValueError(f"chunk {chunk} must divide batch {batch}")
        self.lib = N.lib()
        self.chunk, self.nchunks = chunk, batch // chunk
        self.parallel_chunks = bool(parallel_chunks) and self.nchunks > 1
        self.batch, self.height, self.width = batch, height, width
        self.device = torch.device(device)
        self.input_layout = input_layout
        self.input_dtype = input_dtype
        self.dtype = dtype
        head = model.head
        self.num_classes = head.num_classes if head is not None else 0
        ctx = PlanCtx(chunk, dtype, self.device, fuse_stem=fuse_stem, fuse_bottleneck=fuse_bottleneck,
                      fuse_stem_s2=fuse_stem_s2, csp_fusion=csp_fusion)
        ctx.input_layout, ctx.input_dtype = input_layout, input_dtype
        if stage == "head":
            if chunk != batch or not head_inputs or len(head_inputs) != 3:
                raise ValueError("a head plan takes three feature maps and no chunking")
            feats = [ctx.buffer(h, w, c).full() for c, h, w in head_inputs]
        elif stage == "block":
            if chunk != batch:
                raise ValueError("a block plan takes no chunking")
            if block.takes_image:
                self.block_input = None
                outs = block.plan_block(ctx, ctx.image(height, width))
            else:
                c, h, w = head_inputs[0]
                self.block_input = ctx.buffer(h, w, c).full()
                outs = block.plan_block(ctx, self.block_input)
            feats = list(outs) if isinstance(outs, (tuple, list)) else [outs]
        else:
            feats = model.backbone.plan(ctx, ctx.image(height, width))
        self.feats = feats
        anchors = sum(f.lh * f.lw for f in feats)
        self.out_spec = OutBuffer(anchors, 5 + self.num_classes)
        if stage in ("full", "head"):
            head.plan(ctx, feats, self.out_spec, train=train)
        elif chunk != batch:
            raise ValueError("a features plan takes no chunking")
        self.ctx = ctx
        self.anchors = anchors
        # independent head levels run as separate graph branches (YOLOX_AMD_LANES=0: one stream)
        self.nlanes = 1 + max((r.lane for r in ctx.ops), default=0)
        # YOLOX_AMD_LANE_HOIST=1 moves each head level up to its input (engine.hoist_lanes): level 0
        # then overlaps the PAFPN bottom-up path, but on MI355X the forward got slower (1.635-1.641 vs
        # 1.629-1.631 ms, profiles/r05/lane_hoist_ab.txt): the level-0 head convs take every CU and
        # the neck's small layers stretch 3-5x beside them -- the chip is already full, so it stays off
        if self.nlanes > 1 and os.environ.get("YOLOX_AMD_LANE_HOIST", "0") == "1":
            ctx.ops[:] = hoist_lanes(ctx.ops)
        self._deps = op_dependencies(ctx.ops)
        self.use_lanes = os.environ.get("YOLOX_AMD_LANES", "1") != "0"
        # captured graph form: "lanes" (multi-stream capture: head levels on lanes, or one lane
        # per chunk with parallel_chunks; default), "dag" (one child-graph node per op, dataflow
        # edges), "linear" (one stream).  Measured on MI355X (profiles/r03/graph_forms.txt):
        # yolox_s bs32 forward 1.97 ms as lanes vs 2.27 ms as the DAG -- the runtime pays for
        # every cross-stream edge of a many-branch graph
        self.graph_mode = os.environ.get("YOLOX_AMD_GRAPH", "lanes")
        self._segments = None  # graph_mode "streams": per-segment graphs + lane streams / events
        self.flops = ctx.flops * self.nchunks
        # ------------------------------------------------ arenas
        off = 0
        for b in ctx.buffers:
            b.offset = off
            off += _align(chunk * b.nelem_image * b.esize)
        self.act_bytes = off  # one chunk's activations
        narenas = self.nchunks if self.parallel_chunks else 1
        self.arena = torch.empty(max(off * narenas, 1), dtype=torch.uint8, device=self.device)
        woff = boff = 0
        for s in ctx.weights:
            s.w_off = woff
            s.b_off = boff
            if s.stem:
                cpad = (s.cout + 15) // 16 * 16
                woff += _align(cpad * 6 * 32 * ctx.esize)
                boff += _align(cpad * 4)
            else:
                woff += _align(s.cout * s.kh * s.kw * s.cin_pad * ctx.esize)
                boff += _align(s.cout * 4)
        self.warena = torch.empty(max(woff, 1), dtype=torch.uint8, device=self.device)
        # fragment-major copies of the 16-bit conv weights the weight-stationary tiles
        # (conv_ws / conv_ws1) load as whole 1 KiB wave reads (yxh_conv_desc.weight_frag)
        foff = 0
        if dtype != torch.float32 and _WFRAG:
            for rec in ctx.ops:
                a = rec.args
                if rec.kind != N.OP_CONV or a["dst_f32"] or a["groups"] != 1:
                    continue
                sp: WeightSpec = a["spec"]
                if sp.f_off < 0 and not sp.stem and sp.cout % 16 == 0 and sp.cin_pad % 32 == 0:
                    sp.f_off = foff
                    foff += _align(sp.cout * sp.kh * sp.kw * sp.cin_pad * ctx.esize)
        self.farena = torch.empty(max(foff, 1), dtype=torch.uint8, device=self.device)
        self.barena = torch.empty(max(boff, 1), dtype=torch.uint8, device=self.device)
        self.output = torch.empty(batch, anchors if stage in ("full", "head") else 0, 5 + self.num_classes,
                                  dtype=torch.float32, device=self.device)
        self._input_slot: Optional[torch.Tensor] = None
        self._nops = len(ctx.ops)
        self._ops = (N.Op * (len(ctx.ops) * self.nchunks))()  # chunk c = ops [c*nops, (c+1)*nops)
        self._input_index = None
        self._graph = None
        # a second graph of the same forward writing its rows to ``output_alt`` (capture(slots=2)):
        # a serving loop alternates the two, so batch k+1's forward never waits for batch k's NMS
        # to finish reading the rows
        self._graph_alt = None
        self.output_alt: Optional[torch.Tensor] = None
        # per-anchor serving score records written by the head launches (enable_scores, ABI 18)
        self.scores: Optional[torch.Tensor] = None
        self._graph_ptrs = None
        self._param_sig = None
        self._packed_epoch = -1
        self._model = model
        self._encode_ops()

    # -------------------------------------------------------------- encoding
    def _ptr(self, v: View, c: int = 0) -> int:
        return self._arena_base(c) + v.buf.offset + v.coff * v.buf.esize

    def _arena_base(self, c: int) -> int:
        """Activation arena of chunk c (all chunks share one unless parallel_chunks)."""
        return self.arena.data_ptr() + (c * self.act_bytes if self.parallel_chunks else 0)

    def _encode_ops(self) -> None:
        for c in range(self.nchunks):
            self._encode_chunk(c)

    def _encode_chunk(self, c: int, out_ptr: Optional[int] = None, heads_only: bool = False) -> None:
        ctx, B = self.ctx, self.chunk
        out_ptr = self.output.data_ptr() if out_ptr is None else out_ptr
        out_base = out_ptr + c * B * self.anchors * self.out_spec.row * 4
        for i, rec in enumerate(ctx.ops):
            a = rec.args
            if heads_only and not (rec.kind == N.OP_HEAD or (rec.kind == N.OP_CONV and (a["dst_f32"] or
                                                                                       a.get("head_post")))):
                continue
            op = self._ops[c * self._nops + i]
            op.kind = rec.kind
            if rec.kind == N.OP_FOCUS:
                f = op.u.focus
                f.layout = self.input_layout
                f.img_dtype = N.DTYPE_CODE[self.input_dtype]
                f.batch, f.h, f.w = B, a["h"], a["w"]
                f.dst_dtype = ctx.dcode
                f.dst = self._ptr(a["dst"], c)
                f.img = None
                self._input_index = i
            elif rec.kind == N.OP_STEM:
                t = op.u.stem
                t.layout = self.input_layout
                t.img_dtype = N.DTYPE_CODE[self.input_dtype]
                t.batch, t.h, t.w = B, a["h"], a["w"]
                t.dtype, t.cout, t.act = ctx.dcode, a["spec"].cout, a["act"]
                t.weight = self.warena.data_ptr() + a["spec"].w_off
                t.bias = self.barena.data_ptr() + a["spec"].b_off
                v = a["dst"]
                t.dst = self._ptr(v, c)
                t.dst_cstride, t.dst_bstride = v.buf.c, v.buf.nelem_image
                t.img = None
                self._input_index = i
            elif rec.kind == N.OP_STEM2:
                t = op.u.stem2
                t.layout = self.input_layout
                t.img_dtype = N.DTYPE_CODE[self.input_dtype]
                t.batch, t.h, t.w = B, a["h"], a["w"]
                t.dtype, t.c1, t.c2, t.act = ctx.dcode, a["c1"], a["c2"], a["act"]
                t.w1 = self.warena.data_ptr() + a["spec1"].w_off
                t.b1 = self.barena.data_ptr() + a["spec1"].b_off
                t.w2 = self.warena.data_ptr() + a["spec2"].w_off
                t.b2 = self.barena.data_ptr() + a["spec2"].b_off
                v = a["dst"]
                if v is not None:
                    t.dst = self._ptr(v, c)
                    t.dst_cstride, t.dst_bstride = v.buf.c, v.buf.nelem_image
                else:  # CSP form: conv1 | conv2 -> dst3, the first Bottleneck's conv1 -> dst4
                    t.dst = None
                    for name, spec, view in (("3", a["spec3"], a["dst3"]), ("4", a["spec4"], a["dst4"])):
                        setattr(t, "w" + name, self.warena.data_ptr() + spec.w_off)
                        setattr(t, "b" + name, self.barena.data_ptr() + spec.b_off)
                        setattr(t, "dst" + name, self._ptr(view, c))
                        setattr(t, f"dst{name}_cstride", view.buf.c)
                        setattr(t, f"dst{name}_bstride", view.buf.nelem_image)
                t.img = None
                self._input_index = i
            elif rec.kind == N.OP_HEAD:
                hd = op.u.head
                hd.dtype, hd.batch, hd.h, hd.w = ctx.dcode, B, a["h"], a["w"]
                hd.cin, hd.num_classes = a["cin"], a["num_classes"]
                for dst, v in ((hd.reg, a["reg"]), (hd.cls, a["cls"])):
                    dst.ptr = self._ptr(v, c)
                    dst.channels, dst.cstride, dst.bstride = v.ch, v.buf.c, v.buf.nelem_image
                    dst.h, dst.w, dst.upsample = v.buf.h, v.buf.w, 0
                hd.w_reg = self.warena.data_ptr() + a["spec_ro"].w_off
                hd.b_reg = self.barena.data_ptr() + a["spec_ro"].b_off
                hd.w_cls = self.warena.data_ptr() + a["spec_cls"].w_off
                hd.b_cls = self.barena.data_ptr() + a["spec_cls"].b_off
                out, a_off, _ = a["head_out"]
                hd.out = out_base
                hd.out_bstride = out.anchors * out.row
                hd.a_off, hd.stride, hd.train = a_off, a["stride"], a["train"]
                hd.scores = (self.scores.data_ptr() + c * B * self.anchors * 32) if self.scores is not None else None
            elif rec.kind == N.OP_SPP:
                s = op.u.spp
                buf: Buffer = a["buf"]
                s.buf = self._arena_base(c) + buf.offset
                s.dtype, s.batch, s.h, s.w, s.c = ctx.dcode, B, buf.h, buf.w, a["c"]
                s.cstride, s.bstride = buf.c, buf.nelem_image
            else:
                d = op.u.conv
                d.dtype, d.batch = ctx.dcode, B
                d.in_h, d.in_w, d.out_h, d.out_w = a["in_h"], a["in_w"], a["out_h"], a["out_w"]
                d.cin, d.cout, d.kh, d.kw = a["cin"], a["cout"], a["k"], a["k"]
                d.stride, d.pad, d.groups = a["stride"], a["pad"], a["groups"]
                d.nsrc = len(a["srcs"])
                for j, v in enumerate(a["srcs"]):
                    s = d.src[j]
                    s.ptr = self._ptr(v, c)
                    s.channels, s.cstride, s.bstride = v.ch, v.buf.c, v.buf.nelem_image
                    s.h, s.w, s.upsample = v.buf.h, v.buf.w, v.up
                spec: WeightSpec = a["spec"]
                d.weight = self.warena.data_ptr() + spec.w_off
                d.bias = self.barena.data_ptr() + spec.b_off
                d.flags = N.CONV_GROUPS2 if a.get("grouped2") else 0
                d.grid_cap = _LANE_CUS.get(rec.lane, 0)
                d.weight_frag = self.farena.data_ptr() + spec.f_off if spec.f_off >= 0 else None
                pre = a.get("pre_spec")
                if pre is not None:
                    d.pre_weight = self.warena.data_ptr() + pre.w_off
                    d.pre_bias = self.barena.data_ptr() + pre.b_off
                res = a["residual"]
                if res is not None:
                    d.residual = self._ptr(res, c)
                    d.res_cstride, d.res_bstride = res.buf.c, res.buf.nelem_image
                d.act = a["act"]
                pspec = a.get("post_spec")
                hp = a.get("head_post")
                if hp is not None:  # head form: each group's preds + decode into the level's rows
                    out, a_off = hp["out"], hp["a_off"]
                    d.post_weight = self.warena.data_ptr() + hp["cls"].w_off
                    d.post_bias = self.barena.data_ptr() + hp["cls"].b_off
                    d.post_weight2 = self.warena.data_ptr() + hp["ro"].w_off
                    d.post_bias2 = self.barena.data_ptr() + hp["ro"].b_off
                    d.post_cout, d.post_cout2, d.post_stride = hp["num_classes"], 5, hp["stride"]
                    d.post_dst = out_base + a_off * out.row * 4
                    d.post_dst_cstride, d.post_dst_bstride = out.row, out.anchors * out.row
                    d.dst = d.post_dst
                    d.dst_dtype = ctx.dcode
                    d.dst_cstride, d.dst_bstride = out.row, out.anchors * out.row
                elif pspec is not None:  # 1x1 post conv: its output replaces the conv's own
                    d.post_weight = self.warena.data_ptr() + pspec.w_off
                    d.post_bias = self.barena.data_ptr() + pspec.b_off
                    d.post_cout = pspec.cout
                    ps = a["post_src"]
                    if ps is not None:
                        q = d.post_src
                        q.ptr = self._ptr(ps, c)
                        q.channels, q.cstride, q.bstride = ps.ch, ps.buf.c, ps.buf.nelem_image
                        q.h, q.w, q.upsample = ps.buf.h, ps.buf.w, 0
                    po = a["post_out"]
                    d.post_dst = self._ptr(po, c)
                    d.post_dst_cstride, d.post_dst_bstride = po.buf.c, po.buf.nelem_image
                    so = a.get("post_store_out")
                    if so is not None:  # the Bottleneck chain: the 3x3's output is stored as well
                        d.flags |= N.CONV_POST_STORE
                        po = so
                    d.dst = self._ptr(po, c)
                    d.dst_dtype = ctx.dcode
                    d.dst_cstride, d.dst_bstride = po.buf.c, po.buf.nelem_image
                elif a["dst_f32"]:
                    out, a_off, coff = a["head_out"]
                    row = out.row
                    d.dst = out_base + (a_off * row + coff) * 4
                    d.dst_dtype = N.F32
                    d.dst_cstride, d.dst_bstride = row, out.anchors * row
                    d.decode_stride, d.decode_coff = a["decode_stride"], a["decode_coff"]
                else:
                    v = a["out"]
                    d.dst = self._ptr(v, c)
                    d.dst_dtype = ctx.dcode
                    d.dst_cstride, d.dst_bstride = v.buf.c, v.buf.nelem_image

    # -------------------------------------------------------------- weights
    def _signature(self):
        # parameters and buffers (BN running statistics), by storage and version counter
        m = self._model
        return tuple((t.data_ptr(), t._version) for t in list(m.parameters()) + list(m.buffers()))

    def _epoch(self) -> int:
        return getattr(self._model, "_weights_epoch", 0)

    def pack_weights(self, force: bool = False) -> None:
        sig = self._signature()
        if not force and sig == self._param_sig:
            self._packed_epoch = self._epoch()
            return
        stream = N.stream_ptr(self.device)
        dt = self.ctx.dcode
        keep = []
        # a 16-bit YoloxModule folds from the float32 values it had before its cast (models/yolox.py
        # fp32_master): the packed weights are then rounded once, like the oracle's bf16 emulation; a
        # submodule of a YoloxModule planned on its own (module.backbone(x), a block) holds the
        # module's masters as _fold_masters
        from .models.yolox import fold_master
        masters = self._model.__dict__.get("_masters") or self._model.__dict__.get("_fold_masters") or {}

        def f32(t):
            m = fold_master(masters, t)
            return (m if m is not None else t.detach()).to(self.device, torch.float32).contiguous()

        for s in self.ctx.weights:
            row = 0
            for conv, bn in s.convs:
                w = f32(conv.weight)
                keep.append(w)
                args = [None, None, None, None, None]
                if conv.bias is not None:
                    args[0] = f32(conv.bias)
                if bn is not None:
                    args[1:] = [f32(t) for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var)]
                keep.extend(a for a in args if a is not None)
                eps = float(bn.eps) if bn is not None else 0.0
                ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
                if s.stem:
                    if args[0] is not None:
                        raise NotImplementedError("fused stem conv with a conv bias")
                    N.check(self.lib.yxh_stem_pack(
                        w.data_ptr(), ptr(args[1]), ptr(args[2]), ptr(args[3]), ptr(args[4]), eps,
                        conv.out_channels, dt, self.warena.data_ptr() + s.w_off,
                        self.barena.data_ptr() + s.b_off, stream), "stem_pack")
                    continue
                wout = self.warena.data_ptr() + s.w_off + row * s.kh * s.kw * s.cin_pad * self.ctx.esize
                bout = self.barena.data_ptr() + s.b_off + row * 4
                N.check(self.lib.yxh_fold_bn_pack(
                    w.data_ptr(), ptr(args[0]), ptr(args[1]), ptr(args[2]), ptr(args[3]), ptr(args[4]), eps,
                    conv.out_channels, conv.in_channels // conv.groups, s.kh, s.kw, s.cin_pad, dt, wout, bout,
                    stream), "fold_bn_pack")
                row += conv.out_channels
            if s.f_off >= 0:
                N.check(self.lib.yxh_pack_frag(self.warena.data_ptr() + s.w_off, s.cout, s.kh * s.kw, s.cin_pad, dt,
                                               self.farena.data_ptr() + s.f_off, stream), "pack_frag")
        torch.cuda.current_stream(self.device).synchronize()  # `keep` tensors die after this
        del keep
        self._param_sig = sig
        self._packed_epoch = self._epoch()

    # -------------------------------------------------------------- execution
    def _bind_input(self, x: torch.Tensor) -> torch.Tensor:
        B, H, W = self.batch, self.height, self.width
        expect = (B, 3, H, W) if self.input_layout == N.NCHW else (B, H, W, 3)
        if tuple(x.shape) != expect:
            raise ValueError(f"input shape {tuple(x.shape)} != planned {expect}")
        if x.dtype != self.input_dtype:
            raise ValueError(f"input dtype {x.dtype} != planned {self.input_dtype}")
        if x.device != self.device:
            x = x.to(self.device, non_blocking=True)
        x = x.contiguous()
        step = self.chunk * x[0].numel() * x.element_size()
        for c in range(self.nchunks):
            op = self._ops[c * self._nops + self._input_index]
            if op.kind == N.OP_STEM:
                op.u.stem.img = x.data_ptr() + c * step
            elif op.kind == N.OP_STEM2:
                op.u.stem2.img = x.data_ptr() + c * step
            else:
                op.u.focus.img = x.data_ptr() + c * step
        return x

    def _bind_output(self, out: Optional[torch.Tensor]) -> None:
        """Point the head-pred ops' decoded rows at ``out`` (None: the plan's own buffer)."""
        ptr = None
        if out is not None:
            if (tuple(out.shape) != tuple(self.output.shape) or out.dtype != torch.float32 or out.device != self.device
                    or not out.is_contiguous()):
                raise ValueError(f"output must be a contiguous float32 {tuple(self.output.shape)} tensor on "
                                 f"{self.device}")
            ptr = out.data_ptr()
        for c in range(self.nchunks):
            self._encode_chunk(c, ptr, heads_only=True)

    def run(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Eager execution of the op list on the current stream.  Writes ``out`` if given
        (a fresh tensor the caller owns), else returns the plan's output buffer
        [B, A, 5+C] (overwritten by the next run)."""
        self.pack_weights()
        x = self._bind_input(x)
        if out is None:
            N.check(self.lib.yxh_run_ops(self._ops, len(self._ops), N.stream_ptr(self.device)), "forward")
            return self.output
        self._bind_output(out)
        try:
            N.check(self.lib.yxh_run_ops(self._ops, len(self._ops), N.stream_ptr(self.device)), "forward")
        finally:
            self._bind_output(None)
        return out

    def feature_view(self, v: View) -> torch.Tensor:
        """An arena view as an NCHW tensor (a copy) in the compute dtype."""
        b = v.buf
        t = self.arena[b.offset:b.offset + self.batch * b.nelem_image * b.esize].view(self.dtype)
        return t.view(self.batch, b.h, b.w, b.c)[..., v.coff:v.coff + v.ch].permute(0, 3, 1, 2).contiguous()

    def run_features(self, x: torch.Tensor) -> tuple:
        """stage "features": the PAFPN outputs (pan_out2, pan_out1, pan_out0), NCHW."""
        if self.stage != "features":
            raise RuntimeError("run_features needs a features plan")
        self.pack_weights()
        self._bind_input(x)
        N.check(self.lib.yxh_run_ops(self._ops, len(self._ops), N.stream_ptr(self.device)), "backbone")
        return tuple(self.feature_view(v) for v in self.feats)

    def run_block(self, x: torch.Tensor) -> list:
        """stage "block": the block's output map(s) of one NCHW input, NCHW in the compute dtype."""
        if self.stage != "block":
            raise RuntimeError("run_block needs a block plan")
        self.pack_weights()
        if self.block_input is None:
            self._bind_input(x)
        else:
            b = self.block_input.buf
            if tuple(x.shape) != (self.batch, b.c, b.h, b.w):
                raise ValueError(f"input shape {tuple(x.shape)} != planned {(self.batch, b.c, b.h, b.w)}")
            dst = self.arena[b.offset:b.offset + self.batch * b.nelem_image * b.esize].view(self.dtype)
            dst.view(self.batch, b.h, b.w, b.c).copy_(x.to(self.device).permute(0, 2, 3, 1))
        N.check(self.lib.yxh_run_ops(self._ops, len(self._ops), N.stream_ptr(self.device)), "block")
        return [self.feature_view(v) for v in self.feats]

    def run_head(self, xin, out: torch.Tensor) -> torch.Tensor:
        """stage "head": decoded [B, A, 5+C] rows of three NCHW feature maps."""
        if self.stage != "head":
            raise RuntimeError("run_head needs a head plan")
        self.pack_weights()
        for v, x in zip(self.feats, xin):
            b = v.buf
            dst = self.arena[b.offset:b.offset + self.batch * b.nelem_image * b.esize].view(self.dtype)
            dst.view(self.batch, b.h, b.w, b.c).copy_(x.to(self.device).permute(0, 2, 3, 1))
        self._bind_output(out)
        try:
            N.check(self.lib.yxh_run_ops(self._ops, len(self._ops), N.stream_ptr(self.device)), "head")
        finally:
            self._bind_output(None)
        return out

    def static_input(self) -> torch.Tensor:
        """The fixed input buffer a captured graph reads."""
        if self._input_slot is None:
            shape = ((self.batch, 3, self.height, self.width) if self.input_layout == N.NCHW
                     else (self.batch, self.height, self.width, 3))
            self._input_slot = torch.zeros(shape, dtype=self.input_dtype, device=self.device)
        return self._input_slot

    def _stream_segments(self):
        """graph_mode "streams": the op list cut into graph segments per lane.  A head lane
        k (one level, yolo_head.py:140-211) is one segment that may start as soon as the
        neck op producing its feature map is done (its fork point); the neck / backbone
        lane is cut at every fork point.  None when the lanes do not have that shape."""
        ops, deps = self.ctx.ops, self._deps
        lane = [r.lane for r in ops]
        if max(lane) == 0:
            return None
        fork = {}
        for i, r in enumerate(ops):
            for j in deps[i]:
                if lane[j] != lane[i]:
                    if lane[i] == 0 or lane[j] != 0:
                        return None  # the neck never waits for a head lane; lanes meet only via lane 0
                    fork[lane[i]] = max(fork.get(lane[i], -1), j)
        cuts = sorted(set(fork.values()))
        segs, start = [], 0
        main = [i for i in range(len(ops)) if lane[i] == 0]
        if main != list(range(len(main))):
            return None
        for c in cuts + [len(main) - 1]:
            if c >= start:
                segs.append((0, list(range(start, c + 1)), [k for k, f in fork.items() if f == c]))
                start = c + 1
        lanes = {k: [i for i in range(len(ops)) if lane[i] == k] for k in fork}
        return segs, lanes

    def _capture_segment(self, idx: list, c: int):
        n = self._nops
        arr = (N.Op * len(idx))(*[self._ops[c * n + i] for i in idx])
        g = C.c_void_p()
        N.check(self.lib.yxh_graph_create(arr, len(idx), N.stream_ptr(self.device), C.byref(g)), "graph capture")
        return g

    def _capture_streams(self) -> bool:
        shape = self._stream_segments()
        if shape is None:
            return False
        segs, lanes = shape
        plan = []
        for c in range(self.nchunks):
            chunk = []
            for _, idx, forks in segs:
                chunk.append((self._capture_segment(idx, c), [(k, self._capture_segment(lanes[k], c)) for k in forks]))
            plan.append(chunk)
        ks = sorted(lanes)
        self._lane_streams = {k: torch.cuda.Stream(self.device) for k in ks}
        self._fork_ev = {k: torch.cuda.Event() for k in ks}
        self._done_ev = {k: torch.cuda.Event() for k in ks}
        self._segments = plan
        return True

    def _launch_streams(self) -> None:
        main = torch.cuda.current_stream(self.device)
        mp = main.cuda_stream
        for chunk in self._segments:
            for g, forks in chunk:
                N.check(self.lib.yxh_graph_launch(g, mp), "graph replay")
                for k, gk in forks:
                    s = self._lane_streams[k]
                    self._fork_ev[k].record(main)
                    s.wait_event(self._fork_ev[k])
                    N.check(self.lib.yxh_graph_launch(gk, s.cuda_stream), "graph replay (lane)")
                    self._done_ev[k].record(s)
            for k in self._lane_streams:  # join: outputs ready / arena free on the caller's stream
                main.wait_event(self._done_ev[k])

    def _destroy_graphs(self) -> None:
        if self._graph is not None:
            N.check(self.lib.yxh_graph_destroy(self._graph))
            self._graph = None
        if self._graph_alt is not None:
            N.check(self.lib.yxh_graph_destroy(self._graph_alt))
            self._graph_alt = None
        if self._segments is not None:
            for chunk in self._segments:
                for g, forks in chunk:
                    self.lib.yxh_graph_destroy(g)
                    for _, gk in forks:
                        self.lib.yxh_graph_destroy(gk)
            self._segments = None

    def enable_scores(self) -> Optional[torch.Tensor]:
        """Have the head launches also write per-anchor serving records [B, A, 8] fp32
        {obj * max class, max class, class index, obj, cx, cy, w, h} (yxh_head_desc.scores), which
        ``postprocess_device(..., scores=)`` filters instead of the rows (32 instead of 340 bytes read
        per anchor).  The records belong to the forward that wrote the output
        rows: the next forward overwrites them.  Eval decode plans whose every level is one
        head_pred launch over 64 / 128 / 256 16-bit channels only; returns None (nothing enabled)
        otherwise.  Call before capture()."""
        if self._graph is not None or self._graph_alt is not None:
            raise RuntimeError("enable_scores() before capture()")
        heads = [r for r in self.ctx.ops if r.kind == N.OP_HEAD]
        other = [r for r in self.ctx.ops if r.kind == N.OP_CONV and (r.args["dst_f32"] or r.args.get("head_post"))]
        if (self.stage != "full" or not heads or other or self.ctx.dtype == torch.float32
                or any(r.args["cin"] not in (64, 128, 256) or r.args["train"] != PlanCtx.HEAD_EVAL for r in heads)):
            return None
        if self.scores is None:
            self.scores = torch.zeros(self.batch, self.anchors, 8, dtype=torch.float32, device=self.device)
            self._encode_ops()
        return self.scores

    def capture(self, slots: int = 1) -> None:
        """Capture the whole forward into a hipGraph reading ``static_input()``; ``slots`` = 2
        also captures it writing ``output_alt`` (replay(1))."""
        if slots not in (1, 2):
            raise ValueError("slots must be 1 or 2")
        if slots == 2 and self.scores is not None:
            raise NotImplementedError("score records are single-buffered: one output slot")
        self.pack_weights()
        self._bind_input(self.static_input())
        self._destroy_graphs()
        torch.cuda.synchronize(self.device)
        if self.graph_mode == "streams" and not self.parallel_chunks and self._capture_streams():
            if slots == 2:
                raise NotImplementedError("two output slots need a single-graph capture form")
            return
        self._graph = self._capture_graph()
        if slots == 2:
            if self.output_alt is None:
                self.output_alt = torch.empty_like(self.output)
            self._bind_output(self.output_alt)
            try:
                self._graph_alt = self._capture_graph()
            finally:
                self._bind_output(None)

    def _capture_graph(self):
        g = C.c_void_p()
        if self.graph_mode == "dag":
            off, deps = self._dag_arrays()
            N.check(self.lib.yxh_graph_create_dag(self._ops, len(self._ops), off, deps, N.stream_ptr(self.device),
                                                  C.byref(g)), "graph capture (dag)")
        elif self.graph_mode == "lanes" and self.parallel_chunks and self.nchunks <= 8:  # yxh_graph_create_lanes cap
            # one capture stream per chunk: independent chains, joined at the end
            lanes = [c for c in range(self.nchunks) for _ in self.ctx.ops]
            off, deps = self._dag_arrays()
            arr = (C.c_int32 * len(lanes))(*lanes)
            N.check(self.lib.yxh_graph_create_lanes(self._ops, len(self._ops), arr, off, deps, self.nchunks,
                                                    N.stream_ptr(self.device), C.byref(g)), "graph capture (chunk lanes)")
        elif self.graph_mode == "lanes" and self.use_lanes and self.nlanes > 1 and not self.parallel_chunks:
            lanes, off, deps = self._lane_arrays()
            N.check(self.lib.yxh_graph_create_lanes(self._ops, len(self._ops), lanes, off, deps, self.nlanes,
                                                    N.stream_ptr(self.device), C.byref(g)), "graph capture (lanes)")
        else:
            N.check(self.lib.yxh_graph_create(self._ops, len(self._ops), N.stream_ptr(self.device), C.byref(g)),
                    "graph capture")
        return g

    def _dag_arrays(self):
        """(dep_off, deps) of the dataflow DAG over all chunks: buffers are keyed by arena
        (per chunk with parallel_chunks, else shared), so chunks that share an arena are
        ordered by their write-after-read / write-after-write edges and independent
        chunks are not ordered at all."""
        rw = []
        for c in range(self.nchunks):
            arena = c if self.parallel_chunks else 0
            for r in self.ctx.ops:
                reads, writes = op_buffers(r)
                rw.append(([(arena, id(b)) for b in reads], [(arena, id(b)) for b in writes]))
        deps_all = dependencies_rw(rw)
        off, deps = [0], []
        for d in deps_all:
            deps.extend(d)
            off.append(len(deps))
        arr = lambda v: (C.c_int32 * max(1, len(v)))(*v)  # noqa: E731
        return arr(off), arr(deps)

    def _lane_arrays(self):
        """(lanes, dep_off, deps) over all chunks.  Chunk c reuses chunk c-1's arena: its
        first op (lane 0) also waits for the last op of every lane of c-1; the head lanes
        of chunk c follow from their inputs (lane-0 ops of chunk c) and stream order."""
        n = self._nops
        last = {}
        for i, r in enumerate(self.ctx.ops):
            last[r.lane] = i
        lanes, off, deps = [], [0], []
        for c in range(self.nchunks):
            for i, r in enumerate(self.ctx.ops):
                lanes.append(r.lane)
                d = {c * n + j for j in self._deps[i]}
                if c and i == 0:
                    d.update((c - 1) * n + j for j in last.values())
                deps.extend(sorted(d))
                off.append(len(deps))
        arr = lambda v: (C.c_int32 * max(1, len(v)))(*v)  # noqa: E731
        return arr(lanes), arr(off), arr(deps)

    def replay(self, slot: int = 0) -> torch.Tensor:
        """Launch the captured forward (``slot`` 1: the graph writing ``output_alt``, see
        capture(slots=2)).  Parameters changed since the last packing are
        re-folded into the same weight arena first (the graph reads it in place); on this
        serving path the check is the module's weights epoch (one integer compare), which
        load_state_dict, FusedStep.step and YoloxModule.weights_changed() advance --
        in-place edits made any other way need weights_changed() before the next replay.
        ``run()`` (the eager API path) compares every parameter's version instead."""
        if self._packed_epoch != self._epoch():
            self.pack_weights()
        if self._graph is None and self._segments is None:
            self.capture(2 if slot else 1)
        if slot:
            if self._graph_alt is None:
                raise RuntimeError("replay(1) needs capture(slots=2)")
            N.check(self.lib.yxh_graph_launch(self._graph_alt, N.stream_ptr(self.device)), "graph replay")
            return self.output_alt
        if self._segments is not None:
            self._launch_streams()
        else:
            N.check(self.lib.yxh_graph_launch(self._graph, N.stream_ptr(self.device)), "graph replay")
        return self.output

    def __del__(self):
        try:
            self._destroy_graphs()
        except Exception:
            pass

    # -------------------------------------------------------------- autotune
    def autotune(self, reps: int = 5, verbose: bool = False) -> dict:
        """Pick each conv's tile (TN x TM, K slabs) by timing every variant on the
        device with HIP events, on this plan's own buffers (after one real forward so
        they hold realistic values).  Results are cached per layer shape for the
        process.  In-place residual layers accumulate during tuning; the next forward
        rewrites every buffer in order, so outputs are unaffected."""
        self.pack_weights()
        self._bind_input(self.static_input())
        L, st = self.lib, N.stream_ptr(self.device)
        N.check(L.yxh_run_ops(self._ops, self._nops, st), "forward")
        stream = torch.cuda.current_stream(self.device)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        chosen = {}
        # YOLOX_AMD_TUNE_COLD=1: time each candidate after streaming 64 MiB through the L2s
        flush = (torch.zeros(16 << 20, dtype=torch.float32, device=self.device)
                 if os.environ.get("YOLOX_AMD_TUNE_COLD", "0") == "1" else None)
        for i, rec in enumerate(self.ctx.ops):
            if rec.kind != N.OP_CONV or rec.args["groups"] != 1:
                continue
            op = self._ops[i]
            key = _tune_key(op.u.conv)
            if key in _TUNE_CACHE:
                op.u.conv.tile = _TUNE_CACHE[key]
                chosen[i] = _TUNE_CACHE[key]
                continue
            best, times = (float("inf"), 0), []
            ptr = C.pointer(op)
            cands = (TILE_CANDIDATES if self.dtype == torch.float32 or _TUNE_ALL_FAMILIES else TILE_CANDIDATES_16)
            for tile in cands:
                op.u.conv.tile = tile
                if L.yxh_run_ops(ptr, 1, st) != N.OK:  # variant not applicable
                    continue
                if flush is None:
                    ev0.record(stream)
                    for _ in range(reps):
                        L.yxh_run_ops(ptr, 1, st)
                    ev1.record(stream)
                    ev1.synchronize()
                    t = ev0.elapsed_time(ev1) / reps
                else:  # each rep after evicting the XCD L2s, as in the forward (weights come from HBM / MALL)
                    t = 0.0
                    for _ in range(reps):
                        flush.add_(1)
                        ev0.record(stream)
                        L.yxh_run_ops(ptr, 1, st)
                        ev1.record(stream)
                        ev1.synchronize()
                        t += ev0.elapsed_time(ev1) / reps
                if _TUNE_ALL:
                    print(f"  op {i} tile {tile >> 1} slabs {(tile & 1) + 1}: {t * 1e3:.1f} us", file=sys.stderr)
                times.append((t, tile))
                if t < best[0]:
                    best = (t, tile)
            op.u.conv.tile = best[1]
            _TUNE_CACHE[key] = best[1]
            _TUNE_TIMES[key] = sorted(times)
            chosen[i] = best[1]
            if verbose:
                a = rec.args
                print(f"tune op {i}: k{a['k']}s{a['stride']} {a['cin']}->{a['cout']} @{a['out_h']}x{a['out_w']}"
                      f" -> tile {best[1] >> 1} slabs {(best[1] & 1) + 1} {best[0] * 1e3:.1f} us", file=sys.stderr)
        for c in range(1, self.nchunks):
            for i, t in chosen.items():
                self._ops[c * self._nops + i].u.conv.tile = t
        torch.cuda.synchronize(self.device)
        if self._graph is not None or self._segments is not None:  # captured graphs hold the old tiles
            self.capture(2 if self._graph_alt is not None else 1)
        return chosen

    def refine_in_graph(self, margin: float = 0.15, alts: int = 2, reps: int = 50, trials: int = 3,
                        min_gain: float = 0.002, verbose: bool = False) -> dict:
        """Second tuning pass, inside the captured forward.  autotune() times each conv alone,
        five times back to back on warm caches; in the forward a launch meets the L2 state its
        producer left and, on the head lanes, shares the CUs with another level.  For every conv
        shape (in forward order) whose runner-up tiles timed within ``margin`` of the best alone,
        the whole forward is replayed with the chosen tile and with each of up to ``alts``
        runner-ups, ``trials`` alternating A/B rounds of ``reps`` replays each, and a runner-up
        replaces the choice only if the median forward drops by more than ``min_gain``
        (a fraction).  Changes go into the per-shape cache like autotune's (save_tune_cache
        writes them).  Returns {shape key: (old tile, new tile, old ms, new ms)}."""
        sites = {}  # shape key -> indices of the first chunk's ops with that shape
        for i, rec in enumerate(self.ctx.ops):
            if rec.kind == N.OP_CONV and rec.args["groups"] == 1:
                key = _tune_key(self._ops[i].u.conv)
                if key in _TUNE_TIMES:
                    sites.setdefault(key, []).append(i)
        had_graph = self._graph is not None or self._segments is not None
        stream = torch.cuda.current_stream(self.device)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def set_tile(key, tile):
            for c in range(self.nchunks):
                for i in sites[key]:
                    self._ops[c * self._nops + i].u.conv.tile = tile

        def forward_ms(key, tile):
            set_tile(key, tile)
            self.capture(1)
            for _ in range(3):
                self.replay()
            ev0.record(stream)
            for _ in range(reps):
                self.replay()
            ev1.record(stream)
            ev1.synchronize()
            return ev0.elapsed_time(ev1) / reps

        changed = {}
        for key, idx in sites.items():
            cur = self._ops[idx[0]].u.conv.tile
            times = _TUNE_TIMES[key]
            t_cur = next((t for t, tile in times if tile == cur), times[0][0])
            cands = [tile for t, tile in times if tile != cur and t <= t_cur * (1 + margin)][:alts]
            for alt in cands:
                ta, tb = [], []
                for _ in range(trials):
                    ta.append(forward_ms(key, cur))
                    tb.append(forward_ms(key, alt))
                ma, mb = statistics.median(ta), statistics.median(tb)
                if verbose:
                    a = self.ctx.ops[idx[0]].args
                    print(f"refine k{a['k']}s{a['stride']} {a['cin']}->{a['cout']} @{a['out_h']}x{a['out_w']}: tile "
                          f"{cur >> 1}/{(cur & 1) + 1} {ma * 1e3:.1f} us vs {alt >> 1}/{(alt & 1) + 1} {mb * 1e3:.1f} us",
                          file=sys.stderr)
                if mb < ma * (1 - min_gain):
                    changed[key] = (changed.get(key, (cur,))[0], alt, ma, mb)
                    cur = alt
            set_tile(key, cur)
            _TUNE_CACHE[key] = cur
        self._destroy_graphs()
        torch.cuda.synchronize(self.device)
        if had_graph:
            self.capture(1)
        return changed

    # -------------------------------------------------------------- reporting
    def conv_ops(self):
        """(index, ConvDesc) of every conv op of the first chunk, for per-kernel accounting."""
        return [(i, self._ops[i].u.conv) for i, r in enumerate(self.ctx.ops) if r.kind == N.OP_CONV]
