"""YOLOX module tree: CSPDarknet backbone, PAFPN neck, decoupled head.

The attribute names and parameter shapes follow the reference exactly
(network_blocks.py, darknet.py:95-177, yolo_pafpn.py:12-116, yolo_head.py:16-138)
so MegVii ``.pth`` checkpoints and reference state_dicts load unchanged (462 keys
for yolox_s; tests/test_api.py checks every preset).  The modules here only own
parameters and topology: execution is planned onto libyoloxhip ops by
``plan(...)`` methods (engine.py) -- there is no eager PyTorch forward.
"""
from __future__ import annotations

import math
from typing import Sequence

import torch
import torch.nn as nn


def _act_module(name: str) -> nn.Module:
    # network_blocks.py:15-24
    if name == "silu":
        return nn.SiLU(inplace=True)
    if name == "relu":
        return nn.ReLU(inplace=True)
    if name == "lrelu":
        return nn.LeakyReLU(0.1, inplace=True)
    raise AttributeError(f"Unsupported act type: {name}")


class _Planned(nn.Module):
    """Modules of this tree run as parts of a planned YoloxModule forward; standalone, a block's
    forward (the reference's eager call, e.g. ``module.backbone.backbone.dark3(x)``) runs a
    one-block HIP plan of it (``plan_block``, eval mode: BatchNorm's running statistics folded),
    cached per input shape -- or, in train mode (a freshly built block is), the model train
    step's kernels: BatchNorm batch statistics, running-statistics update, and autograd through
    the HIP reverse pass (train.block_train_forward)."""

    takes_image = False  # plan_block's input: the [B, 3, H, W] image (Focus / CspDarknet) or a map

    def plan_block(self, ctx, x):  # pragma: no cover - every planned block overrides it
        raise NotImplementedError(f"{type(self).__name__} has no standalone plan")

    def forward(self, x):
        outs = _block_forward(self, x)
        return outs[0]

    def _apply(self, fn, *args, **kwargs):
        self.__dict__.pop("_stage_plans", None)
        return super()._apply(fn, *args, **kwargs)


def _block_forward(block: nn.Module, x: torch.Tensor) -> list:
    """Standalone forward of one building block (network_blocks.py / darknet.py modules) through
    a block plan: NCHW in, NCHW out in the parameters' dtype."""
    from .. import _native as N
    from ..engine import Plan
    if not isinstance(x, torch.Tensor) or x.dim() != 4:
        raise ValueError(f"{type(block).__name__} takes one [B, C, H, W] tensor")
    p = _param0(block)
    if p.device.type != "cuda":
        raise RuntimeError(f"{type(block).__name__} runs on a ROCm device only; call .to('cuda') first")
    if block.training:
        from ..train import block_train_forward
        if block.takes_image and x.shape[1] != 3:
            raise ValueError(f"expected [B, 3, H, W] images, got {tuple(x.shape)}")
        return block_train_forward(block, x)
    B, C, H, W = x.shape
    if block.takes_image:
        if C != 3:
            raise ValueError(f"expected [B, 3, H, W] images, got {tuple(x.shape)}")
        if x.dtype not in (torch.float32, torch.bfloat16, torch.float16, torch.uint8):
            x = x.float()
    else:
        x = x.to(p.dtype)
    key = ("block", B, C, H, W, x.dtype, p.dtype, str(p.device), tuple(getattr(block, "out_features", ())))
    plan = _stage_plan(block, key, lambda: Plan(_StageModel(block), B, H, W, p.dtype, p.device, N.NCHW, x.dtype,
                                                stage="block", block=block, head_inputs=[(C, H, W)]))
    return plan.run_block(x)


class _StageModel:
    """What engine.Plan needs of a model (backbone / head / parameters) for a plan of one
    submodule: YoloPafpn.forward ("features") and YoloxHead.forward ("head")."""

    def __init__(self, owner: nn.Module, backbone=None, head=None):
        self.owner, self.backbone, self.head = owner, backbone, head

    def parameters(self):
        return self.owner.parameters()

    def buffers(self):
        return self.owner.buffers()


def _stage_plan(owner: nn.Module, key: tuple, make):
    cache = owner.__dict__.setdefault("_stage_plans", {})
    if key not in cache:
        cache[key] = make()
    return cache[key]


def _param0(m: nn.Module) -> torch.Tensor:
    return next(m.parameters())


class BaseConv(_Planned):
    """Conv2d(bias=False, same padding) -> BatchNorm2d -> activation."""

    def __init__(self, in_channels, out_channels, ksize, stride, groups=1, bias=False, act="silu"):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, ksize, stride, (ksize - 1) // 2, groups=groups, bias=bias)
        self.bn = nn.BatchNorm2d(out_channels)
        self.act = _act_module(act)
        self.act_name = act

    def plan(self, ctx, srcs, out=None, residual=None):
        return ctx.conv(self, srcs, out=out, residual=residual)

    def plan_block(self, ctx, x):
        return self.plan(ctx, [x])


class DWConv(_Planned):
    """Depthwise BaseConv (groups = cin) followed by a pointwise BaseConv."""

    def __init__(self, in_channels, out_channels, ksize, stride=1, act="silu"):
        super().__init__()
        self.dconv = BaseConv(in_channels, in_channels, ksize, stride, groups=in_channels, act=act)
        self.pconv = BaseConv(in_channels, out_channels, 1, 1, groups=1, act=act)

    def plan(self, ctx, srcs, out=None, residual=None):
        t = ctx.conv(self.dconv, srcs)
        return ctx.conv(self.pconv, [t], out=out, residual=residual)

    def plan_block(self, ctx, x):
        return self.plan(ctx, [x])


def _conv_cls(depthwise: bool):
    return DWConv if depthwise else BaseConv


class Bottleneck(_Planned):
    def __init__(self, in_channels, out_channels, shortcut=True, expansion=0.5, depthwise=False, act="silu"):
        super().__init__()
        hidden = int(out_channels * expansion)
        self.conv1 = BaseConv(in_channels, hidden, 1, stride=1, act=act)
        self.conv2 = _conv_cls(depthwise)(hidden, out_channels, 3, stride=1, act=act)
        self.use_add = shortcut and in_channels == out_channels

    def plan(self, ctx, x, out):
        """y = conv2(conv1(x)) (+ x); ``out`` may alias ``x`` (in-place residual)."""
        t = self.conv1.plan(ctx, [x])
        return self.conv2.plan(ctx, [t], out=out, residual=x if self.use_add else None)

    def plan_block(self, ctx, x):
        out = ctx.buffer(x.lh, x.lw, _out_channels(self.conv2)).full()
        return self.plan(ctx, x, out)


class SPPBottleneck(_Planned):
    def __init__(self, in_channels, out_channels, kernel_sizes=(5, 9, 13), activation="silu"):
        super().__init__()
        hidden = in_channels // 2
        self.conv1 = BaseConv(in_channels, hidden, 1, stride=1, act=activation)
        self.m = nn.ModuleList([nn.MaxPool2d(kernel_size=k, stride=1, padding=k // 2) for k in kernel_sizes])
        self.conv2 = BaseConv(hidden * (len(kernel_sizes) + 1), out_channels, 1, stride=1, act=activation)
        if tuple(kernel_sizes) != (5, 9, 13):
            raise NotImplementedError("the SPP kernel implements kernel_sizes (5, 9, 13)")

    def plan(self, ctx, srcs, out=None):
        hidden = self.conv1.conv.out_channels
        src = srcs[0]
        cat = ctx.buffer(src.lh, src.lw, 4 * hidden)
        self.conv1.plan(ctx, srcs, out=cat.slice(0, hidden))
        ctx.spp(cat, hidden)
        return self.conv2.plan(ctx, [cat.full()], out=out)

    def plan_block(self, ctx, x):
        return self.plan(ctx, [x])


class CspLayer(_Planned):
    """CSP bottleneck with 3 convs; the concat buffer [x_1 | x_2] is written in place."""

    def __init__(self, in_channels, out_channels, n=1, shortcut=True, expansion=0.5, depthwise=False,
                 act="silu"):
        super().__init__()
        hidden = int(out_channels * expansion)
        self.conv1 = BaseConv(in_channels, hidden, 1, stride=1, act=act)
        self.conv2 = BaseConv(in_channels, hidden, 1, stride=1, act=act)
        self.conv3 = BaseConv(2 * hidden, out_channels, 1, stride=1, act=act)
        self.m = nn.Sequential(*[Bottleneck(hidden, hidden, shortcut, 1.0, depthwise, act=act) for _ in range(n)])

    def plan_block(self, ctx, x):
        return self.plan(ctx, [x])

    def plan(self, ctx, srcs, out=None, fused_head=None):
        """``fused_head``: (the [x_1 | x_2] buffer, the first Bottleneck's hidden map) already
        written by the launch that produced this layer's input (stem_s2's CSP form)."""
        hidden = self.conv1.conv.out_channels
        if fused_head is not None:
            cat, t0 = fused_head
            x1 = cat.slice(0, hidden)
            rest = list(self.m)
            return self._plan_tail(ctx, rest, x1, cat, out, t=t0)  # t0: the first conv1 already ran
        cat = ctx.buffer(srcs[0].lh, srcs[0].lw, 2 * hidden)
        x1 = cat.slice(0, hidden)
        # conv1 | conv2 read the same input: one conv writes the whole [x_1 | x_2]
        ctx.conv_multi([self.conv1, self.conv2], srcs, out=cat.full())
        if self.m and all(ctx.bottleneck_fusable(b) for b in self.m):
            # fused Bottlenecks cannot run in place: ping-pong between x_1 and a side buffer;
            # conv3 then reads [last | x_2] as two sources
            side = ctx.buffer(srcs[0].lh, srcs[0].lw, hidden).full()
            cur = x1
            for b in self.m:
                nxt = side if cur is x1 else x1
                ctx.bottleneck(b, cur, nxt)
                cur = nxt
            if cur is not x1:
                return self.conv3.plan(ctx, [cur, cat.slice(hidden, hidden)], out=out)
            return self.conv3.plan(ctx, [cat.full()], out=out)
        return self._plan_tail(ctx, list(self.m), x1, cat, out)

    def _post_fusable(self, ctx, b) -> bool:
        hidden = self.conv1.conv.out_channels
        return hasattr(ctx, "post_fusable") and ctx.post_fusable(b.conv2, [self.conv3], hidden)

    def _plan_post(self, ctx, b, t, x1, cat, out):
        """The last Bottleneck's 3x3 (+ shortcut) and conv3 over [its output | x_2] as one launch."""
        hidden = self.conv1.conv.out_channels
        if out is None:
            out = ctx.buffer(x1.lh, x1.lw, self.conv3.conv.out_channels).full()
        return ctx.conv_post(b.conv2, [t], [self.conv3], cat.slice(hidden, hidden), out,
                             residual=x1 if b.use_add else None)

    def _plan_tail(self, ctx, bottlenecks, x1, cat, out, t=None):
        """The Bottlenecks in place on x_1, then conv3.  ``t``: the first Bottleneck's conv1 output
        when an earlier launch computed it.  Fused where the tiles exist: Bottleneck i's 3x3 +
        shortcut with Bottleneck i+1's conv1 as its post conv (the chain: its output stored too),
        and the last one's 3x3 with conv3 over [y | x_2] (the output never stored)."""
        hidden = self.conv1.conv.out_channels
        for i, b in enumerate(bottlenecks):
            last = i == len(bottlenecks) - 1
            if t is None and not (last and self._post_fusable(ctx, b)) and not self._chain_fusable(ctx, bottlenecks, i):
                b.plan(ctx, x1, out=x1)
                continue
            if t is None:
                t = b.conv1.plan(ctx, [x1])
            if last and self._post_fusable(ctx, b):
                return self._plan_post(ctx, b, t, x1, cat, out)
            res = x1 if b.use_add else None
            if self._chain_fusable(ctx, bottlenecks, i):
                t_next = ctx.buffer(x1.lh, x1.lw, hidden).full()
                ctx.conv_post(b.conv2, [t], [bottlenecks[i + 1].conv1], None, t_next, residual=res, out=x1)
                t = t_next
            else:
                b.conv2.plan(ctx, [t], out=x1, residual=res)
                t = None
        return self.conv3.plan(ctx, [cat.full()], out=out)

    @staticmethod
    def _chain_fusable(ctx, bottlenecks, i) -> bool:
        return (i + 1 < len(bottlenecks) and hasattr(ctx, "post_fusable")
                and ctx.post_fusable(bottlenecks[i].conv2, [bottlenecks[i + 1].conv1], 0))


class Focus(_Planned):
    """Space-to-depth (TL, BL, TR, BR) + BaseConv; the slicing is yxh_focus_pack."""

    def __init__(self, in_channels, out_channels, ksize=1, stride=1, act="silu"):
        super().__init__()
        self.conv = BaseConv(in_channels * 4, out_channels, ksize, stride, act=act)

    takes_image = True

    def plan_block(self, ctx, image):
        return self.plan(ctx, image)

    def plan(self, ctx, image):
        """Fused into one 6x6 s2 conv on the image (yxh_stem_conv) when the geometry
        allows; otherwise yxh_focus_pack + the 3x3 conv on the packed channels."""
        if ctx.stem_fusable(self.conv):
            return ctx.stem(self.conv, image)
        return self.conv.plan(ctx, [ctx.focus(image.h, image.w)])


class CspDarknet(_Planned):
    def __init__(self, dep_mul, wid_mul, out_features=("dark3", "dark4", "dark5"), depthwise=False, act="silu"):
        super().__init__()
        self.out_features = out_features
        Conv = _conv_cls(depthwise)
        bc = int(wid_mul * 64)
        bd = max(round(dep_mul * 3), 1)
        self.stem = Focus(3, bc, ksize=3, act=act)
        self.dark2 = nn.Sequential(Conv(bc, bc * 2, 3, 2, act=act),
                                   CspLayer(bc * 2, bc * 2, n=bd, depthwise=depthwise, act=act))
        self.dark3 = nn.Sequential(Conv(bc * 2, bc * 4, 3, 2, act=act),
                                   CspLayer(bc * 4, bc * 4, n=bd * 3, depthwise=depthwise, act=act))
        self.dark4 = nn.Sequential(Conv(bc * 4, bc * 8, 3, 2, act=act),
                                   CspLayer(bc * 8, bc * 8, n=bd * 3, depthwise=depthwise, act=act))
        self.dark5 = nn.Sequential(Conv(bc * 8, bc * 16, 3, 2, act=act),
                                   SPPBottleneck(bc * 16, bc * 16, activation=act),
                                   CspLayer(bc * 16, bc * 16, n=bd, shortcut=False, depthwise=depthwise, act=act))

    takes_image = True

    def forward(self, x):
        """darknet.py:165-177 standalone: {"dark3", "dark4", "dark5"} feature maps of [B, 3, H, W]
        images (NCHW, the parameters' dtype) by a backbone-only HIP plan."""
        names = self._names()
        return dict(zip(names, _block_forward(self, x)))

    FEATURES = ("stem", "dark2", "dark3", "dark4", "dark5")

    def _names(self) -> list:
        """The requested maps in the reference's output order (darknet.py:165-177)."""
        if set(self.out_features) - set(self.FEATURES):
            raise AttributeError(f"unknown out_features {self.out_features}")
        return [k for k in self.FEATURES if k in self.out_features]

    def plan_block(self, ctx, image):
        names = self._names()
        if "stem" in names:  # the stem map exists only when Focus + stem run as their own launch
            ctx.fuse_stem_s2 = False
        outs = self.plan_all(ctx, image)
        return [outs[k] for k in names]

    def plan(self, ctx, packed):
        outs = self.plan_all(ctx, packed)
        return outs["dark3"], outs["dark4"], outs["dark5"]

    def plan_all(self, ctx, packed) -> dict:
        """{stem (None when fused into the stride-2 launch), dark2 .. dark5} maps."""
        fused = ctx.stem_s2_fusable(self.stem.conv, self.dark2[0])
        csp2 = self.dark2[1]
        head2 = None
        # Focus stem + dark2[0] as one launch where the geometry allows (yxh_stem_s2), with
        # dark2's CspLayer conv1 | conv2 and first Bottleneck conv1 in the same launch if they fit
        if fused and isinstance(csp2, CspLayer) and ctx.stem_s2_csp_fusable(csp2) and len(self.dark2) == 2:
            head2 = ctx.stem_s2_csp(self.stem.conv, self.dark2[0], csp2, packed)
            x = None
        else:
            x = ctx.stem_s2(self.stem.conv, self.dark2[0], packed) if fused else self.stem.plan(ctx, packed)
        stem = None if fused else x
        feats = []
        for stage in (self.dark2, self.dark3, self.dark4, self.dark5):
            blocks = list(stage)[1:]
            if not (fused and stage is self.dark2):
                csp = blocks[0] if blocks and isinstance(blocks[0], CspLayer) else None
                if (csp is not None and hasattr(ctx, "post_fusable")
                        and ctx.post_fusable(stage[0], [csp.conv1, csp.conv2], 0)):
                    # the stride-2 conv + the CspLayer's conv1 | conv2 as one launch (conv_ws post tile)
                    h = csp.conv1.conv.out_channels
                    oh, ow = (x.lh - 1) // 2 + 1, (x.lw - 1) // 2 + 1
                    cat = ctx.buffer(oh, ow, 2 * h)
                    ctx.conv_post(stage[0], [x], [csp.conv1, csp.conv2], None, cat.full())
                    x = csp.plan(ctx, None, fused_head=(cat, None))
                    blocks = blocks[1:]
                else:
                    x = stage[0].plan(ctx, [x])
            for blk in blocks:
                if head2 is not None and blk is csp2:
                    x = blk.plan(ctx, None, fused_head=head2)
                else:
                    x = blk.plan(ctx, [x])
            feats.append(x)
        return {"stem": stem, "dark2": feats[0], "dark3": feats[1], "dark4": feats[2], "dark5": feats[3]}


class YoloPafpn(_Planned):
    def __init__(self, depth=1.0, width=1.0, in_features=("dark3", "dark4", "dark5"),
                 in_channels: Sequence[int] = (256, 512, 1024), depthwise=False, act="silu"):
        super().__init__()
        self.backbone = CspDarknet(depth, width, depthwise=depthwise, act=act)
        self.in_features = in_features
        self.in_channels = in_channels
        Conv = _conv_cls(depthwise)
        c0, c1, c2 = (int(c * width) for c in in_channels)
        n = round(3 * depth)
        self.upsample = nn.Upsample(scale_factor=2, mode="nearest")
        self.lateral_conv0 = BaseConv(c2, c1, 1, 1, act=act)
        self.C3_p4 = CspLayer(2 * c1, c1, n, False, depthwise=depthwise, act=act)
        self.reduce_conv1 = BaseConv(c1, c0, 1, 1, act=act)
        self.C3_p3 = CspLayer(2 * c0, c0, n, False, depthwise=depthwise, act=act)
        self.bu_conv2 = Conv(c0, c0, 3, 2, act=act)
        self.C3_n3 = CspLayer(2 * c0, c1, n, False, depthwise=depthwise, act=act)
        self.bu_conv1 = Conv(c1, c1, 3, 2, act=act)
        self.C3_n4 = CspLayer(2 * c1, c2, n, False, depthwise=depthwise, act=act)

    def forward(self, input):
        """yolo_pafpn.py:83-116 standalone: [B, 3, H, W] images -> (pan_out2, pan_out1,
        pan_out0) NCHW in the parameters' dtype, computed by a features-only HIP plan."""
        from .. import _native as N
        from ..engine import Plan
        x = input
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected [B, 3, H, W] images, got {tuple(x.shape)}")
        p = _param0(self)
        if p.device.type != "cuda":
            raise RuntimeError("YoloPafpn runs on a ROCm device only; call .to('cuda') first")
        if x.dtype not in (torch.float32, torch.bfloat16, torch.float16, torch.uint8):
            x = x.float()
        B, _, H, W = x.shape
        key = ("features", B, H, W, x.dtype, p.dtype, str(p.device))
        plan = _stage_plan(self, key, lambda: Plan(_StageModel(self, backbone=self), B, H, W, p.dtype, p.device,
                                                   N.NCHW, x.dtype, stage="features"))
        return plan.run_features(x)

    def _apply(self, fn, *args, **kwargs):
        self.__dict__.pop("_stage_plans", None)
        return super()._apply(fn, *args, **kwargs)

    def plan(self, ctx, packed):
        """yolo_pafpn.py:83-116.  Every torch.cat is a pre-sliced buffer and every
        upsample a strided read: fpn_out0 / fpn_out1 are written straight into the
        right half of the bottom-up concat buffers they later join."""
        x2, x1, x0 = self.backbone.plan(ctx, packed)
        lat0 = self.lateral_conv0.conv.out_channels
        red1 = self.reduce_conv1.conv.out_channels
        bu1 = _out_channels(self.bu_conv1)
        bu2 = _out_channels(self.bu_conv2)
        p0 = ctx.buffer(x0.lh, x0.lw, bu1 + lat0)
        fpn_out0 = self.lateral_conv0.plan(ctx, [x0], out=p0.slice(bu1, lat0))
        f_out0 = self.C3_p4.plan(ctx, [fpn_out0.upsampled(), x1])
        p1 = ctx.buffer(x1.lh, x1.lw, bu2 + red1)
        fpn_out1 = self.reduce_conv1.plan(ctx, [f_out0], out=p1.slice(bu2, red1))
        pan_out2 = self.C3_p3.plan(ctx, [fpn_out1.upsampled(), x2])
        self.bu_conv2.plan(ctx, [pan_out2], out=p1.slice(0, bu2))
        pan_out1 = self.C3_n3.plan(ctx, [p1.full()])
        self.bu_conv1.plan(ctx, [pan_out1], out=p0.slice(0, bu1))
        pan_out0 = self.C3_n4.plan(ctx, [p0.full()])
        return pan_out2, pan_out1, pan_out0


def _out_channels(m: nn.Module) -> int:
    return m.pconv.conv.out_channels if isinstance(m, DWConv) else m.conv.out_channels


class YoloxHead(_Planned):
    def __init__(self, num_classes, width=1.0, strides=(8, 16, 32), in_channels=(256, 512, 1024), act="silu",
                 depthwise=False):
        super().__init__()
        self.num_classes = num_classes
        self.decode_in_inference = True
        Conv = _conv_cls(depthwise)
        hw_ = int(256 * width)
        self.stems = nn.ModuleList()
        self.cls_convs = nn.ModuleList()
        self.reg_convs = nn.ModuleList()
        self.cls_preds = nn.ModuleList()
        self.reg_preds = nn.ModuleList()
        self.obj_preds = nn.ModuleList()
        for c in in_channels:
            self.stems.append(BaseConv(int(c * width), hw_, 1, 1, act=act))
            self.cls_convs.append(nn.Sequential(Conv(hw_, hw_, 3, 1, act=act), Conv(hw_, hw_, 3, 1, act=act)))
            self.reg_convs.append(nn.Sequential(Conv(hw_, hw_, 3, 1, act=act), Conv(hw_, hw_, 3, 1, act=act)))
            self.cls_preds.append(nn.Conv2d(hw_, num_classes, 1, 1, 0))
            self.reg_preds.append(nn.Conv2d(hw_, 4, 1, 1, 0))
            self.obj_preds.append(nn.Conv2d(hw_, 1, 1, 1, 0))
        self.use_l1 = False
        self.strides = list(strides)

    def forward(self, xin, labels=None, imgs=None):
        """yolo_head.py:140-211 standalone, eval mode: three NCHW feature maps -> decoded
        [B, A, 5+C] rows (in xin[0]'s dtype, as decode_outputs returns them), by a head-only
        HIP plan.  The training form (losses) runs inside YoloxModule.forward."""
        from .. import _native as N
        from ..engine import Plan
        if self.training:
            raise NotImplementedError("YoloxHead.forward in training mode: call YoloxModule.forward(x, targets)")
        if len(xin) != 3:
            raise ValueError("YoloxHead takes three feature maps")
        p = _param0(self)
        if p.device.type != "cuda":
            raise RuntimeError("YoloxHead runs on a ROCm device only; call .to('cuda') first")
        B = xin[0].shape[0]
        shapes = [tuple(int(v) for v in t.shape[1:]) for t in xin]
        key = ("head", B, tuple(shapes), p.dtype, str(p.device), bool(self.decode_in_inference))
        owner = self
        plan = _stage_plan(self, key, lambda: Plan(_StageModel(owner, head=owner), B, 32, 32, p.dtype, p.device,
                                                   stage="head", head_inputs=shapes))
        out = torch.empty(B, plan.anchors, 5 + self.num_classes, dtype=torch.float32, device=p.device)
        plan.run_head(xin, out)
        return out.to(xin[0].dtype)

    def _apply(self, fn, *args, **kwargs):
        self.__dict__.pop("_stage_plans", None)
        return super()._apply(fn, *args, **kwargs)

    def initialize_biases(self, prior_prob: float) -> None:
        """yolo_head.py:129-138: cls/obj pred biases = -log((1 - p) / p)."""
        v = -math.log((1 - prior_prob) / prior_prob)
        with torch.no_grad():
            for conv in list(self.cls_preds) + list(self.obj_preds):
                conv.bias.fill_(v)

    def plan(self, ctx, feats, out, train: bool = False):
        """Per level: stem, 2x cls conv, 2x reg conv, then the 1x1 preds write decoded
        rows straight into ``out`` [B, A, 5+C] (yolo_head.py:140-251); eval with
        ``decode_in_inference = False``: the same rows without the box decode (:208-211)."""
        if not train and not self.decode_in_inference:
            train = 2  # PlanCtx.HEAD_RAW
        a_off = 0
        for k, x in enumerate(feats):
            n0 = len(ctx.ops)
            s = self.stems[k].plan(ctx, [x])
            c0, r0 = self.cls_convs[k][0], self.reg_convs[k][0]
            if isinstance(c0, BaseConv) and isinstance(r0, BaseConv):
                # both branch heads read the stem output: one conv writes [cls | reg]
                hw_ = c0.conv.out_channels
                cr = ctx.conv_multi([c0, r0], [s])
                c, r = cr.buf.slice(0, hw_), cr.buf.slice(hw_, hw_)
            else:
                c, r = c0.plan(ctx, [s]), r0.plan(ctx, [s])
            c1, r1 = self.cls_convs[k][1], self.reg_convs[k][1]
            two = (c.buf is r.buf and c.coff == 0 and r.coff == c.ch and c.buf.c == 2 * c.ch
                   and ctx.grouped2_fusable(c1, r1, c.buf.full()))
            if two and hasattr(ctx, "grouped2_head_fusable") and ctx.grouped2_head_fusable(self, c.buf.full(), train, k):
                # ... with the level's preds + decode riding in the same launch
                ctx.conv_grouped2_head([c1, r1], c.buf.full(), self, k, out, a_off, self.strides[k])
                for rec in ctx.ops[n0:]:
                    rec.lane = 1 + k
                a_off += x.lh * x.lw
                continue
            if two:
                # cls_convs[k][1] | reg_convs[k][1] over [cls | reg]: one two-group launch
                cr2 = ctx.conv_grouped2([c1, r1], c.buf.full())
                half = c1.conv.out_channels
                c, r = cr2.buf.slice(0, half), cr2.buf.slice(half, half)
            else:
                c = c1.plan(ctx, [c])
                r = r1.plan(ctx, [r])
            ctx.head_preds(k, self, c, r, out, a_off, self.strides[k], train)
            for rec in ctx.ops[n0:]:  # levels are independent: one graph branch each
                rec.lane = 1 + k
            a_off += x.lh * x.lw
        return out
