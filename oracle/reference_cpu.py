"""ORACLE -- test infrastructure only.

CPU restatement of the reference's hot path, used as the checker by tests/,
``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg.  The product
(``yolox_amd``) never imports this module and never falls back to it.

Floating-point parts are restated functionally in PyTorch-CPU fp32 (the reference
itself is PyTorch); the integer/index-heavy post-processing (filter + torchvision
NMS) is restated in plain C (``postprocess_oracle.c``), loaded through ctypes.

Pinned against the reference: ``tests/golden/*.npz`` were produced by importing
the reference model files in the build container (``tests/golden/make_golden.py``)
and ``tests/test_oracle.py`` checks every function here against them.  NMS itself is
pinned only by hand-made known-answer vectors (torchvision is absent).

Citations are to /root/reference (pixeltable-yolox 0.4.1).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Mapping, Optional

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

Tensor = torch.Tensor
SD = Mapping[str, Tensor]


# ----------------------------------------------------------------- architecture
@dataclass(frozen=True)
class Arch:
    """Preset multipliers, reference config.py:412-469."""
    depth: float
    width: float
    depthwise: bool = False
    act: str = "silu"
    num_classes: int = 80
    bn_eps: float = 1e-3  # config.get_model init_yolo, config.py:162-166

    @property
    def base_ch(self) -> int:
        return int(self.width * 64)

    @property
    def base_depth(self) -> int:
        return max(round(self.depth * 3), 1)


ARCHS = {
    "yolox_s": Arch(0.33, 0.50),
    "yolox_m": Arch(0.67, 0.75),
    "yolox_l": Arch(1.0, 1.0),
    "yolox_x": Arch(1.33, 1.25),
    "yolox_tiny": Arch(0.33, 0.375),
    "yolox_nano": Arch(0.33, 0.25, depthwise=True),
}


def _act(x: Tensor, act: str) -> Tensor:
    # network_blocks.py:15-24
    if act == "silu":
        return F.silu(x)
    if act == "relu":
        return F.relu(x)
    if act == "lrelu":
        return F.leaky_relu(x, 0.1)
    raise AttributeError(act)


# ------------------------------------------------------------------ storage rounding
# Emulation of a 16-bit inference path's STORAGE precision (not of its summation order), the
# yardstick the bf16/fp16 parity bounds are derived from: inside
# ``stored_as(dtype)`` every BaseConv uses its BN-folded weight rounded to ``dtype`` (fp32 bias),
# sums in fp32, and rounds its output (after the activation and any Bottleneck shortcut) to
# ``dtype``, as the device stores every map; the head preds use rounded weights on the rounded
# features and stay fp32.  In train mode (batch-statistics BN, forward_train) it rounds the
# input image, each conv's weight and output and each block output instead (the --fp16 step).
_STORE: Optional[torch.dtype] = None


class stored_as:
    def __init__(self, dtype: Optional[torch.dtype]):
        self.dtype = dtype

    def __enter__(self):
        global _STORE
        self.prev, _STORE = _STORE, self.dtype
        return self

    def __exit__(self, *exc):
        global _STORE
        _STORE = self.prev


def _rnd(t: Tensor) -> Tensor:
    return t.to(_STORE).float() if _STORE is not None else t


# ------------------------------------------------------------------ blocks
def base_conv(sd: SD, p: str, x: Tensor, k: int, s: int, act: str, eps: float,
              groups: int = 1, bn_train: bool = False, residual: Optional[Tensor] = None) -> Tensor:
    """BaseConv: conv(bias=False, pad=(k-1)//2) -> BN -> act (network_blocks.py:27-52), then
    the Bottleneck shortcut when given (network_blocks.py:97-99)."""
    if _STORE is not None and not bn_train:
        w, b = fuse_conv_bn(sd[p + ".conv.weight"], sd[p + ".bn.weight"], sd[p + ".bn.bias"],
                            sd[p + ".bn.running_mean"], sd[p + ".bn.running_var"], eps)
        y = _act(F.conv2d(x, _rnd(w), b, s, (k - 1) // 2, 1, groups), act)
        return _rnd(y + residual if residual is not None else y)
    # train mode under stored_as (the --fp16 step): 16-bit conv operands with an fp32 sum, the
    # conv output and the block output stored in 16 bits, BN batch statistics in fp32; autograd
    # then differentiates through the roundings as identities (the backward itself stays fp32)
    y = F.conv2d(x, _rnd(sd[p + ".conv.weight"]), None, s, (k - 1) // 2, 1, groups)
    y = F.batch_norm(_rnd(y), sd[p + ".bn.running_mean"], sd[p + ".bn.running_var"],
                     sd[p + ".bn.weight"], sd[p + ".bn.bias"], bn_train, 0.03, eps)
    y = _act(y, act)
    return _rnd(y + residual if residual is not None else y)


def conv(sd: SD, p: str, x: Tensor, k: int, s: int, arch: Arch, bn_train: bool,
         depthwise: Optional[bool] = None, residual: Optional[Tensor] = None) -> Tensor:
    """BaseConv or DWConv (network_blocks.py:55-74) depending on the preset."""
    dw = arch.depthwise if depthwise is None else depthwise
    if dw:
        c = x.shape[1]
        x = base_conv(sd, p + ".dconv", x, k, s, arch.act, arch.bn_eps, groups=c, bn_train=bn_train)
        return base_conv(sd, p + ".pconv", x, 1, 1, arch.act, arch.bn_eps, bn_train=bn_train, residual=residual)
    return base_conv(sd, p, x, k, s, arch.act, arch.bn_eps, bn_train=bn_train, residual=residual)


def bottleneck(sd: SD, p: str, x: Tensor, shortcut: bool, arch: Arch, bn_train: bool) -> Tensor:
    """network_blocks.py:77-99 (expansion 1.0 inside CSP)."""
    y = base_conv(sd, p + ".conv1", x, 1, 1, arch.act, arch.bn_eps, bn_train=bn_train)
    add = shortcut and x.shape[1] == sd[p + ".conv2" + (".pconv" if arch.depthwise else "") + ".conv.weight"].shape[0]
    return conv(sd, p + ".conv2", y, 3, 1, arch, bn_train, residual=x if add else None)


def csp(sd: SD, p: str, x: Tensor, n: int, shortcut: bool, arch: Arch, bn_train: bool) -> Tensor:
    """CspLayer, network_blocks.py:145-183."""
    x1 = base_conv(sd, p + ".conv1", x, 1, 1, arch.act, arch.bn_eps, bn_train=bn_train)
    x2 = base_conv(sd, p + ".conv2", x, 1, 1, arch.act, arch.bn_eps, bn_train=bn_train)
    for i in range(n):
        x1 = bottleneck(sd, f"{p}.m.{i}", x1, shortcut, arch, bn_train)
    return base_conv(sd, p + ".conv3", torch.cat([x1, x2], 1), 1, 1, arch.act, arch.bn_eps,
                     bn_train=bn_train)


def spp(sd: SD, p: str, x: Tensor, arch: Arch, bn_train: bool, ks=(5, 9, 13)) -> Tensor:
    """SPPBottleneck, network_blocks.py:120-142."""
    x = base_conv(sd, p + ".conv1", x, 1, 1, arch.act, arch.bn_eps, bn_train=bn_train)
    x = torch.cat([x] + [F.max_pool2d(x, k, 1, k // 2) for k in ks], 1)
    return base_conv(sd, p + ".conv2", x, 1, 1, arch.act, arch.bn_eps, bn_train=bn_train)


def focus(x: Tensor) -> Tensor:
    """Space-to-depth, channel order TL, BL, TR, BR (network_blocks.py:193-208)."""
    return torch.cat([x[..., ::2, ::2], x[..., 1::2, ::2], x[..., ::2, 1::2], x[..., 1::2, 1::2]], 1)


# ------------------------------------------------------------------ model
def backbone(sd: SD, arch: Arch, x: Tensor, bn_train: bool = False):
    """CspDarknet (darknet.py:95-177) + YoloPafpn (yolo_pafpn.py:83-116)."""
    b = "backbone.backbone"
    bd = arch.base_depth
    x = base_conv(sd, f"{b}.stem.conv", focus(x), 3, 1, arch.act, arch.bn_eps, bn_train=bn_train)
    x = conv(sd, f"{b}.dark2.0", x, 3, 2, arch, bn_train)
    x = csp(sd, f"{b}.dark2.1", x, bd, True, arch, bn_train)
    x = conv(sd, f"{b}.dark3.0", x, 3, 2, arch, bn_train)
    d3 = csp(sd, f"{b}.dark3.1", x, 3 * bd, True, arch, bn_train)
    x = conv(sd, f"{b}.dark4.0", d3, 3, 2, arch, bn_train)
    d4 = csp(sd, f"{b}.dark4.1", x, 3 * bd, True, arch, bn_train)
    x = conv(sd, f"{b}.dark5.0", d4, 3, 2, arch, bn_train)
    x = spp(sd, f"{b}.dark5.1", x, arch, bn_train)
    d5 = csp(sd, f"{b}.dark5.2", x, bd, False, arch, bn_train)

    n = round(3 * arch.depth)
    a = "backbone"
    up = lambda t: F.interpolate(t, scale_factor=2, mode="nearest")  # noqa: E731
    fpn_out0 = base_conv(sd, f"{a}.lateral_conv0", d5, 1, 1, arch.act, arch.bn_eps, bn_train=bn_train)
    f_out0 = csp(sd, f"{a}.C3_p4", torch.cat([up(fpn_out0), d4], 1), n, False, arch, bn_train)
    fpn_out1 = base_conv(sd, f"{a}.reduce_conv1", f_out0, 1, 1, arch.act, arch.bn_eps, bn_train=bn_train)
    pan_out2 = csp(sd, f"{a}.C3_p3", torch.cat([up(fpn_out1), d3], 1), n, False, arch, bn_train)
    p_out1 = conv(sd, f"{a}.bu_conv2", pan_out2, 3, 2, arch, bn_train)
    pan_out1 = csp(sd, f"{a}.C3_n3", torch.cat([p_out1, fpn_out1], 1), n, False, arch, bn_train)
    p_out0 = conv(sd, f"{a}.bu_conv1", pan_out1, 3, 2, arch, bn_train)
    pan_out0 = csp(sd, f"{a}.C3_n4", torch.cat([p_out0, fpn_out0], 1), n, False, arch, bn_train)
    return pan_out2, pan_out1, pan_out0


def head_raw(sd: SD, arch: Arch, feats, bn_train: bool = False):
    """Per level (reg [B,4,H,W], obj [B,1,H,W], cls [B,C,H,W]) logits (yolo_head.py:140-160)."""
    outs = []
    for k, x in enumerate(feats):
        h = "head"
        x = base_conv(sd, f"{h}.stems.{k}", x, 1, 1, arch.act, arch.bn_eps, bn_train=bn_train)
        c = conv(sd, f"{h}.cls_convs.{k}.0", x, 3, 1, arch, bn_train)
        c = conv(sd, f"{h}.cls_convs.{k}.1", c, 3, 1, arch, bn_train)
        r = conv(sd, f"{h}.reg_convs.{k}.0", x, 3, 1, arch, bn_train)
        r = conv(sd, f"{h}.reg_convs.{k}.1", r, 3, 1, arch, bn_train)
        cls = F.conv2d(c, _rnd(sd[f"{h}.cls_preds.{k}.weight"]), sd[f"{h}.cls_preds.{k}.bias"])
        reg = F.conv2d(r, _rnd(sd[f"{h}.reg_preds.{k}.weight"]), sd[f"{h}.reg_preds.{k}.bias"])
        obj = F.conv2d(r, _rnd(sd[f"{h}.obj_preds.{k}.weight"]), sd[f"{h}.obj_preds.{k}.bias"])
        outs.append((reg, obj, cls))
    return outs


def anchors_for(hw_list, strides=(8, 16, 32), dtype=torch.float32):
    """grid (x, y) and stride per anchor, level-major, row-major (yolo_head.py:233-251)."""
    gx, gy, st = [], [], []
    for (h, w), s in zip(hw_list, strides):
        yv, xv = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
        gx.append(xv.reshape(-1))
        gy.append(yv.reshape(-1))
        st.append(torch.full((h * w,), s))
    return (torch.cat(gx).to(dtype), torch.cat(gy).to(dtype), torch.cat(st).to(dtype))


def forward_eval(sd: SD, arch: Arch, x: Tensor) -> Tensor:
    """YoloxModule.forward in eval mode -> decoded [B, A, 5+C] (yolo_head.py:184-251)."""
    with torch.no_grad():
        levels = head_raw(sd, arch, backbone(sd, arch, x))
        rows = []
        hw = []
        for reg, obj, cls in levels:
            o = torch.cat([reg, obj.sigmoid(), cls.sigmoid()], 1)
            hw.append(o.shape[-2:])
            rows.append(o.flatten(2))
        out = torch.cat(rows, 2).permute(0, 2, 1)
        gx, gy, st = anchors_for(hw)
        grid = torch.stack([gx, gy], 1)[None]
        st = st[None, :, None]
        return torch.cat([(out[..., 0:2] + grid) * st, torch.exp(out[..., 2:4]) * st, out[..., 4:]], -1)


# ----------------------------------------------------------------- boxes
def bboxes_iou(a: Tensor, b: Tensor, xyxy: bool = True) -> Tensor:
    """utils/boxes.py:78-101 (same fp32 operation order)."""
    if a.shape[1] != 4 or b.shape[1] != 4:
        raise IndexError
    if xyxy:
        tl = torch.max(a[:, None, :2], b[:, :2])
        br = torch.min(a[:, None, 2:], b[:, 2:])
        area_a = torch.prod(a[:, 2:] - a[:, :2], 1)
        area_b = torch.prod(b[:, 2:] - b[:, :2], 1)
    else:
        tl = torch.max(a[:, None, :2] - a[:, None, 2:] / 2, b[:, :2] - b[:, 2:] / 2)
        br = torch.min(a[:, None, :2] + a[:, None, 2:] / 2, b[:, :2] + b[:, 2:] / 2)
        area_a = torch.prod(a[:, 2:], 1)
        area_b = torch.prod(b[:, 2:], 1)
    en = (tl < br).type(tl.type()).prod(dim=2)
    area_i = torch.prod(br - tl, 2) * en
    return area_i / (area_a[:, None] + area_b - area_i)


def iou_loss(pred: Tensor, target: Tensor) -> Tensor:
    """IouLoss(loss_type='iou', reduction='none'), models/losses.py:13-51."""
    pred = pred.view(-1, 4)
    target = target.view(-1, 4)
    tl = torch.max(pred[:, :2] - pred[:, 2:] / 2, target[:, :2] - target[:, 2:] / 2)
    br = torch.min(pred[:, :2] + pred[:, 2:] / 2, target[:, :2] + target[:, 2:] / 2)
    area_p = torch.prod(pred[:, 2:], 1)
    area_g = torch.prod(target[:, 2:], 1)
    en = (tl < br).type(tl.type()).prod(dim=1)
    area_i = torch.prod(br - tl, 1) * en
    iou = area_i / (area_p + area_g - area_i + 1e-16)
    return 1 - iou ** 2


# ----------------------------------------------------------------- SimOTA
def simota_assign(gt_boxes: Tensor, gt_classes: Tensor, pred_boxes: Tensor, cls_logits: Tensor,
                  obj_logits: Tensor, x_shifts: Tensor, y_shifts: Tensor, strides: Tensor,
                  num_classes: int = 80):
    """get_assignments + get_geometry_constraint + simota_matching for ONE image
    (yolo_head.py:420-574).

    gt_boxes [G,4] cxcywh, gt_classes [G], pred_boxes [A,4], cls_logits [A,C],
    obj_logits [A,1], shifts/strides [A].  Returns (fg_mask [A] bool,
    matched_gt_inds [F], pred_ious [F], gt_matched_classes [F], num_fg).
    """
    G = gt_boxes.shape[0]
    # geometry constraint, :511-540 (centre radius 1.5 strides, strict > 0)
    xc = ((x_shifts + 0.5) * strides)[None]
    yc = ((y_shifts + 0.5) * strides)[None]
    cd = strides[None] * 1.5
    gl = gt_boxes[:, 0:1] - cd
    gr = gt_boxes[:, 0:1] + cd
    gt_ = gt_boxes[:, 1:2] - cd
    gb = gt_boxes[:, 1:2] + cd
    deltas = torch.stack([xc - gl, yc - gt_, gr - xc, gb - yc], 2)
    in_centers = deltas.min(dim=-1).values > 0.0
    anchor_filter = in_centers.sum(dim=0) > 0
    geom = in_centers[:, anchor_filter]

    boxes_in = pred_boxes[anchor_filter]
    cls_in = cls_logits[anchor_filter]
    obj_in = obj_logits[anchor_filter]
    n_in = boxes_in.shape[0]
    ious = bboxes_iou(gt_boxes, boxes_in, False)
    onehot = F.one_hot(gt_classes.to(torch.int64), num_classes).float()
    iou_cost = -torch.log(ious + 1e-8)
    p = (cls_in.float().sigmoid() * obj_in.float().sigmoid()).sqrt()
    cls_cost = F.binary_cross_entropy(p.unsqueeze(0).repeat(G, 1, 1),
                                      onehot.unsqueeze(1).repeat(1, n_in, 1), reduction="none").sum(-1)
    cost = cls_cost + 3.0 * iou_cost + float(1e6) * (~geom)

    # simota_matching, :542-574
    matching = torch.zeros_like(cost, dtype=torch.uint8)
    n_cand = min(10, ious.size(1))
    topk, _ = torch.topk(ious, n_cand, dim=1)
    dyn_k = torch.clamp(topk.sum(1).int(), min=1)
    for g in range(G):
        _, pos = torch.topk(cost[g], k=int(dyn_k[g]), largest=False)
        matching[g][pos] = 1
    per_anchor = matching.sum(0)
    if per_anchor.max() > 1:
        multi = per_anchor > 1
        _, amin = torch.min(cost[:, multi], dim=0)
        matching[:, multi] *= 0
        matching[amin, multi] = 1
    fg_in = per_anchor > 0
    num_fg = int(fg_in.sum().item())
    fg_mask = anchor_filter.clone()
    fg_mask[anchor_filter.clone()] = fg_in
    matched = matching[:, fg_in].argmax(0)
    pred_ious = (matching * ious).sum(0)[fg_in]
    return fg_mask, matched, pred_ious, gt_classes[matched], num_fg


# ----------------------------------------------------------------- training
def train_outputs(sd: SD, arch: Arch, x: Tensor):
    """Train-mode head outputs (yolo_head.py:161-182, get_output_and_grid :213-231):
    (outputs [B, A, 5+C] with decoded boxes and raw logits, origin reg [B, A, 4],
    level sizes [(h, w)])."""
    levels = head_raw(sd, arch, backbone(sd, arch, _rnd(x), bn_train=True), bn_train=True)
    C = arch.num_classes
    outs, origin, hw = [], [], []
    for (reg, obj, cls), s in zip(levels, (8, 16, 32)):
        B, _, h, w = reg.shape
        o = torch.cat([reg, obj, cls], 1).permute(0, 2, 3, 1).reshape(B, h * w, 5 + C)
        gx, gy, _ = anchors_for([(h, w)], (s,))
        grid = torch.stack([gx, gy], 1)[None]
        outs.append(torch.cat([(o[..., :2] + grid) * s, torch.exp(o[..., 2:4]) * s, o[..., 4:]], -1))
        origin.append(reg.permute(0, 2, 3, 1).reshape(B, h * w, 4))
        hw.append((h, w))
    return torch.cat(outs, 1), torch.cat(origin, 1), hw


def forward_train(sd: SD, arch: Arch, x: Tensor, labels: Tensor, use_l1: bool = False):
    """YoloxModule.forward in train mode -> loss dict (yolox.py:76-87, yolo_head.py:161-411).

    BN uses batch statistics.  ``sd`` tensors may require grad; the returned total loss
    is differentiable w.r.t. them (autograd on CPU).
    """
    levels = head_raw(sd, arch, backbone(sd, arch, x, bn_train=True), bn_train=True)
    C = arch.num_classes
    outs, origin, xs_, ys_, ss_ = [], [], [], [], []
    for (reg, obj, cls), s in zip(levels, (8, 16, 32)):
        B, _, h, w = reg.shape
        o = torch.cat([reg, obj, cls], 1).permute(0, 2, 3, 1).reshape(B, h * w, 5 + C)
        gx, gy, _ = anchors_for([(h, w)], (s,))
        grid = torch.stack([gx, gy], 1)[None]
        o = torch.cat([(o[..., :2] + grid) * s, torch.exp(o[..., 2:4]) * s, o[..., 4:]], -1)
        outs.append(o)
        xs_.append(gx)
        ys_.append(gy)
        ss_.append(torch.full((h * w,), float(s)))
        if use_l1:
            origin.append(reg.permute(0, 2, 3, 1).reshape(B, h * w, 4))
    out = torch.cat(outs, 1)
    x_shifts, y_shifts, strides = torch.cat(xs_), torch.cat(ys_), torch.cat(ss_)
    return losses(out, torch.cat(origin, 1) if use_l1 else None, labels, x_shifts, y_shifts, strides, C)


def level_grid(hw, strides=(8, 16, 32)):
    """(x_shifts, y_shifts, strides) [A] for the levels' (h, w) (yolo_head.py:213-231)."""
    xs_, ys_, ss_ = [], [], []
    for (h, w), s in zip(hw, strides):
        gx, gy, _ = anchors_for([(h, w)], (s,))
        xs_.append(gx)
        ys_.append(gy)
        ss_.append(torch.full((h * w,), float(s)))
    return torch.cat(xs_), torch.cat(ys_), torch.cat(ss_)


def losses(out: Tensor, origin, labels: Tensor, x_shifts: Tensor, y_shifts: Tensor, strides: Tensor,
           C: int = 80):
    """YoloxHead.get_losses (yolo_head.py:253-411) from train-mode head outputs ``out``
    [B, A, 5+C] (decoded boxes, raw logits) and, for the L1 term, the raw reg outputs
    ``origin`` [B, A, 4] (None: use_l1 False)."""
    use_l1 = origin is not None
    bbox, obj, cls = out[..., :4], out[..., 4:5], out[..., 5:]
    B, A = out.shape[:2]
    nlabel = (labels.sum(dim=2) > 0).sum(dim=1)
    cls_t, reg_t, l1_t, obj_t, fg_all = [], [], [], [], []
    num_fg, num_gts = 0.0, 0.0
    for b in range(B):
        G = int(nlabel[b])
        num_gts += G
        if G == 0:
            cls_t.append(out.new_zeros((0, C)))
            reg_t.append(out.new_zeros((0, 4)))
            l1_t.append(out.new_zeros((0, 4)))
            obj_t.append(out.new_zeros((A, 1)))
            fg_all.append(out.new_zeros(A).bool())
            continue
        gtb = labels[b, :G, 1:5]
        gtc = labels[b, :G, 0]
        with torch.no_grad():
            fg, matched, piou, gcls, nfg = simota_assign(
                gtb, gtc, bbox[b].detach(), cls[b].detach(), obj[b].detach(),
                x_shifts, y_shifts, strides, C)
        num_fg += nfg
        cls_t.append(F.one_hot(gcls.to(torch.int64), C) * piou.unsqueeze(-1))
        obj_t.append(fg.unsqueeze(-1).to(out.dtype))
        reg_t.append(gtb[matched])
        fg_all.append(fg)
        if use_l1:
            g = gtb[matched]
            st = strides[fg]
            l1 = out.new_zeros((nfg, 4))
            l1[:, 0] = g[:, 0] / st - x_shifts[fg]
            l1[:, 1] = g[:, 1] / st - y_shifts[fg]
            l1[:, 2] = torch.log(g[:, 2] / st + 1e-8)
            l1[:, 3] = torch.log(g[:, 3] / st + 1e-8)
            l1_t.append(l1)
    cls_t, reg_t, obj_t, fg_all = (torch.cat(cls_t), torch.cat(reg_t), torch.cat(obj_t),
                                   torch.cat(fg_all))
    num_fg = max(num_fg, 1)
    loss_iou = iou_loss(bbox.reshape(-1, 4)[fg_all], reg_t).sum() / num_fg
    loss_obj = F.binary_cross_entropy_with_logits(obj.reshape(-1, 1), obj_t, reduction="none").sum() / num_fg
    loss_cls = F.binary_cross_entropy_with_logits(cls.reshape(-1, C)[fg_all], cls_t,
                                                  reduction="none").sum() / num_fg
    if use_l1:
        l1_t = torch.cat(l1_t)
        loss_l1 = F.l1_loss(origin.reshape(-1, 4)[fg_all], l1_t, reduction="none").sum() / num_fg
    else:
        loss_l1 = 0.0
    loss = 5.0 * loss_iou + loss_obj + loss_cls + loss_l1
    return {"total_loss": loss, "iou_loss": 5.0 * loss_iou, "l1_loss": loss_l1,
            "conf_loss": loss_obj, "cls_loss": loss_cls, "num_fg": num_fg / max(num_gts, 1)}


# ----------------------------------------------------------------- postprocess
_lib = None


def _oracle_lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle library missing: build it with `make -C {HERE}`")
        lib = ctypes.CDLL(LIB_PATH)
        i64, f32p, i64p = ctypes.c_int64, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int64)
        lib.oracle_nms.argtypes = [f32p, f32p, i64, ctypes.c_double, i64p]
        lib.oracle_nms.restype = i64
        lib.oracle_batched_nms.argtypes = [f32p, f32p, f32p, i64, ctypes.c_double, i64, i64p]
        lib.oracle_batched_nms.restype = i64
        lib.oracle_postprocess.argtypes = [f32p, i64, i64, i64, ctypes.c_float, ctypes.c_double,
                                           ctypes.c_int, i64, f32p, i64p]
        lib.oracle_postprocess.restype = ctypes.c_int
        lib.oracle_xyxy_inplace.argtypes = [f32p, i64, i64]
        lib.oracle_xyxy_inplace.restype = None
        lib.oracle_filter.argtypes = [f32p, i64, i64, ctypes.c_float, f32p]
        lib.oracle_filter.restype = i64
        _lib = lib
    return _lib


def _fp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _ip(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


VANILLA_NUMEL_CPU = 4000  # torchvision batched_nms CPU branch rule


def nms(boxes: np.ndarray, scores: np.ndarray, thr: float) -> np.ndarray:
    boxes = np.ascontiguousarray(boxes, np.float32)
    scores = np.ascontiguousarray(scores, np.float32)
    keep = np.zeros(max(len(scores), 1), np.int64)
    n = _oracle_lib().oracle_nms(_fp(boxes), _fp(scores), len(scores), float(thr), _ip(keep))
    return keep[:n]


def batched_nms(boxes, scores, idxs, thr, vanilla_numel: int = VANILLA_NUMEL_CPU) -> np.ndarray:
    boxes = np.ascontiguousarray(boxes, np.float32)
    scores = np.ascontiguousarray(scores, np.float32)
    idxs = np.ascontiguousarray(idxs, np.float32)
    keep = np.zeros(max(len(scores), 1), np.int64)
    n = _oracle_lib().oracle_batched_nms(_fp(boxes), _fp(scores), _fp(idxs), len(scores), float(thr),
                                         int(vanilla_numel), _ip(keep))
    return keep[:n]


def xyxy_inplace(prediction: np.ndarray) -> None:
    """boxes.py:32-37 on a float32 [B, A, D] array, in place."""
    assert prediction.dtype == np.float32 and prediction.flags.c_contiguous
    B, A, D = prediction.shape
    _oracle_lib().oracle_xyxy_inplace(_fp(prediction), B * A, D)


def filter_candidates(image_pred_xyxy: np.ndarray, num_classes: int, conf_thre: float) -> np.ndarray:
    """boxes.py:46-51 for one image (rows already xyxy): [N, 7] in anchor order."""
    p = np.ascontiguousarray(image_pred_xyxy, np.float32)
    det = np.zeros((max(p.shape[0], 1), 7), np.float32)
    n = _oracle_lib().oracle_filter(_fp(p), p.shape[0], num_classes, np.float32(conf_thre), _fp(det))
    return det[:n]


def postprocess(prediction: np.ndarray, num_classes: int, conf_thre: float = 0.7,
                nms_thre: float = 0.45, class_agnostic: bool = False,
                vanilla_numel: int = VANILLA_NUMEL_CPU):
    """utils.postprocess restated (boxes.py:31-75).  ``prediction`` (float32 numpy
    [B,A,5+C]) is converted to xyxy IN PLACE, like the reference.  Returns a list of
    [N,7] float32 arrays or None."""
    assert prediction.dtype == np.float32 and prediction.flags.c_contiguous
    B, A, D = prediction.shape
    assert D == 5 + num_classes
    rows = np.zeros((B, max(A, 1), 7), np.float32)
    counts = np.zeros(B, np.int64)
    _oracle_lib().oracle_postprocess(_fp(prediction), B, A, num_classes, np.float32(conf_thre),
                                     float(nms_thre), int(class_agnostic), int(vanilla_numel),
                                     _fp(rows), _ip(counts))
    return [rows[b, :counts[b]].copy() if counts[b] > 0 else None for b in range(B)]


def letterbox_identity(images_u8: np.ndarray) -> np.ndarray:
    """ValTransform/preproc for r == 1 (input already at test_size): HWC uint8 ->
    CHW float32, RGB kept, pad value irrelevant (data_augment.py:140-156)."""
    return np.ascontiguousarray(images_u8.transpose(0, 3, 1, 2), dtype=np.float32)


def fuse_conv_bn(w: Tensor, gamma: Tensor, beta: Tensor, mean: Tensor, var: Tensor, eps: float):
    """BN folding (utils/model_utils.py:33-75): W' = W*g/sqrt(v+eps), b' = beta - g*mu/sqrt(v+eps)."""
    s = gamma / torch.sqrt(var + eps)
    return w * s.view(-1, 1, 1, 1), beta - mean * s


# ----------------------------------------------------------------- processor
def _lb_coeffs(dst: int, scale: float, ssize: int):
    """cv2 INTER_LINEAR source index + 11-bit weights per destination index (restated,
    see csrc/preprocess.hip): fx = float((d+0.5)*scale - 0.5), clamped at the borders."""
    f = ((np.arange(dst, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = 0.0, 0
    hi = s >= ssize - 1
    f[hi], s[hi] = 0.0, ssize - 1
    a0 = np.rint((np.float32(1.0) - f) * np.float32(2048.0)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048.0)).astype(np.int64)
    return s, np.minimum(s + 1, ssize - 1), a0, a1


def letterbox(image: np.ndarray, size) -> np.ndarray:
    """preproc (data_augment.py:140-156) of one H x W x 3 uint8 image -> float32 CHW:
    r = min(th/h, tw/w), resize to (int(w*r), int(h*r)), top-left paste on a 114 canvas.
    r == 1 is the reference exactly; the resize restates cv2's fixed-point INTER_LINEAR
    (vector-path rounding; exact 2x takes INTER_AREA) -- parity unpinned (no cv2)."""
    th, tw = size
    h, w = image.shape[:2]
    r = min(th / h, tw / w)
    rw, rh = int(w * r), int(h * r)
    out = np.full((th, tw, 3), 114, np.uint8)
    if rw == w and rh == h:
        res = image
    else:
        sx, sy = 1.0 / (rw / w), 1.0 / (rh / h)
        if abs(sx - 2.0) < 2.220446049250313e-16 and abs(sy - 2.0) < 2.220446049250313e-16:
            a = image.astype(np.int64)
            res = ((a[0:2 * rh:2, 0:2 * rw:2] + a[0:2 * rh:2, 1:2 * rw:2] + a[1:2 * rh:2, 0:2 * rw:2]
                    + a[1:2 * rh:2, 1:2 * rw:2] + 2) >> 2).astype(np.uint8)
        else:
            x0, x1, ax0, ax1 = _lb_coeffs(rw, sx, w)
            y0, y1, by0, by1 = _lb_coeffs(rh, sy, h)
            a = image.astype(np.int64)
            h0 = a[y0][:, x0] * ax0[None, :, None] + a[y0][:, x1] * ax1[None, :, None]
            h1 = a[y1][:, x0] * ax0[None, :, None] + a[y1][:, x1] * ax1[None, :, None]
            t = (((h0 >> 4) * by0[:, None, None]) >> 16) + (((h1 >> 4) * by1[:, None, None]) >> 16) + 2
            res = np.clip(t >> 2, 0, 255).astype(np.uint8)
    out[:rh, :rw] = res
    return np.ascontiguousarray(out.transpose(2, 0, 1), dtype=np.float32)


def detections(rows, image_hw, test_size):
    """YoloxProcessor.postprocess formatting (processor.py:39-54) of one image's [N, 7]
    float32 rows (or None): boxes / ratio as a CPU fp32 tensor op, scores as the Python
    double product of the two fp32 confidences, integer labels."""
    if rows is None:
        return {"bboxes": [], "scores": [], "labels": []}
    h, w = image_hw
    ratio = min(test_size[0] / h, test_size[1] / w)
    t = torch.from_numpy(np.asarray(rows, np.float32))
    return {"bboxes": [tuple((r[:4] / ratio).tolist()) for r in t],
            "scores": [r[4].item() * r[5].item() for r in t],
            "labels": [int(r[6]) for r in t]}
