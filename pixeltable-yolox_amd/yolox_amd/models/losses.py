"""YOLOX training losses with on-device SimOTA (yxh_yolox_loss).

Replaces YoloxHead.get_losses (reference yolo_head.py:253-411): the reference loops
over images and ground truths in Python with host syncs; here one call assigns and
reduces the whole batch on the device.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .. import _native as N

LOSS_KEYS = ("total_loss", "iou_loss", "conf_loss", "cls_loss", "l1_loss", "num_fg")


def yolox_losses(outputs: torch.Tensor, labels: torch.Tensor, level_hw: Sequence[tuple[int, int]],
                 strides: Sequence[int] = (8, 16, 32), origin_reg: Optional[torch.Tensor] = None):
    """outputs [B, A, 5+C] (train-mode decoded boxes, raw obj/cls logits), labels
    [B, L, 5].  Returns (losses dict of 0-d tensors, assignment dict)."""
    N.require_device(outputs, "outputs")
    if outputs.dtype != torch.float32:
        raise ValueError("outputs must be float32")
    B, A, D = outputs.shape
    C = D - 5
    L = labels.shape[1]
    dev = outputs.device
    outputs = outputs.contiguous()
    labels = labels.to(dev, torch.float32).contiguous()
    if origin_reg is not None:
        origin_reg = origin_reg.to(dev, torch.float32).contiguous()
    # level geometry is read on the host by the launcher (host arrays, not device memory)
    hw = torch.tensor([v for h, w in level_hw for v in (h, w)], dtype=torch.int32)
    st = torch.tensor(list(strides), dtype=torch.int32)
    fg = torch.empty(B, A, dtype=torch.uint8, device=dev)
    matched = torch.empty(B, A, dtype=torch.int32, device=dev)
    piou = torch.empty(B, A, dtype=torch.float32, device=dev)
    num_fg = torch.empty(B, dtype=torch.int32, device=dev)
    losses = torch.empty(6, dtype=torch.float32, device=dev)
    lib = N.lib()
    ws = torch.empty(int(lib.yxh_yolox_loss_workspace_bytes(B, A, L)), dtype=torch.uint8, device=dev)
    N.check(lib.yxh_yolox_loss(
        outputs.data_ptr(), origin_reg.data_ptr() if origin_reg is not None else None, labels.data_ptr(), B, A, C,
        L, hw.data_ptr(), st.data_ptr(), len(strides), fg.data_ptr(), matched.data_ptr(), piou.data_ptr(),
        num_fg.data_ptr(), losses.data_ptr(), ws.data_ptr(), ws.numel(), N.stream_ptr(dev)), "yolox_loss")
    out = {k: losses[i] for i, k in enumerate(LOSS_KEYS)}
    assign = {"fg_mask": fg.bool(), "matched_gt_inds": matched, "pred_ious": piou, "num_fg": num_fg}
    return out, assign
