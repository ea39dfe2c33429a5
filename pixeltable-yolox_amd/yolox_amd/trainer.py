"""One training iteration of the reference's Trainer on the HIP path.

Mirrors ``Trainer.train_one_iter`` (reference core/trainer.py:96-129): autocast forward
-> zero_grad -> (scaled) backward -> optimizer step -> EMA update, with the reference's
optimizer grouping (config.py:307-333: SGD nesterov, momentum 0.9; BN weights without
decay, conv weights with weight decay, biases) and ModelEMA (utils/ema.py:20-58, decay
0.9998 * (1 - exp(-updates / 2000)) over every floating state_dict entry).  The step's
element-wise optimizer / EMA / GradScaler passes run fused on the device
(yolox_amd.optim.FusedStep) or as torch multi-tensor kernels; the forward/backward is the
HIP path (yolox_amd.train), data parallel through yolox_amd.dp.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn


def get_optimizer(model: nn.Module, lr: float, momentum: float = 0.9, weight_decay: float = 5e-4):
    """config.py:307-333 parameter groups."""
    pg0, pg1, pg2 = [], [], []
    for k, v in model.named_modules():
        if hasattr(v, "bias") and isinstance(v.bias, nn.Parameter):
            pg2.append(v.bias)
        if isinstance(v, nn.BatchNorm2d) or "bn" in k:
            pg0.append(v.weight)
        elif hasattr(v, "weight") and isinstance(v.weight, nn.Parameter):
            pg1.append(v.weight)
    opt = torch.optim.SGD(pg0, lr=lr, momentum=momentum, nesterov=True, foreach=True)
    opt.add_param_group({"params": pg1, "weight_decay": weight_decay})
    opt.add_param_group({"params": pg2})
    return opt


class ModelEMA:
    """utils/ema.py:20-58 with multi-tensor updates."""

    def __init__(self, model: nn.Module, decay: float = 0.9998, updates: int = 0):
        import copy
        m = model.module if hasattr(model, "module") else model
        self.ema = copy.deepcopy(m).eval()
        self.updates = updates
        self.decay = lambda x: decay * (1 - math.exp(-x / 2000))
        for p in self.ema.parameters():
            p.requires_grad_(False)
        self._pairs = None

    def update(self, model: nn.Module) -> None:
        m = model.module if hasattr(model, "module") else model
        if self._pairs is None:
            msd = m.state_dict()
            e, s = [], []
            for k, v in self.ema.state_dict().items():
                if v.dtype.is_floating_point:
                    e.append(v)
                    s.append(msd[k])
            self._pairs = (e, s)
        with torch.no_grad():
            self.updates += 1
            d = self.decay(self.updates)
            e, s = self._pairs
            torch._foreach_mul_(e, d)
            torch._foreach_add_(e, [t.detach() for t in s], alpha=1.0 - d)


def train_one_iter(model: nn.Module, optimizer, images: torch.Tensor, targets: torch.Tensor,
                   amp_dtype: Optional[torch.dtype] = None, scaler=None, ema: Optional[ModelEMA] = None,
                   fused=None) -> dict:
    """trainer.py:96-129 (minus data loading / logging / LR schedule).

    ``fused`` (yolox_amd.optim.FusedStep over the same optimizer and EMA) replaces
    ``optimizer.step()`` + ``ema.update(model)`` with one HIP pass; with a GradScaler
    (--fp16) it also takes over ``scaler.step`` / ``scaler.update`` (inf check, unscale,
    skip, scale update on the device, no host sync)."""
    with torch.autocast("cuda", dtype=amp_dtype or torch.float16, enabled=amp_dtype is not None):
        outputs = model(images, targets)
    loss = outputs["total_loss"]
    optimizer.zero_grad(set_to_none=True)
    if scaler is not None:
        scaler.scale(loss).backward()
        if fused is not None:
            fused.step(scaler)  # scaler.step + scaler.update + EMA in three launches
            return outputs
        scaler.step(optimizer)
        scaler.update()
    else:
        loss.backward()
        if fused is not None:
            fused.step()  # SGD + EMA in one pass
            return outputs
        optimizer.step()
    if ema is not None:
        ema.update(model)
    return outputs
