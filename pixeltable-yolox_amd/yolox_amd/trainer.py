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
        _weights_changed(self.ema)


def _weights_changed(model: nn.Module) -> None:
    """Advance the weights epoch a replayed inference plan checks (engine.Plan.replay)."""
    m = model.module if hasattr(model, "module") else model
    if hasattr(m, "weights_changed"):
        m.weights_changed()


def train_one_iter(model: nn.Module, optimizer, images: torch.Tensor, targets: torch.Tensor,
                   amp_dtype: Optional[torch.dtype] = None, scaler=None, ema: Optional[ModelEMA] = None,
                   fused=None, captured=None) -> dict:
    """trainer.py:96-129 (minus data loading / logging / LR schedule).

    ``fused`` (yolox_amd.optim.FusedStep over the same optimizer and EMA) replaces
    ``optimizer.step()`` + ``ema.update(model)`` with one HIP pass; with a GradScaler
    (--fp16) it also takes over ``scaler.step`` / ``scaler.update`` (inf check, unscale,
    skip, scale update on the device, no host sync).

    ``captured`` (yolox_amd.train.CapturedTrainStep of this batch shape, its grad_scale the
    scaler's scale under fp16) replaces the forward + ``backward()`` with one graph replay."""
    if captured is not None:
        if fused is None:
            raise ValueError("train_one_iter(captured=...) needs the fused optimizer step")
        outputs = captured(images, targets)
        fused.step(scaler)
        return outputs
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
        _weights_changed(model)
    else:
        loss.backward()
        if fused is not None:
            fused.step()  # SGD + EMA in one pass
            return outputs
        optimizer.step()
        _weights_changed(model)
    if ema is not None:
        ema.update(model)
    return outputs


# ------------------------------------------------------------------ LR schedule
def yolox_warm_cos_lr(lr, min_lr_ratio, total_iters, warmup_total_iters, warmup_lr_start, no_aug_iter, iters):
    """utils/lr_scheduler.py:119-146 (quadratic warm-up, cosine, flat min_lr for the
    no-aug epochs)."""
    min_lr = lr * min_lr_ratio
    if iters <= warmup_total_iters:
        return (lr - warmup_lr_start) * pow(iters / float(warmup_total_iters), 2) + warmup_lr_start
    if iters >= total_iters - no_aug_iter:
        return min_lr
    return min_lr + 0.5 * (lr - min_lr) * (1.0 + math.cos(
        math.pi * (iters - warmup_total_iters) / (total_iters - warmup_total_iters - no_aug_iter)))


def cos_lr(lr, total_iters, iters):
    return lr * 0.5 * (1.0 + math.cos(math.pi * iters / total_iters))


def warm_cos_lr(lr, total_iters, warmup_total_iters, warmup_lr_start, iters):
    if iters <= warmup_total_iters:
        return (lr - warmup_lr_start) * iters / float(warmup_total_iters) + warmup_lr_start
    return 0.5 * lr * (1.0 + math.cos(math.pi * (iters - warmup_total_iters) / (total_iters - warmup_total_iters)))


class LRScheduler:
    """utils/lr_scheduler.py:7-117 for the schedules a YoloxConfig names (cos, warmcos,
    yoloxwarmcos)."""

    def __init__(self, name: str, lr: float, iters_per_epoch: int, total_epochs: int, **kwargs):
        self.lr = lr
        self.iters_per_epoch = iters_per_epoch
        self.total_epochs = total_epochs
        self.total_iters = iters_per_epoch * total_epochs
        self.__dict__.update(kwargs)
        from functools import partial
        if name == "cos":
            self.lr_func = partial(cos_lr, self.lr, self.total_iters)
        elif name == "warmcos":
            self.lr_func = partial(warm_cos_lr, self.lr, self.total_iters, self.iters_per_epoch * self.warmup_epochs,
                                   getattr(self, "warmup_lr_start", 1e-6))
        elif name == "yoloxwarmcos":
            self.lr_func = partial(yolox_warm_cos_lr, self.lr, getattr(self, "min_lr_ratio", 0.2), self.total_iters,
                                   self.iters_per_epoch * self.warmup_epochs, getattr(self, "warmup_lr_start", 0),
                                   self.iters_per_epoch * self.no_aug_epochs)
        else:
            raise ValueError(f"Scheduler version {name} not supported.")

    def update_lr(self, iters: int) -> float:
        return self.lr_func(iters)


# ------------------------------------------------------------------ data
class InfiniteSampler:
    """data/samplers.py:28-82: an infinite stream of seeded shuffles of range(size); rank r
    of w reads elements r, r + w, r + 2w, ... (every rank sees a disjoint slice)."""

    def __init__(self, size: int, shuffle: bool = True, seed: int = 0, rank: Optional[int] = None,
                 world_size: Optional[int] = None):
        from .launch import get_rank, get_world_size
        assert size > 0
        self._size, self._shuffle, self._seed = size, shuffle, int(seed)
        self._rank = get_rank() if rank is None else rank
        self._world_size = get_world_size() if world_size is None else world_size

    def _infinite_indices(self):
        g = torch.Generator()
        g.manual_seed(self._seed)
        while True:
            if self._shuffle:
                yield from torch.randperm(self._size, generator=g).tolist()
            else:
                yield from range(self._size)

    def __iter__(self):
        import itertools
        yield from itertools.islice(self._infinite_indices(), self._rank, None, self._world_size)

    def __len__(self) -> int:
        return self._size // self._world_size


# ------------------------------------------------------------------ trainer
class Trainer:
    """core/trainer.py:34-330 on the HIP path: before_train builds the model, the reference
    optimizer groups, the data loader (per-rank batch), the yoloxwarmcos schedule, DDP
    (yolox_amd.dp) and EMA; ``train_one_iter`` is trainer.py:96-129 -- dtype cast,
    ``config.preprocess`` to the current multiscale size, autocast forward, scaled backward,
    fused SGD + EMA (+ GradScaler) step, LR update; ``after_iter`` redraws the input size
    every 10 iterations on rank 0 and broadcasts it (:301-306).  Logging is a print every
    ``print_interval`` iterations on rank 0; evaluation / checkpoint files are out of scope
    (DESIGN.md).  ``args.max_iter`` (not in the reference) stops after that many iterations."""

    def __init__(self, config, args):
        from .launch import get_local_rank, get_rank, get_world_size
        self.exp = config
        self.args = args
        self.max_epoch = config.max_epoch
        self.amp_training = bool(args.fp16)
        self.scaler = torch.amp.GradScaler("cuda", enabled=self.amp_training)
        self.is_distributed = get_world_size() > 1
        self.rank = get_rank()
        self.local_rank = get_local_rank()
        self.device = f"cuda:{self.local_rank}"
        self.use_model_ema = config.ema
        self.data_type = torch.float16 if args.fp16 else torch.float32
        self.input_size = tuple(config.input_size)
        self.start_epoch = 0
        self.last = None  # (progress, input_size, detached loss) of the latest iteration only

    def train(self) -> None:
        self.before_train()
        self.train_in_epoch()

    def train_in_epoch(self) -> None:
        for self.epoch in range(self.start_epoch, self.max_epoch):
            self.before_epoch()
            if not self.train_in_iter():
                return

    def train_in_iter(self) -> bool:
        limit = getattr(self.args, "max_iter", None)
        for self.iter in range(self.max_iter):
            if limit is not None and self.progress_in_iter >= limit:
                return False
            self.train_one_iter()
            self.after_iter()
        return True

    @property
    def progress_in_iter(self) -> int:
        return self.epoch * self.max_iter + self.iter

    def before_train(self) -> None:
        from .dp import DistributedDataParallel
        from .optim import FusedStep
        torch.cuda.set_device(self.local_rank)
        model = self.exp.get_model()
        model.to(self.device)
        self.optimizer = self.exp.get_optimizer(self.args.batch_size)
        self.no_aug = self.start_epoch >= self.max_epoch - self.exp.no_aug_epochs
        self.train_loader = self.exp.get_data_loader(batch_size=self.args.batch_size,
                                                     is_distributed=self.is_distributed, no_aug=self.no_aug,
                                                     dataset_size=getattr(self.args, "dataset_size", 118287))
        self.max_iter = len(self.train_loader)
        self.lr_scheduler = self.exp.get_lr_scheduler(self.exp.basic_lr_per_img * self.args.batch_size,
                                                      self.max_iter)
        if self.is_distributed:
            model = DistributedDataParallel(model, device_ids=[self.local_rank], broadcast_buffers=False)
        self.ema_model = None
        if self.use_model_ema:
            self.ema_model = ModelEMA(model, 0.9998)
            self.ema_model.updates = self.max_iter * self.start_epoch
        self.model = model
        self.fused = FusedStep(model, self.optimizer, self.ema_model)

    def before_epoch(self) -> None:
        if self.epoch + 1 == self.max_epoch - self.exp.no_aug_epochs or self.no_aug:
            self.train_loader.close_mosaic()
            m = self.model.module if self.is_distributed else self.model
            m.head.use_l1 = True

    def train_one_iter(self) -> None:
        inps, targets = self.train_loader.next()
        inps = inps.to(self.device, non_blocking=True).to(self.data_type)
        targets = targets.to(self.device, non_blocking=True).to(self.data_type)
        targets.requires_grad = False
        inps, targets = self.exp.preprocess(inps, targets, self.input_size)
        with torch.autocast("cuda", dtype=torch.float16, enabled=self.amp_training):
            outputs = self.model(inps, targets)
        loss = outputs["total_loss"]
        self.optimizer.zero_grad(set_to_none=True)
        self.scaler.scale(loss).backward()
        self.fused.step(self.scaler if self.amp_training else None)  # SGD + EMA (+ scaler.step/update)
        lr = self.lr_scheduler.update_lr(self.progress_in_iter + 1)
        for param_group in self.optimizer.param_groups:
            param_group["lr"] = lr
        self.last = (self.progress_in_iter, self.input_size, loss.detach())

    def after_iter(self) -> None:
        if self.rank == 0 and (self.iter + 1) % self.exp.print_interval == 0:
            _, size, loss = self.last
            print(f"epoch: {self.epoch + 1}/{self.max_epoch}, iter: {self.iter + 1}/{self.max_iter}, "
                  f"total_loss: {float(loss):.3f}, lr: {self.optimizer.param_groups[0]['lr']:.3e}, size: {size[0]}",
                  flush=True)
        if not self.exp.deterministic and (self.progress_in_iter + 1) % 10 == 0:
            self.input_size = self.exp.random_resize(self.train_loader, self.epoch, self.rank, self.is_distributed)
