"""YoloxConfig: model/test/train settings and the named presets.

Mirrors the reference's ``yolox.config.YoloxConfig`` API (config.py:17-157,
412-469): the same field names and defaults, ``get_named_config`` accepting ``-``
or ``_``, ``update`` with type coercion, ``validate`` and ``get_model``.  Named
configs are module-level singletons, as in the reference (quirk: they cache the
model they build, config.py:168-172, 466-469).  The training-side factories the
trainer calls are here too: ``get_optimizer`` (:307-333), ``get_lr_scheduler``
(:335-348), ``random_resize`` (:275-294, rank-0 draw broadcast to every rank),
``preprocess`` (:296-305, bilinear multiscale on the device) and ``get_data_loader`` -- the latter
over a synthetic COCO-shaped dataset (no datasets offline; COCO files and the
Mosaic/MixUp CPU pipeline are out of scope).
"""
from __future__ import annotations

import ast
import random
from dataclasses import dataclass, field
from typing import Any, Literal, Optional


@dataclass
class YoloxConfig:
    name: str
    # model
    num_classes: int = 80
    depth: float = 1.00
    width: float = 1.00
    depthwise: bool = False
    act: Literal["silu", "relu", "lrelu"] = "silu"
    seed: Optional[Any] = None
    output_dir: str = "./out"
    # data
    deterministic: bool = False
    data_num_workers: int = 4
    input_size: tuple[int, int] = (640, 640)
    multiscale_range: int = 5
    random_size: Optional[tuple[int, int]] = None
    data_dir: Optional[str] = None
    train_ann: str = "instances_train2017.json"
    val_ann: str = "instances_val2017.json"
    test_ann: str = "instances_test2017.json"
    # augmentation
    mosaic_prob: float = 1.0
    mixup_prob: float = 1.0
    hsv_prob: float = 1.0
    flip_prob: float = 0.5
    degrees: float = 10.0
    translate: float = 0.1
    mosaic_scale: tuple[float, float] = (0.1, 2)
    enable_mixup: bool = True
    mixup_scale: tuple[float, float] = (0.5, 1.5)
    shear: float = 2.0
    # training
    warmup_epochs: int = 5
    max_epoch: int = 300
    warmup_lr: int = 0
    min_lr_ratio: float = 0.05
    basic_lr_per_img: float = 0.01 / 64.0
    scheduler: str = "yoloxwarmcos"
    no_aug_epochs: int = 15
    ema: bool = True
    weight_decay: float = 5e-4
    momentum: float = 0.9
    print_interval: int = 10
    eval_interval: int = 10
    save_history_ckpt: bool = True
    # testing
    test_size: tuple[int, int] = (640, 640)
    test_conf: float = 0.01
    nmsthre: float = 0.65
    model: Any = field(default=None, repr=False, compare=False)

    @classmethod
    def get_named_config(cls, name: str) -> Optional["YoloxConfig"]:
        return _NAMED_CONFIG.get(name.replace("-", "_"))

    def validate(self) -> None:
        h, w = self.input_size
        assert h % 32 == 0 and w % 32 == 0, "input size must be multiples of 32"

    def update(self, opts: dict[str, str]) -> None:
        """``-D key=value`` overrides with the reference's coercion rules (config.py:129-157)."""
        for k, v in opts.items():
            if not hasattr(self, k) or k == "model":
                raise AttributeError(f"Unknown model configuration option: {k}")
            cur = getattr(self, k)
            if isinstance(cur, (list, tuple)):
                items = [t.strip() for t in str(v).strip("[]()").split(",")]
                if cur:
                    items = [type(cur[0])(t) for t in items]
                v = items
            if cur is not None and type(cur) is not type(v):
                try:
                    v = type(cur)(v)
                except Exception:
                    v = ast.literal_eval(v)
            if k == "seed":
                v = int(v)
            setattr(self, k, v)

    def get_model(self):
        """Build (once) the YoloxModule for this config: BN eps 1e-3 / momentum 0.03,
        prior-probability bias init 1e-2 (config.py:159-177), train mode."""
        from .models.network import YoloPafpn, YoloxHead
        from .models.yolox import YoloxModule

        if self.model is None:
            in_ch = [256, 512, 1024]
            backbone = YoloPafpn(self.depth, self.width, in_channels=in_ch, depthwise=self.depthwise, act=self.act)
            head = YoloxHead(self.num_classes, self.width, in_channels=in_ch, depthwise=self.depthwise, act=self.act)
            self.model = YoloxModule(backbone, head)
        import torch.nn as nn

        for m in self.model.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eps = 1e-3
                m.momentum = 0.03
        self.model.head.initialize_biases(1e-2)
        self.model.train()
        return self.model

    # ------------------------------------------------------------ training factories
    def get_optimizer(self, batch_size: int):
        """config.py:307-333: SGD nesterov, BN weights without decay, conv weights with
        ``weight_decay``, biases; lr = warmup_lr while warming up (the scheduler sets it
        from the first iteration on)."""
        if getattr(self, "optimizer", None) is None:
            from .trainer import get_optimizer
            lr = self.warmup_lr if self.warmup_epochs > 0 else self.basic_lr_per_img * batch_size
            self.optimizer = get_optimizer(self.model, lr, self.momentum, self.weight_decay)
        return self.optimizer

    def get_lr_scheduler(self, lr: float, iters_per_epoch: int):
        """config.py:335-348."""
        from .trainer import LRScheduler
        return LRScheduler(self.scheduler, lr, iters_per_epoch, self.max_epoch, warmup_epochs=self.warmup_epochs,
                           warmup_lr_start=self.warmup_lr, no_aug_epochs=self.no_aug_epochs,
                           min_lr_ratio=self.min_lr_ratio)

    def get_data_loader(self, batch_size: int, is_distributed: bool, no_aug: bool = False, cache_img=None,
                        dataset_size: int = 118287, device=None, distinct_images: int = 512, dataset=None):
        """config.py:203-273 on the device pipeline: MosaicDetection (mosaic / random affine /
        mixup) + TrainTransform (HSV / mirror / padded labels) over a ``pull_item`` detection
        dataset whose images live in HBM (yolox_amd.data.GpuMosaicDetection: the host draws the
        reference's random numbers in its order and does the label arithmetic, one
        yxh_augment_batch launch renders the batch).  ``dataset`` defaults to the synthetic
        COCO-shaped one (no datasets offline: ``dataset_size`` items over ``distinct_images``
        resident images).  The per-rank batch is batch_size // world (:249-250) and every rank
        reads its rank-strided slice of one seeded shuffled index stream (InfiniteSampler,
        samplers.py:28-82); ``no_aug`` starts with mosaic off (YoloBatchSampler(mosaic=not
        no_aug), :255-260), ``close_mosaic()`` turns it off later (trainer.py:217-230)."""
        from .data.mosaic import GpuMosaicDetection, MosaicBatches, SyntheticDetectionDataset, TrainTransform
        from .launch import get_world_size
        from .trainer import InfiniteSampler
        if is_distributed:
            batch_size = batch_size // get_world_size()
        seed = self.seed if self.seed else 0
        if dataset is None:
            dataset = SyntheticDetectionDataset(dataset_size, self.input_size, seed=seed,
                                                num_classes=self.num_classes, distinct=distinct_images)
        ds = GpuMosaicDetection(
            dataset, self.input_size, mosaic=not no_aug,
            preproc=TrainTransform(max_labels=120, flip_prob=self.flip_prob, hsv_prob=self.hsv_prob),
            degrees=self.degrees, translate=self.translate, mosaic_scale=self.mosaic_scale,
            mixup_scale=self.mixup_scale, shear=self.shear, enable_mixup=self.enable_mixup,
            mosaic_prob=self.mosaic_prob, mixup_prob=self.mixup_prob, device=device or "cuda")
        sampler = InfiniteSampler(len(ds), seed=seed)
        return MosaicBatches(ds, sampler, batch_size)

    def get_eval_loader(self, batch_size: int, is_distributed: bool, dataset=None, testdev: bool = False,
                        legacy: bool = False):
        """config.py:350-382 over any ``pull_item`` detection dataset with ``.coco`` (the ground
        truth: a COCO json dict or pycocotools COCO) and ``.class_ids``: (imgs, targets, info_imgs,
        ids) batches letterboxed to test_size on the device (ValTransform = yxh_letterbox_batch;
        ``legacy``: ValTransform(legacy=True)'s channel flip + /255 + mean/std, data_augment.py:236-240);
        distributed: batch_size // world per rank over the rank's contiguous-strided shard (the
        DistributedSampler without its padding duplicates).  COCO dataset readers are out of scope
        (no datasets offline): ``dataset`` is required -- ``testdev`` picks the reference's
        annotation file (test_ann), so here it is the caller's choice of ``dataset``."""
        from .evaluators.coco_evaluator import EvalLoader
        if dataset is None:
            raise NotImplementedError("COCO dataset readers are out of scope: pass dataset= (pull_item, coco, "
                                      "class_ids)")
        rank, world = 0, 1
        if is_distributed:
            import torch.distributed as dist
            rank, world = dist.get_rank(), dist.get_world_size()
            batch_size = batch_size // world
        return EvalLoader(dataset, batch_size, self.test_size, rank, world, legacy=legacy)

    def get_evaluator(self, batch_size: int, is_distributed: bool, testdev: bool = False, legacy: bool = False,
                      dataset=None):
        """config.py:384-395."""
        from .evaluators import CocoEvaluator
        return CocoEvaluator(dataloader=self.get_eval_loader(batch_size, is_distributed, dataset=dataset,
                                                             testdev=testdev, legacy=legacy),
                             img_size=self.test_size, confthre=self.test_conf, nmsthre=self.nmsthre,
                             num_classes=self.num_classes, testdev=testdev)

    def eval(self, model, evaluator, is_distributed: bool, half: bool = False, return_outputs: bool = False):
        """config.py:403-404."""
        return evaluator.evaluate(model, is_distributed, half, return_outputs=return_outputs)

    def random_resize(self, data_loader, epoch: int, rank: int, is_distributed: bool):
        """config.py:275-294: rank 0 draws the next multiscale input size (multiples of 32
        around input_size) and broadcasts it; every rank returns the same (h, w)."""
        import torch
        import torch.distributed as dist
        dev = "cuda" if is_distributed and dist.get_backend() == "nccl" else "cpu"
        tensor = torch.zeros(2, dtype=torch.int64, device=dev)
        if rank == 0:
            size_factor = self.input_size[1] * 1.0 / self.input_size[0]
            if self.random_size is None:
                min_size = int(self.input_size[0] / 32) - self.multiscale_range
                max_size = int(self.input_size[0] / 32) + self.multiscale_range
                self.random_size = (min_size, max_size)
            size = random.randint(*self.random_size)
            size = (int(32 * size), 32 * int(size * size_factor))
            tensor[0] = size[0]
            tensor[1] = size[1]
        if is_distributed:
            dist.barrier()
            dist.broadcast(tensor, 0)
        return (int(tensor[0].item()), int(tensor[1].item()))

    def preprocess(self, inputs, targets, tsize):
        """config.py:296-305: bilinear resize of the batch to ``tsize`` (align_corners False:
        yxh_resize_bilinear, one HIP launch, ATen's arithmetic) with the box columns scaled to
        match (``scale_targets``).  The batch must be on the ROCm device (the training loader
        produces it there); a CPU batch raises ValueError rather than taking another resize."""
        from .utils.resize import resize_bilinear
        if self._multiscale(tsize) != (1, 1):
            inputs = resize_bilinear(inputs, tsize)
            targets = self.scale_targets(targets, tsize)
        return inputs, targets

    def _multiscale(self, tsize):
        return tsize[1] / self.input_size[1], tsize[0] / self.input_size[0]

    def scale_targets(self, targets, tsize):
        """The label half of ``preprocess`` (config.py:301-304): x columns (1, 3) and y columns
        (2, 4) of [B, L, 5] targets scaled by tsize / input_size, in place."""
        scale_x, scale_y = self._multiscale(tsize)
        if scale_x != 1 or scale_y != 1:
            targets[..., 1::2] = targets[..., 1::2] * scale_x
            targets[..., 2::2] = targets[..., 2::2] * scale_y
        return targets

    def get_trainer(self, args):
        from .trainer import Trainer
        return Trainer(self, args)


_PRESETS: dict[str, dict[str, Any]] = {
    "yolox_s": dict(depth=0.33, width=0.50),
    "yolox_m": dict(depth=0.67, width=0.75),
    "yolox_l": dict(depth=1.0, width=1.0),
    "yolox_x": dict(depth=1.33, width=1.25),
    "yolox_tiny": dict(depth=0.33, width=0.375, input_size=(416, 416), random_size=(10, 20),
                       mosaic_scale=(0.5, 1.5), test_size=(416, 416), enable_mixup=False),
    "yolox_nano": dict(depth=0.33, width=0.25, depthwise=True, input_size=(416, 416), random_size=(10, 20),
                       mosaic_scale=(0.5, 1.5), test_size=(416, 416), mosaic_prob=0.5, enable_mixup=False),
}

_NAMED_CONFIG: dict[str, YoloxConfig] = {n: YoloxConfig(n, **kw) for n, kw in _PRESETS.items()}


def named_config(name: str) -> YoloxConfig:
    """A fresh (non-singleton) copy of a preset."""
    key = name.replace("-", "_")
    if key not in _PRESETS:
        raise ValueError(f"Unknown model: {name}")
    return YoloxConfig(key, **_PRESETS[key])
