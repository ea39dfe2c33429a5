"""YoloxConfig: model/test/train settings and the named presets.

Mirrors the reference's ``yolox.config.YoloxConfig`` API (config.py:17-157,
412-469): the same field names and defaults, ``get_named_config`` accepting ``-``
or ``_``, ``update`` with type coercion, ``validate`` and ``get_model``.  Named
configs are module-level singletons, as in the reference (quirk: they cache the
model they build, config.py:168-172, 466-469).  Data-loader / evaluator factories
(CPU data pipeline, COCO files) are out of scope.
"""
from __future__ import annotations

import ast
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
