"""Yolox / YoloxModule: the drop-in façade (reference yolox/models/yolox.py:22-131).

Differences from the reference, all deliberate:
* execution is the libyoloxhip plan (engine.py) on a ROCm device -- there is no
  CPU path; CPU inputs are moved to the module's device;
* ``from_pretrained(<name>)`` never downloads (no network): it loads
  ``$YOLOX_HOME/weights/<name>.pth`` if present and raises FileNotFoundError
  otherwise; ``YoloxModule.synthetic(name)`` builds seeded weights instead;
* the compute dtype follows the parameters: float32 by default (numerical parity
  with the reference), bfloat16 / float16 after ``.to(dtype)`` / ``.half()``;
* ``from_pretrained(..., device=...)`` defaults to the ROCm device (the reference's
  default is ``'cpu'``, yolox.py:35,103) and refuses a non-ROCm device right there,
  before anything is loaded, instead of at the first forward.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Iterable, Optional, Union

import torch
import torch.nn as nn

from .. import _native as N
from ..config import YoloxConfig, named_config
from .network import YoloPafpn, YoloxHead
from .processor import Detections, YoloxProcessor

HOME = Path(os.environ.get("YOLOX_HOME", str(Path.home() / ".cache" / "yolox")))


def fold_master(masters: dict, t: torch.Tensor) -> Optional[torch.Tensor]:
    """The float32 fold master of parameter / buffer ``t`` in a YoloxModule's ``masters`` (see
    YoloxModule._record_masters), or None when it has none or ``t`` changed since its cast."""
    m = masters.get(id(t))
    if m is None or m[2] != t.data_ptr() or m[3] != t._version:
        return None
    return m[1]


def default_device() -> str:
    return "cuda" if torch.cuda.is_available() else "cpu"


class YoloxModule(nn.Module):
    def __init__(self, backbone: Optional[YoloPafpn] = None, head: Optional[YoloxHead] = None):
        super().__init__()
        self.backbone = backbone if backbone is not None else YoloPafpn()
        self.head = head if head is not None else YoloxHead(80)
        self._plans: dict = {}
        self._weights_epoch = 0  # advanced on every weight change the captured plans must see
        # fp32 fold masters (below): one dict for the module's life, mutated in place, which every
        # submodule also holds -- a submodule planned on its own (module.backbone(x), a block) folds
        # from it too
        self.__dict__["_masters"] = {}
        for m in self.modules():
            if m is not self:
                m.__dict__["_fold_masters"] = self._masters

    def weights_changed(self) -> None:
        """Tell captured plans (engine.Plan.replay) that parameters or BN statistics were
        edited in place; load_state_dict and FusedStep.step call this themselves."""
        self._weights_epoch += 1

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        r = super().load_state_dict(state_dict, strict=strict, assign=assign)
        # a float32 state dict loaded into a 16-bit module: keep its values as the fold masters
        self._record_masters({k: v for k, v in state_dict.items()
                              if torch.is_tensor(v) and v.dtype == torch.float32})
        self.weights_changed()
        return r

    # ---------------------------------------------------------------- fp32 fold masters
    # Perf mode (``.to(torch.bfloat16)`` / ``.half()``) rounds every parameter AND the BatchNorm
    # statistics to 16 bits.  Folding BN into the conv weights from those rounded values
    # (w16 * g16 / sqrt(var16 + eps), beta16 - mean16 * ...) rounds each weight twice and shifts
    # every channel's bias by up to half a 16-bit ulp of beta and mean -- an offset shared by all
    # pixels of the channel, which the next layers do not average out.  Measured on the 32
    # configs[1] images (tools/map_noise.py, profiles/r06/map_noise.txt): the oracle with
    # bf16-rounded parameters + bf16 storage is 1.56x further from the fp32 oracle at p99 than
    # with fp32 parameters -- the device's whole round-5 excess.  So the module keeps the float32
    # values it had before the cast (on the module's device), and the plans fold from them: the
    # packed weights are rounded once.  A master is used only while its 16-bit parameter is the
    # tensor (storage and version) the cast produced; any later edit of that parameter makes the
    # plan fold from the edited 16-bit value.
    def _float_tensors(self):
        for n, t in self.named_parameters():
            if t.is_floating_point():
                yield n, t
        for n, t in self.named_buffers():
            if t.is_floating_point():
                yield n, t

    def _record_masters(self, sources: dict) -> None:
        """sources: name -> float32 value of that parameter / buffer before its 16-bit cast."""
        masters = self._masters
        for n, t in self._float_tensors():
            src = sources.get(n)
            if t.dtype in (torch.bfloat16, torch.float16) and src is not None and tuple(src.shape) == tuple(t.shape):
                masters[id(t)] = (n, src.detach().to(t.device, torch.float32).contiguous(), t.data_ptr(), t._version)
            elif id(t) in masters and t.dtype == torch.float32:
                del masters[id(t)]

    def fp32_master(self, t: torch.Tensor) -> Optional[torch.Tensor]:
        """The float32 value ``t`` (a parameter or BN buffer of this module) had before its
        16-bit cast, if ``t`` is unchanged since; else None."""
        return fold_master(self._masters, t)

    # ---------------------------------------------------------------- execution
    @property
    def compute_dtype(self) -> torch.dtype:
        return self.backbone.backbone.stem.conv.conv.weight.dtype

    @property
    def device(self) -> torch.device:
        return self.backbone.backbone.stem.conv.conv.weight.device

    def plan_for(self, batch: int, height: int, width: int, input_layout: int = N.NCHW,
                 input_dtype: torch.dtype = torch.float32, dtype: Optional[torch.dtype] = None,
                 chunk: Optional[int] = None, parallel_chunks: bool = False):
        """The (cached) HIP execution plan for this input geometry (``chunk``: images
        per pass of the op list; ``parallel_chunks``: chunks on arenas of their own, run
        side by side in the captured graph -- see engine.Plan)."""
        from ..engine import Plan

        dtype = dtype or self.compute_dtype
        key = (batch, height, width, input_layout, input_dtype, dtype, str(self.device), chunk, parallel_chunks,
               bool(self.head.decode_in_inference))
        plan = self._plans.get(key)
        if plan is None:
            if self.device.type != "cuda":
                raise RuntimeError("YoloxModule runs on a ROCm device only; call .to('cuda') first")
            plan = Plan(self, batch, height, width, dtype, self.device, input_layout, input_dtype, chunk=chunk,
                        parallel_chunks=parallel_chunks)
            self._plans[key] = plan
        return plan

    def forward(self, x, targets=None):
        if self.training:
            # yolox.py:76-87: loss dict; BN batch statistics, on-device SimOTA, HIP
            # reverse pass behind total_loss.backward() (yolox_amd/train.py)
            assert targets is not None
            from ..train import train_forward

            if self.device.type != "cuda":
                raise RuntimeError("YoloxModule runs on a ROCm device only; call .to('cuda') first")
            return train_forward(self, x, targets)
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected [B, 3, H, W] images, got {tuple(x.shape)}")
        B, _, H, W = x.shape
        if x.dtype not in (torch.float32, torch.bfloat16, torch.float16, torch.uint8):
            x = x.float()
        plan = self.plan_for(B, H, W, N.NCHW, x.dtype)
        return plan.run(x, out=torch.empty_like(plan.output))

    def forward_nhwc(self, x: torch.Tensor) -> torch.Tensor:
        """Eval forward from letterboxed NHWC images ([B, H, W, 3] uint8 / bfloat16 on
        the device, as YoloxProcessor.images_to_device writes them): the fused
        Focus+stem conv reads them directly, so no float32 NCHW tensor is built.  Same
        output as ``forward`` on the equivalent float32 NCHW tensor."""
        if self.training:
            raise RuntimeError("forward_nhwc is the eval path")
        if x.dim() != 4 or x.shape[3] != 3:
            raise ValueError(f"expected [B, H, W, 3] images, got {tuple(x.shape)}")
        B, H, W, _ = x.shape
        plan = self.plan_for(B, H, W, N.NHWC, x.dtype)
        return plan.run(x, out=torch.empty_like(plan.output))

    def _apply(self, fn, *args, **kwargs):
        self._plans = {}  # device / dtype changes invalidate every plan
        # float32 values before the cast (or the masters of a 16-bit module being moved): the
        # fold masters of the 16-bit result (see _record_masters)
        before = {}
        for n, t in self._float_tensors():
            if t.dtype == torch.float32:
                before[n] = t.data
            elif self.fp32_master(t) is not None:
                before[n] = self.fp32_master(t)
        r = super()._apply(fn, *args, **kwargs)
        self._masters.clear()
        self._record_masters(before)
        return r

    # ---------------------------------------------------------------- loading
    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: Union[str, os.PathLike],
                        config: Optional[YoloxConfig] = None, device: Optional[str] = None) -> "YoloxModule":
        """yolox.py:100-131 (a local checkpoint, eval mode, on ``device``): the reference's
        argument errors first, then a non-ROCm device is refused before anything is loaded."""
        path, config = cls._checkpoint_path(pretrained_model_name_or_path, config)
        dev = torch.device(device or default_device())
        if dev.type != "cuda":
            raise RuntimeError(f"YoloxModule runs on a ROCm device only (device={str(dev)!r}): the HIP path has "
                               "no CPU execution; pass device='cuda' (the reference's CPU default is not supported)")
        return cls.load_checkpoint(path, config).to(dev)

    @staticmethod
    def _checkpoint_path(name_or_path, config):
        """(checkpoint file, config) as yolox.py:109-127 resolves them -- without the download."""
        path = str(name_or_path)
        if os.path.isfile(path):
            if config is None:
                raise ValueError("config must be provided when loading model from a file")
            return path, config
        config = YoloxConfig.get_named_config(path)
        if config is None:
            raise ValueError(f"Unknown model: {name_or_path}")
        path = str(HOME / "weights" / f"{config.name}.pth")
        if not os.path.isfile(path):
            raise FileNotFoundError(
                f"{path} not found: pretrained weights are not downloaded by yolox_amd (no network); "
                "place the MegVii checkpoint there or use YoloxModule.synthetic()")
        return path, config

    @classmethod
    def load_checkpoint(cls, pretrained_model_name_or_path: Union[str, os.PathLike],
                        config: Optional[YoloxConfig] = None) -> "YoloxModule":
        """The loading half of ``from_pretrained``: the model built from ``config`` with the
        checkpoint's weights (weights_only load), on the host, eval mode."""
        path, config = cls._checkpoint_path(pretrained_model_name_or_path, config)
        model = config.get_model()
        weights = torch.load(path, map_location="cpu", weights_only=True)
        model.load_state_dict(weights["model"] if "model" in weights else weights)
        model.eval()
        return model

    @classmethod
    def synthetic(cls, name: str = "yolox_s", seed: int = 0, device: Optional[str] = None,
                  dtype: torch.dtype = torch.float32) -> "YoloxModule":
        """A fresh model of preset ``name`` with seeded weights and calibrated BN
        statistics (yolox_amd.weights) -- used by tests and the benchmark."""
        from ..weights import synthetic_state_dict

        cfg = named_config(name)
        model = cfg.get_model()
        model.load_state_dict(synthetic_state_dict(model.state_dict(), seed=seed, bn_stats=cfg.name))
        model = model.to(device or default_device(), dtype)
        model.eval()
        return model


class Yolox:
    module: YoloxModule
    processor: YoloxProcessor

    def __init__(self, module: YoloxModule, processor: YoloxProcessor):
        self.module = module
        self.processor = processor

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: Union[str, os.PathLike],
                        config: Optional[YoloxConfig] = None, device: Optional[str] = None) -> "Yolox":
        module = YoloxModule.from_pretrained(pretrained_model_name_or_path, config, device)
        processor = YoloxProcessor(config or str(pretrained_model_name_or_path))
        return cls(module, processor)

    def __call__(self, inputs: Iterable, threshold: float = 0.5) -> list[Detections]:
        if isinstance(inputs, torch.Tensor):
            return self.module(inputs)  # deprecated call pattern, as in the reference
        from PIL import Image

        images = [im if isinstance(im, Image.Image) else Image.open(im) for im in inputs]
        # processor + module of the reference (yolox.py:47-52) with the letterboxed batch
        # kept as uint8 NHWC on the device (bit-identical values, a quarter of the bytes)
        batch = self.processor.images_to_device(images, "u8_nhwc")
        output = self.module.forward_nhwc(batch)
        return self.processor.postprocess(images, output, threshold=threshold)
