"""Deterministic synthetic weights for YOLOX state_dicts.

There is no network in this environment, so the MegVii `.pth` checkpoints that
`YoloxModule.from_pretrained` downloads (reference `yolox/models/yolox.py:122-131`)
are unavailable.  Parity fixtures, tests and the benchmark therefore run on seeded
random weights:

* conv / pred weights and BN affine parameters are drawn from a generator seeded by
  ``(seed, crc32(key))`` -- independent of state_dict ordering, so the fixture
  script (building the reference's module tree) and this package's own module tree
  obtain bit-identical tensors from the same seed;
* BN ``running_mean`` / ``running_var`` are *calibrated*: set to the per-channel
  statistics of each BN's input on a synthetic batch, as a trained network's BN
  would be (a random, uncalibrated 80-layer SiLU stack either collapses or
  overflows).  The calibrated tables are small (23k floats for yolox_s) and ship as
  ``data/bn_stats_<model>.npz``; ``tests/golden/make_golden.py`` produced them on
  the reference model.
"""
from __future__ import annotations

import math
import os
import zlib
from typing import Mapping, Optional, Sequence

import numpy as np
import torch

__all__ = ["synthetic_state_dict", "synthetic_images", "load_bn_stats", "DATA_DIR"]

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.default_rng([int(seed) & 0xFFFFFFFF, zlib.crc32(key.encode())])


def _is_bn(key: str) -> bool:
    return ".bn." in key or key.startswith("bn.")


def _tensor_for(key: str, shape: Sequence[int], seed: int) -> torch.Tensor:
    rng = _rng(seed, key)
    shape = tuple(int(s) for s in shape)
    leaf = key.rsplit(".", 1)[-1]
    is_pred = any(p in key for p in ("cls_preds", "reg_preds", "obj_preds"))
    if leaf == "num_batches_tracked":
        return torch.zeros(shape, dtype=torch.int64)
    if leaf == "running_mean":
        a = np.zeros(shape)
    elif leaf == "running_var":
        a = np.ones(shape)
    elif _is_bn(key) and leaf == "weight":
        # small gamma + positive beta keep the SiLUs near their linear range: a
        # random BN network at init is otherwise on the chaotic side (relative
        # perturbations grow ~7%/layer, so bf16 rounding of the weights alone would
        # flip detections); this one is ordered like a trained net.
        a = rng.uniform(0.4, 0.8, shape)
    elif _is_bn(key) and leaf == "bias":
        a = rng.normal(1.0, 0.5, shape)
    elif is_pred and leaf == "weight":
        fan_in = int(np.prod(shape[1:]))
        gain = 0.08 if "reg_preds" in key else 4.0
        a = rng.normal(0.0, gain / math.sqrt(fan_in), shape)
    elif is_pred and leaf == "bias":
        if "cls_preds" in key:
            a = rng.normal(-2.0, 1.5, shape)
        elif "obj_preds" in key:
            a = rng.normal(0.0, 1.0, shape)
        else:
            a = rng.normal(0.0, 0.2, shape)
    elif len(shape) == 4:
        fan_in = int(np.prod(shape[1:]))
        a = rng.normal(0.0, 1.0 / math.sqrt(fan_in), shape)
    else:
        a = rng.normal(0.0, 0.1, shape)
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))


def load_bn_stats(model_name: str) -> dict[str, torch.Tensor]:
    path = os.path.join(DATA_DIR, f"bn_stats_{model_name}.npz")
    with np.load(path) as z:
        return {k: torch.from_numpy(np.array(z[k])) for k in z.files}


def synthetic_state_dict(
    shapes: Mapping[str, Sequence[int]] | Mapping[str, torch.Tensor],
    seed: int = 0,
    bn_stats: Optional[Mapping[str, torch.Tensor] | str] = None,
) -> dict[str, torch.Tensor]:
    """Return a state_dict with the given keys/shapes filled deterministically.

    ``bn_stats`` is a mapping of running_mean/running_var tensors (or a model
    name whose shipped table is loaded); its keys override the identity
    statistics used otherwise.
    """
    if isinstance(bn_stats, str):
        bn_stats = load_bn_stats(bn_stats)
    out = {}
    for key, val in shapes.items():
        shape = val.shape if isinstance(val, torch.Tensor) else val
        if bn_stats is not None and key in bn_stats:
            out[key] = bn_stats[key].to(torch.float32).reshape(tuple(shape)).clone()
        else:
            out[key] = _tensor_for(key, shape, seed)
    return out


def synthetic_images(batch: int, height: int, width: int, seed: int = 0) -> np.ndarray:
    """uint8 HWC images, uniform in [0, 255] (SURVEY.md §8d synthetic inputs)."""
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(batch, height, width, 3), dtype=np.uint8)


def synthetic_labels(batch: int, height: int, width: int, max_gt: int = 50,
                     max_labels: int = 120, num_classes: int = 80, seed: int = 0) -> np.ndarray:
    """Padded COCO-shaped targets ``[B, max_labels, 5]`` = (cls, cx, cy, w, h) in pixels.

    G ~ U{1..max_gt} per image; centers inside the image margin; sizes scaled to
    the image (SURVEY.md §8d, config 3 generator).  Rows past G are zero, which is
    how the reference counts labels (`yolo_head.py:269`).
    """
    rng = np.random.default_rng(seed)
    out = np.zeros((batch, max_labels, 5), dtype=np.float32)
    s = min(height, width) / 640.0
    for b in range(batch):
        g = int(rng.integers(1, max_gt + 1))
        out[b, :g, 0] = rng.integers(0, num_classes, g)
        out[b, :g, 1] = rng.uniform(50 * s, width - 50 * s, g)
        out[b, :g, 2] = rng.uniform(50 * s, height - 50 * s, g)
        out[b, :g, 3] = rng.uniform(10 * s, 160 * s, g)
        out[b, :g, 4] = rng.uniform(10 * s, 160 * s, g)
    return out


def anchor_grid(height: int, width: int, strides=(8, 16, 32)):
    """(x_shifts, y_shifts, expanded_strides), each float32 ``[1, A]``, level-major,
    row-major (y then x) inside a level -- the anchor order of the reference head
    (`yolo_head.py:205-207, 213-231`)."""
    xs, ys, ss = [], [], []
    for s in strides:
        h, w = height // s, width // s
        yv, xv = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
        xs.append(xv.reshape(-1))
        ys.append(yv.reshape(-1))
        ss.append(np.full(h * w, s))
    f = lambda parts: np.concatenate(parts).astype(np.float32)[None]  # noqa: E731
    return f(xs), f(ys), f(ss)


def synthetic_head_outputs(batch: int, height: int, width: int, num_classes: int = 80,
                           seed: int = 0):
    """Synthetic training-mode head outputs for SimOTA tests.

    Returns ``bbox [B,A,4]`` (decoded cx,cy,w,h near each anchor), ``cls [B,A,C]``
    and ``obj [B,A,1]`` logits, all float32.
    """
    x_s, y_s, st = anchor_grid(height, width)
    rng = np.random.default_rng(seed)
    A = x_s.shape[1]
    cx = (x_s[0] + 0.5) * st[0] + rng.normal(0, 4, A).astype(np.float32)
    cy = (y_s[0] + 0.5) * st[0] + rng.normal(0, 4, A).astype(np.float32)
    wh = rng.uniform(8, 160, (A, 2)).astype(np.float32)
    bbox = np.stack([cx, cy, wh[:, 0], wh[:, 1]], 1)[None].repeat(batch, 0).astype(np.float32)
    cls = rng.normal(-2, 1.5, (batch, A, num_classes)).astype(np.float32)
    obj = rng.normal(0, 1.5, (batch, A, 1)).astype(np.float32)
    return bbox, cls, obj
