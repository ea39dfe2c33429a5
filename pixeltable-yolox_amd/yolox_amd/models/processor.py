"""YoloxProcessor and Detections (reference yolox/models/processor.py:13-60).

Pre-processing (letterbox) runs as the yxh_letterbox HIP kernel per image; the
batch tensor is float32 [B, 3, H, W] on the ROCm device (the reference returns the
same tensor on the CPU).  Post-processing calls the on-device ``utils.postprocess``
and then builds the Python result lists exactly as the reference does: boxes
divided by the letterbox ratio in fp32, scores as the Python-double product of the
fp32 obj and class confidences (processor.py:50), integer labels.
"""
from __future__ import annotations

from typing import Iterable, TypedDict, Union

import numpy as np
import torch

from .. import _native as N
from ..config import YoloxConfig


class Detections(TypedDict):
    bboxes: list[tuple[float, float, float, float]]
    scores: list[float]
    labels: list[int]


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("yolox_amd pre/post-processing needs a ROCm device")
    return torch.device("cuda", torch.cuda.current_device())


def letterbox_batch(arrays: list[np.ndarray], size: tuple[int, int], out_nchw: bool = True,
                    device=None) -> torch.Tensor:
    """uint8 HWC RGB arrays -> [B,3,H,W] float32 (or [B,H,W,3] uint8) on device."""
    device = device or _device()
    th, tw = size
    B = len(arrays)
    out = (torch.empty(B, 3, th, tw, dtype=torch.float32, device=device) if out_nchw
           else torch.empty(B, th, tw, 3, dtype=torch.uint8, device=device))
    L, st = N.lib(), N.stream_ptr(device)
    srcs = []
    for i, a in enumerate(arrays):
        if a.ndim == 2:
            a = np.repeat(a[:, :, None], 3, axis=2)
        if a.ndim != 3 or a.shape[2] != 3 or a.dtype != np.uint8:
            raise ValueError(f"expected HxWx3 uint8 RGB images, got {a.shape} {a.dtype}")
        src = torch.from_numpy(np.ascontiguousarray(a)).to(device, non_blocking=True)
        srcs.append(src)
        N.check(L.yxh_letterbox(src.data_ptr(), a.shape[0], a.shape[1], th, tw, int(out_nchw),
                                out[i].data_ptr(), st), "letterbox")
    torch.cuda.current_stream(device).synchronize() if srcs else None
    return out


class YoloxProcessor:
    config: YoloxConfig

    def __init__(self, model_name_or_config: Union[str, YoloxConfig]):
        if isinstance(model_name_or_config, str):
            self.config = YoloxConfig.get_named_config(model_name_or_config)
        elif isinstance(model_name_or_config, YoloxConfig):
            self.config = model_name_or_config
        else:
            raise ValueError("model_name_or_config must be a string or YoloxConfig")

    def __call__(self, inputs: Iterable) -> torch.Tensor:
        arrays = [np.array(im.convert("RGB") if getattr(im, "mode", "RGB") not in ("RGB", "L") else im)
                  for im in inputs]
        return letterbox_batch(arrays, tuple(self.config.test_size), out_nchw=True)

    def postprocess(self, images: Iterable, tensor: torch.Tensor, threshold: float = 0.5) -> list[Detections]:
        from ..utils.boxes import postprocess

        outputs = postprocess(tensor, self.config.num_classes, threshold, self.config.nmsthre,
                              class_agnostic=False)
        results: list[Detections] = []
        th, tw = self.config.test_size
        for i, image in enumerate(images):
            ratio = min(th / image.height, tw / image.width)
            det = outputs[i]
            if det is None:
                results.append(Detections(bboxes=[], scores=[], labels=[]))
                continue
            boxes = (det[:, :4] / ratio).cpu()
            rows = det.cpu()
            results.append(Detections(
                bboxes=[tuple(b.tolist()) for b in boxes],
                scores=[r[4].item() * r[5].item() for r in rows],
                labels=[int(r[6]) for r in rows]))
        return results
