"""YoloxProcessor and Detections (reference yolox/models/processor.py:13-60).

Pre-processing (letterbox, ``ValTransform`` / ``preproc``, data_augment.py:140-156)
runs as ONE ``yxh_letterbox_batch`` HIP launch per batch: the images are packed into a
reused pinned host buffer, cross PCIe in one copy, and the kernel writes the float32
NCHW tensor the reference returns (on the ROCm device instead of the CPU) -- or, for
``Yolox.__call__``, uint8 NHWC that the fused Focus+stem conv reads directly.
Post-processing calls the on-device ``utils.postprocess`` and then builds the Python
result lists exactly as the reference does, on the host: boxes divided by the
letterbox ratio (fp32 CPU division, processor.py:49), scores as the Python-double
product of the fp32 obj and class confidences (processor.py:50), integer labels.
"""
from __future__ import annotations

import threading
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


_FORMATS = {"f32_nchw": N.LB_F32_NCHW, "u8_nhwc": N.LB_U8_NHWC, "bf16_nhwc": N.LB_BF16_NHWC}


class _Staging:
    """Pinned host staging buffer, reused across calls (pinning per call costs more
    than the copy).  Before a refill, the event recorded after the previous H2D copy
    guarantees that copy has drained."""

    def __init__(self):
        self.buf = None
        self.event = None
        self.lock = threading.Lock()

    def get(self, nbytes: int) -> torch.Tensor:
        if self.event is not None:
            self.event.synchronize()
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(max(nbytes, 1 << 20) * 5 // 4, dtype=torch.uint8, pin_memory=True)
        return self.buf


_staging = _Staging()


def _as_image_array(a: np.ndarray) -> np.ndarray:
    # preproc (data_augment.py:140-156) only works for H x W x 3 uint8 arrays: a 2-D (L
    # mode) array fails its CHW transpose and a 4-channel one its paste, both ValueError
    if a.ndim != 3 or a.shape[2] != 3 or a.dtype != np.uint8:
        raise ValueError(f"expected H x W x 3 uint8 RGB images, got shape {a.shape} dtype {a.dtype}")
    if a.shape[0] <= 0 or a.shape[1] <= 0:
        raise ValueError(f"empty image {a.shape}")
    return a


def letterbox_batch(arrays: list[np.ndarray], size: tuple[int, int], out_format: str = "f32_nchw",
                    device=None) -> torch.Tensor:
    """uint8 HWC RGB arrays -> the letterboxed batch on the device, in one launch:
    ``f32_nchw`` [B,3,H,W] float32 (the reference's tensor), ``u8_nhwc`` / ``bf16_nhwc``
    [B,H,W,3].  Asynchronous on the current stream."""
    device = device or _device()
    th, tw = int(size[0]), int(size[1])
    fmt = _FORMATS[out_format]
    B = len(arrays)
    shape = (B, 3, th, tw) if fmt == N.LB_F32_NCHW else (B, th, tw, 3)
    dtype = {N.LB_F32_NCHW: torch.float32, N.LB_U8_NHWC: torch.uint8, N.LB_BF16_NHWC: torch.bfloat16}[fmt]
    out = torch.empty(shape, dtype=dtype, device=device)
    if B == 0:
        return out
    arrays = [_as_image_array(a) for a in arrays]
    for a in arrays:
        r = min(th / a.shape[0], tw / a.shape[1])
        if int(a.shape[1] * r) <= 0 or int(a.shape[0] * r) <= 0:
            raise ValueError(f"image {a.shape[:2]} resizes to nothing at {size}")
    offs, off = [], 0
    for a in arrays:
        offs.append(off)
        off += (a.nbytes + 15) // 16 * 16
    desc_off = off
    total = desc_off + 16 * B
    with _staging.lock:
        host = _staging.get(total)
        hn = host.numpy()
        for a, o in zip(arrays, offs):
            hn[o:o + a.nbytes] = a.reshape(-1) if a.flags.c_contiguous else np.ascontiguousarray(a).reshape(-1)
        desc = np.zeros(B, dtype=[("off", "<i8"), ("h", "<i4"), ("w", "<i4")])
        desc["off"] = offs
        desc["h"] = [a.shape[0] for a in arrays]
        desc["w"] = [a.shape[1] for a in arrays]
        hn[desc_off:total] = desc.view(np.uint8)
        dev = torch.empty(total, dtype=torch.uint8, device=device)
        dev.copy_(host[:total], non_blocking=True)
        _staging.event = torch.cuda.Event()
        _staging.event.record(torch.cuda.current_stream(device))
    N.check(N.lib().yxh_letterbox_batch(dev.data_ptr(), dev.data_ptr() + desc_off, B, th, tw, fmt, out.data_ptr(),
                                        N.stream_ptr(device)), "letterbox")
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
        return self.images_to_device(inputs, "f32_nchw")

    def images_to_device(self, inputs: Iterable, out_format: str = "f32_nchw") -> torch.Tensor:
        """processor.py:30-37 (np.array of each image as-is, like the reference)."""
        return letterbox_batch([np.asarray(im) for im in inputs], tuple(self.config.test_size), out_format)

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
            rows = det.cpu()
            boxes = rows[:, :4] / ratio  # CPU fp32 divide, as the reference's CPU tensors
            results.append(Detections(
                bboxes=[tuple(b.tolist()) for b in boxes],
                scores=[r[4].item() * r[5].item() for r in rows],
                labels=[int(r[6]) for r in rows]))
        return results
