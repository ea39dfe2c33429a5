"""Multiscale resize of the training batch on the device (yxh_resize_bilinear, csrc/preprocess.hip).

YoloxConfig.preprocess (reference config.py:296-305) resizes every non-``input_size`` training
iteration with ``F.interpolate(inputs, size=tsize, mode="bilinear", align_corners=False)``; here the
same arithmetic runs as one HIP launch over the [B, C, H, W] batch (bit-identical to ATen's bilinear
kernel on the same device: tests/test_gpu_augment.py).  ROCm tensors only -- there is no CPU path:
a CPU batch raises (``N.require_device``) instead of silently taking another kernel.

Layout: the kernel reads contiguous NCHW.  A channels_last batch is made NCHW-contiguous first and
the result is NCHW-contiguous; bit-identity is pinned against ATen's NCHW bilinear kernel only (ATen
runs a separate NHWC kernel for channels_last input, which this module does not claim to match).
"""
from __future__ import annotations

import torch

from .. import _native as N


def resize_bilinear(x: torch.Tensor, size) -> torch.Tensor:
    """F.interpolate(x, size=size, mode="bilinear", align_corners=False) of a [B, C, H, W] float32 /
    bfloat16 / float16 tensor on a ROCm device (a new contiguous tensor of the same dtype)."""
    if x.dim() != 4:
        raise ValueError(f"resize_bilinear takes [B, C, H, W], got {tuple(x.shape)}")
    if x.dtype not in N.DTYPE_CODE or x.dtype == torch.uint8:
        raise ValueError(f"resize_bilinear: dtype {x.dtype} (float32 / bfloat16 / float16)")
    N.require_device(x, "resize_bilinear input")
    oh, ow = (int(v) for v in size)
    x = x.contiguous()
    B, C, H, W = x.shape
    out = torch.empty(B, C, oh, ow, dtype=x.dtype, device=x.device)
    N.check(N.lib().yxh_resize_bilinear(N.DTYPE_CODE[x.dtype], B, C, H, W, x.data_ptr(), oh, ow, out.data_ptr(),
                                        N.stream_ptr(x.device)), "resize_bilinear")
    return out
