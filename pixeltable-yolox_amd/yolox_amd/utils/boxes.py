"""Box utilities (reference yolox/utils/boxes.py).

``postprocess`` runs on the device through ``yxh_postprocess`` (filter, stable
score sort, torchvision nms / batched_nms).  The box-format helpers and
``bboxes_iou`` are small tensor expressions kept with the reference's exact
operation order (they are used on host-side targets, not on the hot path).
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _native as N

__all__ = ["postprocess", "postprocess_device", "bboxes_iou", "xyxy2xywh", "xyxy2cxcywh", "cxcywh2xyxy",
           "VANILLA_NUMEL_CPU", "VANILLA_NUMEL_CUDA"]

# torchvision batched_nms branch rule: boxes.numel() above this -> per-class NMS
VANILLA_NUMEL_CPU = 4000   # the reference CPU path (parity target)
VANILLA_NUMEL_CUDA = 20000

_workspaces: dict = {}
_split_next: dict = {}  # device -> the split path's next workspace slot (1 or 2)


class _Workspace:
    """One yxh_postprocess scratch buffer per (device, slot), shared by every stream: each
    call waits for the previous call's completion event on that slot (on whatever stream that
    ran) and records its own, so calls on different streams never overlap on it, and a caller
    that makes a new stream per request reuses the same buffer instead of leaking one each.

    The split path (filter on the forward stream, the rest on ``rest_stream``) alternates two
    slots: batch k+1's filter reuses the buffer of batch k-1, whose sort / mask / reduce finished
    long before, so the forward stream never waits on the NMS of the batch just before it."""

    def __init__(self):
        self.buf: Optional[torch.Tensor] = None
        self.done: Optional[torch.cuda.Event] = None

    def acquire(self, device, need: int) -> torch.Tensor:
        stream = torch.cuda.current_stream(device)
        if self.done is not None:
            stream.wait_event(self.done)
        if self.buf is None or self.buf.numel() < need:
            # zero-filled: yxh_postprocess_scored expects the candidate counters zero on entry (every
            # call leaves them so)
            self.buf = torch.zeros(need, dtype=torch.uint8, device=device)
        self.buf.record_stream(stream)  # the allocator may recycle it only after this stream's use
        return self.buf

    def release(self, device, stream: Optional[torch.cuda.Stream] = None) -> None:
        if self.done is None:
            self.done = torch.cuda.Event()
        self.done.record(stream if stream is not None else torch.cuda.current_stream(device))


def _workspace(device, B: int, A: int, split: bool = False) -> "_Workspace":
    need = int(N.lib().yxh_postprocess_workspace_bytes(B, A))
    dev = torch.device(device)
    slot = 0
    if split:
        slot = _split_next.get(dev, 1)
        _split_next[dev] = 3 - slot
    ws = _workspaces.setdefault((dev, slot), _Workspace())
    ws.acquire(device, need)
    return ws


def postprocess_device(prediction: torch.Tensor, num_classes: int, conf_thre: float = 0.7,
                       nms_thre: float = 0.45, class_agnostic: bool = False,
                       vanilla_numel: int = VANILLA_NUMEL_CPU, det: Optional[torch.Tensor] = None,
                       counts: Optional[torch.Tensor] = None, filter_done: Optional[torch.cuda.Event] = None,
                       rest_stream: Optional[torch.cuda.Stream] = None, scores: Optional[torch.Tensor] = None):
    """Asynchronous form: returns (det [B, A, 7], counts [B] int32) on the device,
    nothing synchronised, on the current stream.  ``prediction`` (fp32, on device) becomes xyxy
    in place.  ``filter_done`` is recorded once ``prediction`` is no longer read (after the
    filter pass): a producer that waits on it may overwrite ``prediction`` while the rest of
    the NMS runs.  ``rest_stream`` (needs ``filter_done``): only the filter runs on the current
    stream; the sort / mask / reduce passes run on ``rest_stream`` after it (yxh_postprocess_split),
    and det / counts are complete in that stream's order.  ``scores``: the [B, A, 8] serving records
    the forward that wrote ``prediction`` emitted (engine.Plan.enable_scores): the filter reads them
    instead of the class columns (yxh_postprocess_scored, same results)."""
    N.require_device(prediction, "prediction")
    if prediction.dtype != torch.float32 or not prediction.is_contiguous():
        raise ValueError("prediction must be a contiguous float32 [B, A, 5+C] tensor")
    B, A, D = prediction.shape
    if D != 5 + num_classes:
        raise ValueError(f"prediction has {D} columns, expected {5 + num_classes}")
    dev = prediction.device
    if det is None:
        det = torch.empty(B, max(A, 1), 7, dtype=torch.float32, device=dev)
    if counts is None:
        counts = torch.empty(B, dtype=torch.int32, device=dev)
    if rest_stream is not None and filter_done is None:
        raise ValueError("rest_stream needs a filter_done event")
    if filter_done is not None and not filter_done.cuda_event:
        filter_done.record()  # torch creates the event lazily, on its first record
    if scores is not None:
        N.require_device(scores, "scores")
        if tuple(scores.shape) != (B, A, 8) or scores.dtype != torch.float32 or not scores.is_contiguous():
            raise ValueError(f"scores must be a contiguous float32 {(B, A, 8)} tensor")
    ws = _workspace(dev, B, A, split=rest_stream is not None)
    buf = ws.buf
    try:
        if scores is not None:
            if rest_stream is not None:
                for t in (buf, det, counts):
                    t.record_stream(rest_stream)
            N.check(N.lib().yxh_postprocess_scored(
                prediction.data_ptr(), scores.data_ptr(), B, A, num_classes, float(conf_thre), float(nms_thre),
                int(bool(class_agnostic)), int(vanilla_numel), det.data_ptr(), counts.data_ptr(), buf.data_ptr(),
                buf.numel(), filter_done.cuda_event if filter_done is not None else None, N.stream_ptr(dev),
                rest_stream.cuda_stream if rest_stream is not None else None), "postprocess")
        elif filter_done is None:
            N.check(N.lib().yxh_postprocess(
                prediction.data_ptr(), B, A, num_classes, float(conf_thre), float(nms_thre),
                int(bool(class_agnostic)), int(vanilla_numel), det.data_ptr(), counts.data_ptr(), buf.data_ptr(),
                buf.numel(), N.stream_ptr(dev)), "postprocess")
        elif rest_stream is None:
            N.check(N.lib().yxh_postprocess_ev(
                prediction.data_ptr(), B, A, num_classes, float(conf_thre), float(nms_thre),
                int(bool(class_agnostic)), int(vanilla_numel), det.data_ptr(), counts.data_ptr(), buf.data_ptr(),
                buf.numel(), filter_done.cuda_event, N.stream_ptr(dev)), "postprocess")
        else:
            for t in (buf, det, counts):  # written on rest_stream: the allocator must wait for it
                t.record_stream(rest_stream)
            N.check(N.lib().yxh_postprocess_split(
                prediction.data_ptr(), B, A, num_classes, float(conf_thre), float(nms_thre),
                int(bool(class_agnostic)), int(vanilla_numel), det.data_ptr(), counts.data_ptr(), buf.data_ptr(),
                buf.numel(), filter_done.cuda_event, N.stream_ptr(dev), rest_stream.cuda_stream), "postprocess")
    finally:
        ws.release(dev, rest_stream)
    return det, counts


def postprocess(prediction: torch.Tensor, num_classes: int, conf_thre: float = 0.7, nms_thre: float = 0.45,
                class_agnostic: bool = False, vanilla_numel: int = VANILLA_NUMEL_CPU):
    """utils.postprocess (boxes.py:31-75): list of [N, 7] tensors
    (x1, y1, x2, y2, obj_conf, class_conf, class_pred) per image, or None.

    Like the reference, ``prediction[..., :4]`` is rewritten to xyxy in place.  A
    CPU tensor is processed on the device and written back.
    """
    host = not prediction.is_cuda
    pred = prediction
    if host:
        pred = prediction.to(torch.device("cuda", torch.cuda.current_device()), torch.float32).contiguous()
    elif prediction.dtype != torch.float32 or not prediction.is_contiguous():
        pred = prediction.float().contiguous()
    det, counts = postprocess_device(pred, num_classes, conf_thre, nms_thre, class_agnostic, vanilla_numel)
    if pred is not prediction:
        prediction.copy_(pred)
    n = counts.cpu().tolist()
    out = []
    for b, c in enumerate(n):
        if c == 0:
            out.append(None)
        else:
            d = det[b, :c]
            out.append(d.cpu() if host else d)
    return out


def bboxes_iou(bboxes_a: torch.Tensor, bboxes_b: torch.Tensor, xyxy: bool = True) -> torch.Tensor:
    """Pairwise IoU (boxes.py:78-101); raises IndexError unless boxes have 4 columns."""
    if bboxes_a.shape[1] != 4 or bboxes_b.shape[1] != 4:
        raise IndexError
    a, b = bboxes_a, bboxes_b
    if xyxy:
        tl = torch.max(a[:, None, :2], b[:, :2])
        br = torch.min(a[:, None, 2:], b[:, 2:])
        area_a = torch.prod(a[:, 2:] - a[:, :2], 1)
        area_b = torch.prod(b[:, 2:] - b[:, :2], 1)
    else:
        tl = torch.max(a[:, None, :2] - a[:, None, 2:] / 2, b[:, :2] - b[:, 2:] / 2)
        br = torch.min(a[:, None, :2] + a[:, None, 2:] / 2, b[:, :2] + b[:, 2:] / 2)
        area_a = torch.prod(a[:, 2:], 1)
        area_b = torch.prod(b[:, 2:], 1)
    en = (tl < br).type(tl.type()).prod(dim=2)
    area_i = torch.prod(br - tl, 2) * en
    return area_i / (area_a[:, None] + area_b - area_i)


def xyxy2xywh(bboxes):
    bboxes[:, 2] = bboxes[:, 2] - bboxes[:, 0]
    bboxes[:, 3] = bboxes[:, 3] - bboxes[:, 1]
    return bboxes


def xyxy2cxcywh(bboxes):
    bboxes[:, 2] = bboxes[:, 2] - bboxes[:, 0]
    bboxes[:, 3] = bboxes[:, 3] - bboxes[:, 1]
    bboxes[:, 0] = bboxes[:, 0] + bboxes[:, 2] * 0.5
    bboxes[:, 1] = bboxes[:, 1] + bboxes[:, 3] * 0.5
    return bboxes


def cxcywh2xyxy(bboxes):
    bboxes[:, 0] = bboxes[:, 0] - bboxes[:, 2] * 0.5
    bboxes[:, 1] = bboxes[:, 1] - bboxes[:, 3] * 0.5
    bboxes[:, 2] = bboxes[:, 0] + bboxes[:, 2]
    bboxes[:, 3] = bboxes[:, 1] + bboxes[:, 3]
    return bboxes
