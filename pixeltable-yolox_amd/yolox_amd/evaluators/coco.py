"""COCO box-mAP harness: the reference's evaluation path without pycocotools.

* ``convert_to_coco_format`` -- CocoEvaluator.convert_to_coco_format
  (yolox/evaluators/coco_evaluator.py:205-251): postprocess rows -> COCO result dicts
  (boxes / letterbox scale, xyxy -> xywh, score = obj * cls in fp32, dataset class ids).
* ``coco_bbox_eval`` -- COCOeval(bbox) as CocoEvalOpt runs it (yolox/layers/
  fast_coco_eval_api.py:24-149): pycocotools' _prepare / loadRes bookkeeping restated
  here, IoU + EvaluateImages + Accumulate in one host C++ call (``yxh_coco_eval``,
  csrc/coco_map.cpp).  Returns CocoEvalOpt.eval's arrays and the 12 summary stats.
* ``summarize`` -- COCOeval.summarize's statistics (stats[0] = AP@[.5:.95] and stats[1]
  = AP@.5 are what CocoEvaluator.evaluate reports).

EvaluateImages / Accumulate are pinned to the reference's own cocoeval.cpp (compiled from
the reference by ``make -C oracle ref``; tests/test_coco_map.py).  pycocotools itself is
absent: its bookkeeping (ignore = iscrowd for bbox, detection area = w*h, ids 1..N,
sorted unique image / category ids) is restated and checked by known-answer cases.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from .. import _native as N


@dataclass
class COCOParams:
    """pycocotools Params(iouType='bbox') defaults."""
    iouThrs: np.ndarray = field(default_factory=lambda: np.linspace(
        .5, 0.95, int(np.round((0.95 - .5) / .05)) + 1, endpoint=True))
    recThrs: np.ndarray = field(default_factory=lambda: np.linspace(
        .0, 1.00, int(np.round((1.00 - .0) / .01)) + 1, endpoint=True))
    maxDets: list = field(default_factory=lambda: [1, 10, 100])
    areaRng: list = field(default_factory=lambda: [[0 ** 2, 1e5 ** 2], [0 ** 2, 32 ** 2], [32 ** 2, 96 ** 2],
                                                   [96 ** 2, 1e5 ** 2]])
    areaRngLbl: list = field(default_factory=lambda: ["all", "small", "medium", "large"])
    imgIds: Optional[list] = None
    catIds: Optional[list] = None
    useCats: int = 1


def convert_to_coco_format(outputs, info_imgs, ids, img_size, class_ids) -> list:
    """coco_evaluator.py:205-251.  outputs: per image [N, 7] rows (x1, y1, x2, y2, obj,
    cls_conf, cls_idx) or None (utils.postprocess); info_imgs = (heights, widths)."""
    import torch
    data = []
    for output, img_h, img_w, img_id in zip(outputs, info_imgs[0], info_imgs[1], ids):
        if output is None:
            continue
        output = torch.as_tensor(output).cpu()
        bboxes = output[:, 0:4].clone()
        scale = min(img_size[0] / float(img_h), img_size[1] / float(img_w))
        bboxes /= scale
        cls = output[:, 6]
        scores = output[:, 4] * output[:, 5]
        bboxes[:, 2] = bboxes[:, 2] - bboxes[:, 0]  # xyxy2xywh
        bboxes[:, 3] = bboxes[:, 3] - bboxes[:, 1]
        for ind in range(bboxes.shape[0]):
            data.append({"image_id": int(img_id), "category_id": class_ids[int(cls[ind])],
                         "bbox": bboxes[ind].numpy().tolist(), "score": scores[ind].numpy().item(),
                         "segmentation": []})
    return data


def _instances(rows: Sequence[dict], is_det: bool) -> "C.Array":
    arr = (N.CocoInstance * max(1, len(rows)))()
    for i, r in enumerate(rows):
        o = arr[i]
        o.id = int(r["id"])
        o.score = float(r["score"]) if is_det else float(r.get("score", 0.0))
        o.area = float(r["area"])
        for k in range(4):
            o.box[k] = float(r["bbox"][k])
        o.is_crowd = int(bool(r.get("iscrowd", 0)))
        o.ignore = int(bool(r.get("ignore", 0)))
    return arr


def prepare(gt: dict, dets: list, params: Optional[COCOParams] = None):
    """pycocotools COCO / loadRes / COCOeval._prepare (bbox): per (image, category) cells
    of ground truths (annotation order) and detections (result order, ids 1..N)."""
    p = params or COCOParams()
    img_ids = sorted({int(im["id"]) for im in gt["images"]}) if p.imgIds is None else list(p.imgIds)
    cat_ids = sorted({int(c["id"]) for c in gt["categories"]}) if p.catIds is None else list(p.catIds)
    img_ids = [int(v) for v in np.unique(img_ids)]
    cat_ids = [int(v) for v in np.unique(cat_ids)]
    if not p.useCats:
        raise NotImplementedError("useCats=0")
    known = {int(im["id"]) for im in gt["images"]}
    if any(int(d["image_id"]) not in known for d in dets):
        raise ValueError("Results do not correspond to current coco set")  # loadRes assertion
    ii = {v: i for i, v in enumerate(img_ids)}
    ci = {v: i for i, v in enumerate(cat_ids)}
    K = len(cat_ids)
    gts = [[] for _ in range(len(img_ids) * K)]
    for a in gt["annotations"]:
        i, c = ii.get(int(a["image_id"])), ci.get(int(a["category_id"]))
        if i is None or c is None:
            continue
        a = dict(a)
        a["ignore"] = bool(a.get("iscrowd", 0))  # _prepare: ignore <- iscrowd (bbox)
        gts[i * K + c].append(a)
    dts = [[] for _ in range(len(img_ids) * K)]
    for n, d in enumerate(dets):
        i, c = ii.get(int(d["image_id"])), ci.get(int(d["category_id"]))
        bb = d["bbox"]
        r = {"id": n + 1, "score": d["score"], "area": bb[2] * bb[3], "bbox": bb, "iscrowd": 0}  # loadRes
        if i is not None and c is not None:
            dts[i * K + c].append(r)
    return img_ids, cat_ids, gts, dts


def coco_bbox_eval(gt: dict, dets: list, params: Optional[COCOParams] = None) -> dict:
    """COCOeval(bbox).evaluate() + accumulate() + summarize() (CocoEvalOpt's arrays)."""
    p = params or COCOParams()
    img_ids, cat_ids, gts, dts = prepare(gt, dets, p)
    I, K = len(img_ids), len(cat_ids)
    gt_off = np.zeros(I * K + 1, np.int64)
    dt_off = np.zeros(I * K + 1, np.int64)
    gt_off[1:] = np.cumsum([len(c) for c in gts])
    dt_off[1:] = np.cumsum([len(c) for c in dts])
    g_arr = _instances([r for c in gts for r in c], False)
    d_arr = _instances([r for c in dts for r in c], True)
    max_dets = sorted(int(m) for m in p.maxDets)
    area = np.ascontiguousarray(np.asarray(p.areaRng, np.float64).reshape(-1, 2))
    iou_thr = np.ascontiguousarray(p.iouThrs, np.float64)
    rec_thr = np.ascontiguousarray(p.recThrs, np.float64)
    md = np.asarray(max_dets, np.int32)
    T, R, A, M = len(iou_thr), len(rec_thr), len(area), len(md)
    prm = N.CocoParams(I, K, A, T, R, M, area.ctypes.data, iou_thr.ctypes.data, rec_thr.ctypes.data, md.ctypes.data)
    precision = np.empty((T, R, K, A, M), np.float64)
    scores = np.empty((T, R, K, A, M), np.float64)
    recall = np.empty((T, K, A, M), np.float64)
    N.check(N.lib().yxh_coco_eval(C.byref(prm), C.addressof(g_arr), gt_off.ctypes.data, C.addressof(d_arr),
                                  dt_off.ctypes.data, precision.ctypes.data, recall.ctypes.data, scores.ctypes.data),
            "coco_eval")
    ev = {"counts": [T, R, K, A, M], "precision": precision, "recall": recall, "scores": scores,
          "imgIds": img_ids, "catIds": cat_ids}
    ev["stats"] = summarize(ev, p)
    return ev


def summarize(ev: dict, params: Optional[COCOParams] = None) -> np.ndarray:
    """COCOeval.summarize() statistics (12 numbers, -1 where nothing is valid)."""
    p = params or COCOParams()
    max_dets = sorted(p.maxDets)
    iou_thrs = np.asarray(p.iouThrs)

    def one(ap: bool, iou_thr=None, area="all", md=100):
        aind = [i for i, lbl in enumerate(p.areaRngLbl) if lbl == area]
        mind = [i for i, m in enumerate(max_dets) if m == md]
        s = ev["precision"] if ap else ev["recall"]
        if iou_thr is not None:
            s = s[np.where(iou_thr == iou_thrs)[0]]
        s = s[:, :, :, aind, mind] if ap else s[:, :, aind, mind]
        return -1.0 if len(s[s > -1]) == 0 else float(np.mean(s[s > -1]))

    m2 = max_dets[2]
    return np.array([
        one(True), one(True, .5, md=m2), one(True, .75, md=m2),
        one(True, area="small", md=m2), one(True, area="medium", md=m2), one(True, area="large", md=m2),
        one(False, md=max_dets[0]), one(False, md=max_dets[1]), one(False, md=m2),
        one(False, area="small", md=m2), one(False, area="medium", md=m2), one(False, area="large", md=m2)])
