"""CocoEvaluator: the reference's evaluation loop (yolox/evaluators/coco_evaluator.py:78-315) over
the HIP forward, the device NMS and the native COCOeval (``coco.coco_bbox_eval``).

evaluate() runs the model over a loader of (imgs, targets, info_imgs, ids) batches, NMS at
``confthre`` / ``nmsthre`` (utils.postprocess: device NMS, the reference's semantics), converts the
detections to COCO result dicts (coco.convert_to_coco_format), gathers them on rank 0 when
``distributed`` (each rank evaluated its own shard of the loader, as the reference's
DistributedSampler splits it) and scores them: (AP@[.5:.95], AP@.5, summary text) on rank 0,
(0, 0, None) elsewhere.  The ground truth is ``dataloader.dataset.coco``: a COCO json dict
(images / annotations / categories) or an object holding one in ``.dataset`` (pycocotools' COCO).
"""
from __future__ import annotations

import itertools
import time
from collections import ChainMap, defaultdict

import numpy as np
import torch

from .coco import COCOParams, coco_bbox_eval, convert_to_coco_format


def _table(values: dict, headers, colums: int) -> str:
    from tabulate import tabulate
    num_cols = min(colums, len(values) * len(headers))
    result_pair = [x for pair in values.items() for x in pair]
    row_pair = itertools.zip_longest(*[result_pair[i::num_cols] for i in range(num_cols)])
    return tabulate(row_pair, tablefmt="pipe", floatfmt=".3f", headers=headers * (num_cols // len(headers)),
                    numalign="left")


def per_class_AP_table(ev: dict, class_names, headers=("class", "AP"), colums=6) -> str:
    """coco_evaluator.py:52-75: mean precision over IoU thresholds and recall points, area 'all',
    the last maxDets, per class (x100)."""
    precisions = ev["precision"]
    assert len(class_names) == precisions.shape[2]
    out = {}
    for idx, name in enumerate(class_names):
        p = precisions[:, :, idx, 0, -1]
        p = p[p > -1]
        out[name] = float((np.mean(p) if p.size else float("nan")) * 100)
    return _table(out, list(headers), colums)


def per_class_AR_table(ev: dict, class_names, headers=("class", "AR"), colums=6) -> str:
    """coco_evaluator.py:29-49: mean recall over IoU thresholds, area 'all', the last maxDets."""
    recalls = ev["recall"]
    assert len(class_names) == recalls.shape[1]
    out = {}
    for idx, name in enumerate(class_names):
        r = recalls[:, idx, 0, -1]
        r = r[r > -1]
        out[name] = float((np.mean(r) if r.size else float("nan")) * 100)
    return _table(out, list(headers), colums)


def summary_text(stats: np.ndarray, params: COCOParams | None = None) -> str:
    """COCOeval.summarize()'s printed table (pycocotools' format) for the 12 statistics."""
    p = params or COCOParams()
    md = sorted(p.maxDets)
    rows = [(1, None, "all", md[2]), (1, .5, "all", md[2]), (1, .75, "all", md[2]), (1, None, "small", md[2]),
            (1, None, "medium", md[2]), (1, None, "large", md[2]), (0, None, "all", md[0]), (0, None, "all", md[1]),
            (0, None, "all", md[2]), (0, None, "small", md[2]), (0, None, "medium", md[2]), (0, None, "large", md[2])]
    lines = []
    for s, (ap, thr, area, m) in zip(stats, rows):
        title, typ = ("Average Precision", "(AP)") if ap else ("Average Recall", "(AR)")
        iou = f"{p.iouThrs[0]:0.2f}:{p.iouThrs[-1]:0.2f}" if thr is None else f"{thr:0.2f}"
        lines.append(f" {title:<18} {typ} @[ IoU={iou:<9} | area={area:>6s} | maxDets={m:>3d} ] = {s:0.3f}")
    return "\n".join(lines) + "\n"


def _is_main_process() -> bool:
    return not (torch.distributed.is_available() and torch.distributed.is_initialized()) or \
        torch.distributed.get_rank() == 0


def _gather(obj):
    """Every rank's object, in rank order (the reference's utils.gather to rank 0)."""
    out = [None] * torch.distributed.get_world_size()
    torch.distributed.all_gather_object(out, obj)
    return out


_LEGACY_MEAN = (0.485, 0.456, 0.406)
_LEGACY_STD = (0.229, 0.224, 0.225)


def legacy_normalize(imgs: torch.Tensor) -> torch.Tensor:
    """ValTransform(legacy=True) after the letterbox (data_augment.py:236-240): BGR -> RGB, / 255,
    - mean, / std over a float32 [B, 3, H, W] batch, rounded as numpy rounds the reference's
    in-place ops: ``img /= 255.0`` in float32 (a Python scalar), then ``img -= mean`` and
    ``img /= std`` against float64 arrays, i.e. computed in float64 and stored as float32."""
    x = imgs.flip(1) / 255.0
    mean = torch.tensor(_LEGACY_MEAN, dtype=torch.float64, device=x.device).view(1, 3, 1, 1)
    std = torch.tensor(_LEGACY_STD, dtype=torch.float64, device=x.device).view(1, 3, 1, 1)
    x = (x.double() - mean).float()
    return (x.double() / std).float()


class EvalLoader:
    """The evaluation loader (config.py:350-382): batches of ``dataset.pull_item`` images
    letterboxed on the device to ``size`` (yxh_letterbox_batch: preproc / ValTransform,
    data_augment.py:140-156 + 257-264) as (imgs [B, 3, H, W] fp32, targets, (heights, widths),
    ids); rank ``rank`` of ``world`` reads items rank, rank + world, ...  ``legacy``: the
    ValTransform(legacy=True) normalisation of old checkpoints (``legacy_normalize``)."""

    def __init__(self, dataset, batch_size: int, size, rank: int = 0, world: int = 1, legacy: bool = False):
        self.dataset = dataset
        self.batch_size = max(1, int(batch_size))
        self.size = tuple(size)
        self.indices = list(range(rank, len(dataset), world))
        self.legacy = bool(legacy)

    def __len__(self) -> int:
        return (len(self.indices) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        from ..models.processor import letterbox_batch
        for k in range(0, len(self.indices), self.batch_size):
            items = [self.dataset.pull_item(i) for i in self.indices[k:k + self.batch_size]]
            imgs = letterbox_batch([it[0] for it in items], self.size)
            if self.legacy:
                imgs = legacy_normalize(imgs)
            targets = [it[1] for it in items]
            info = ([int(it[2][0]) for it in items], [int(it[2][1]) for it in items])
            yield imgs, targets, info, [int(it[3]) for it in items]


class CocoEvaluator:
    """coco_evaluator.py:78-113: COCO AP evaluation of a model over a loader."""

    def __init__(self, dataloader, img_size, confthre: float, nmsthre: float, num_classes: int,
                 testdev: bool = False, per_class_AP: bool = True, per_class_AR: bool = True):
        self.dataloader = dataloader
        self.img_size = img_size if isinstance(img_size, (tuple, list)) else (img_size, img_size)
        self.confthre = confthre
        self.nmsthre = nmsthre
        self.num_classes = num_classes
        self.testdev = testdev
        self.per_class_AP = per_class_AP
        self.per_class_AR = per_class_AR

    def evaluate(self, model, distributed: bool = False, half: bool = False, trt_file=None, decoder=None,
                 test_size=None, return_outputs: bool = False):
        """coco_evaluator.py:114-203.  Returns (ap50_95, ap50, summary) on rank 0."""
        from ..utils import postprocess
        if trt_file is not None:
            raise NotImplementedError("TensorRT engines are not part of the HIP path")
        model = model.eval()
        if half:
            model = model.half()
        dtype = next(model.parameters()).dtype
        data_list, output_data = [], {}
        inference_time = nms_time = 0.0
        n_samples = max(len(self.dataloader) - 1, 1)
        for cur_iter, (imgs, _, info_imgs, ids) in enumerate(self.dataloader):
            with torch.no_grad():
                imgs = torch.as_tensor(imgs).to(next(model.parameters()).device, dtype)
                # the last batch may be short: it is not timed (the reference's rule)
                is_time_record = cur_iter < len(self.dataloader) - 1
                if is_time_record:
                    torch.cuda.synchronize()
                    start = time.time()
                outputs = model(imgs)
                if decoder is not None:
                    outputs = decoder(outputs, dtype=outputs.type())
                if is_time_record:
                    torch.cuda.synchronize()
                    infer_end = time.time()
                    inference_time += infer_end - start
                outputs = postprocess(outputs.float(), self.num_classes, self.confthre, self.nmsthre)
                if is_time_record:
                    torch.cuda.synchronize()
                    nms_time += time.time() - infer_end
            elems, per_image = self.convert_to_coco_format(outputs, info_imgs, ids, return_outputs=True)
            data_list.extend(elems)
            output_data.update(per_image)
        statistics = [inference_time, nms_time, float(n_samples)]
        if distributed:
            # each rank evaluated its shard; rank 0 scores the union (utils.gather + reduce)
            data_list = list(itertools.chain(*_gather(data_list)))
            output_data = dict(ChainMap(*_gather(output_data)))
            statistics = [float(sum(v)) for v in zip(*_gather(statistics))]
        eval_results = self.evaluate_prediction(data_list, statistics)
        if distributed:
            torch.distributed.barrier()
        if return_outputs:
            return eval_results, output_data
        return eval_results

    def convert_to_coco_format(self, outputs, info_imgs, ids, return_outputs: bool = False):
        """coco_evaluator.py:205-251: rows -> COCO result dicts (and the per-image boxes /
        scores / categories the reference returns with return_outputs)."""
        class_ids = self.dataloader.dataset.class_ids
        data_list = convert_to_coco_format(outputs, info_imgs, ids, self.img_size, class_ids)
        if not return_outputs:
            return data_list
        image_wise = defaultdict(dict)
        for output, img_h, img_w, img_id in zip(outputs, info_imgs[0], info_imgs[1], ids):
            if output is None:
                continue
            out = torch.as_tensor(output).cpu()
            scale = min(self.img_size[0] / float(img_h), self.img_size[1] / float(img_w))
            bboxes = out[:, 0:4] / scale
            scores = out[:, 4] * out[:, 5]
            image_wise[int(img_id)] = {"bboxes": [b.numpy().tolist() for b in bboxes],
                                       "scores": [s.numpy().item() for s in scores],
                                       "categories": [class_ids[int(c)] for c in out[:, 6]]}
        return data_list, image_wise

    def _ground_truth(self) -> dict:
        coco = self.dataloader.dataset.coco
        return coco if isinstance(coco, dict) else coco.dataset

    def evaluate_prediction(self, data_dict, statistics):
        """coco_evaluator.py:253-315: time info + COCOeval(bbox) summary (+ per-class tables)."""
        if not _is_main_process():
            return 0, 0, None
        inference_time, nms_time, n_samples = statistics
        bs = self.dataloader.batch_size
        a_infer_time = 1000 * inference_time / (n_samples * bs)
        a_nms_time = 1000 * nms_time / (n_samples * bs)
        info = ", ".join("Average {} time: {:.2f} ms".format(k, v) for k, v in
                         zip(["forward", "NMS", "inference"], [a_infer_time, a_nms_time, a_infer_time + a_nms_time]))
        info += "\n"
        if len(data_dict) == 0:
            return 0, 0, info
        gt = self._ground_truth()
        if self.testdev:
            import json
            json.dump(data_dict, open("./yolox_testdev_2017.json", "w"))
        ev = coco_bbox_eval(gt, data_dict)
        info += summary_text(ev["stats"])
        cats = {int(c["id"]): c["name"] for c in gt["categories"]}
        cat_names = [cats[c] for c in sorted(cats)]
        if self.per_class_AP:
            info += "per class AP:\n" + per_class_AP_table(ev, cat_names) + "\n"
        if self.per_class_AR:
            info += "per class AR:\n" + per_class_AR_table(ev, cat_names) + "\n"
        return float(ev["stats"][0]), float(ev["stats"][1]), info
