"""CocoEvaluator end to end on the device (coco_evaluator.py:114-315 via config.get_evaluator):
device letterbox -> HIP forward -> device NMS -> COCO conversion -> native COCOeval.  The ground
truth is the model's own detections at the evaluation thresholds, mapped back to each image
(self-consistency: AP = AP50 = 1), then one image's boxes shifted off (AP drops)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _ValSet:
    """pull_item dataset (coco.py:131-160's contract): ragged uint8 RGB images, COCO ground truth."""
    class_ids = list(range(1, 81))

    def __init__(self, n):
        rng = np.random.default_rng(0)
        self.imgs = [rng.integers(0, 256, (int(rng.integers(300, 700)), int(rng.integers(300, 700)), 3),
                                  dtype=np.uint8) for _ in range(n)]
        self.coco = {"images": [{"id": 10 + i, "height": a.shape[0], "width": a.shape[1]}
                                for i, a in enumerate(self.imgs)],
                     "annotations": [], "categories": [{"id": c, "name": f"c{c}"} for c in self.class_ids]}

    def __len__(self):
        return len(self.imgs)

    def pull_item(self, i):
        a = self.imgs[i]
        return a, np.zeros((0, 5), np.float32), (a.shape[0], a.shape[1]), 10 + i


def test_coco_evaluator_self_consistent_ap():
    from yolox_amd.config import named_config
    from yolox_amd.models import YoloxModule
    cfg = named_config("yolox_s")
    cfg.test_conf, cfg.nmsthre = 0.65, 0.65
    model = YoloxModule.synthetic("yolox_s", seed=0, device="cuda")
    ds = _ValSet(5)
    ev = cfg.get_evaluator(batch_size=2, is_distributed=False, dataset=ds)
    (_, _, _), per_image = cfg.eval(model, ev, False, return_outputs=True)
    anns = []
    for img_id, d in per_image.items():
        for b, c in zip(d["bboxes"], d["categories"]):
            w, h = b[2] - b[0], b[3] - b[1]
            anns.append({"id": len(anns) + 1, "image_id": img_id, "category_id": c, "bbox": [b[0], b[1], w, h],
                         "area": w * h, "iscrowd": 0})
    assert len(anns) > 10
    ds.coco["annotations"] = anns
    ap, ap50, info = cfg.eval(model, cfg.get_evaluator(2, False, dataset=ds), False)
    assert ap == pytest.approx(1.0) and ap50 == pytest.approx(1.0), info
    assert "Average forward time" in info and "per class AP" in info
    for a in anns:  # image 10's ground truth moved away: its detections become false positives
        if a["image_id"] == 10:
            a["bbox"][0] += 1000.0
    ap2, _, _ = cfg.eval(model, cfg.get_evaluator(2, False, dataset=ds), False)
    assert ap2 < 1.0
