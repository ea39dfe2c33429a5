"""mAP harness (yolox_amd.evaluators, csrc/coco_map.cpp) vs the reference's own COCO
evaluator: yolox/layers/cocoeval/cocoeval.cpp compiled from the reference by
`make -C oracle ref` (oracle/_ref, build container only) and driven exactly as
CocoEvalOpt (fast_coco_eval_api.py:24-149) drives it.  pycocotools is absent; its
computeIoU / _prepare / loadRes steps are restated on the test side (numpy) to feed the
reference module.  Bar: identical precision / recall / scores arrays (bit for bit) and
summary stats; plus known answers that need no reference."""
import glob
import importlib.util
import os
import types

import numpy as np
import pytest

from conftest import REPO

REF_SO = glob.glob(os.path.join(REPO, "oracle", "_ref", "fast_cocoeval*.so"))


def ref_module():
    if not REF_SO:
        pytest.skip("oracle/_ref/fast_cocoeval not built (needs /root/reference: make -C oracle ref)")
    spec = importlib.util.spec_from_file_location("fast_cocoeval", REF_SO[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def synthetic(seed, n_img=10, cats=(1, 3, 7, 8, 20), dets_per_img=140):
    rng = np.random.default_rng(seed)
    images = [{"id": int(i)} for i in rng.choice(1000, n_img, replace=False)]
    anns, dets, aid = [], [], 1
    for im in images:
        for _ in range(int(rng.integers(0, 25))):
            x, y = rng.uniform(0, 500, 2)
            w, h = rng.uniform(2, 200, 2)
            crowd = int(rng.random() < 0.08)
            area = float(w * h * rng.uniform(0.5, 1.0))  # segmentation area, not the box's
            anns.append({"id": aid, "image_id": im["id"], "category_id": int(rng.choice(cats)),
                         "bbox": [x, y, w, h], "area": area, "iscrowd": crowd})
            aid += 1
        own = [a for a in anns if a["image_id"] == im["id"]]
        for _ in range(dets_per_img):
            if own and rng.random() < 0.6:
                a = own[int(rng.integers(len(own)))]
                bx = [v + rng.normal(0, 0.1 * max(a["bbox"][2], a["bbox"][3])) for v in a["bbox"][:2]]
                bb = bx + [max(1.0, a["bbox"][2] * rng.uniform(0.7, 1.3)), max(1.0, a["bbox"][3] * rng.uniform(0.7, 1.3))]
                c = a["category_id"] if rng.random() < 0.85 else int(rng.choice(cats))
            else:
                bb = list(rng.uniform(0, 500, 2)) + list(rng.uniform(2, 150, 2))
                c = int(rng.choice(cats))
            dets.append({"image_id": im["id"], "category_id": c, "bbox": [float(v) for v in bb],
                         "score": float(np.round(rng.random(), 2))})  # rounded: many score ties
    gt = {"images": images, "annotations": anns, "categories": [{"id": c} for c in cats]}
    return gt, dets


def bb_iou(d, g, crowd):
    """pycocotools maskApi bbIou (bbox, x y w h), double."""
    out = np.zeros((len(d), len(g)))
    for i, a in enumerate(d):
        for j, b in enumerate(g):
            w = min(a[0] + a[2], b[0] + b[2]) - max(a[0], b[0])
            if w <= 0:
                continue
            h = min(a[1] + a[3], b[1] + b[3]) - max(a[1], b[1])
            if h <= 0:
                continue
            inter = w * h
            da = a[2] * a[3]
            out[i, j] = inter / (da if crowd[j] else da + b[2] * b[3] - inter)
    return out


def reference_eval(mod, gt, dets, p):
    """CocoEvalOpt.evaluate() + accumulate() with the reference's C++ (pycocotools parts
    restated)."""
    from yolox_amd.evaluators.coco import prepare
    img_ids, cat_ids, gts, dts = prepare(gt, dets, p)
    K = len(cat_ids)
    max_det = sorted(p.maxDets)[-1]
    ious, g_inst, d_inst = [], [], []
    for i in range(len(img_ids)):
        ious.append([])
        g_inst.append([])
        d_inst.append([])
        for c in range(K):
            g, d = gts[i * K + c], dts[i * K + c]
            order = np.argsort([-x["score"] for x in d], kind="mergesort")  # computeIoU
            ds = [d[k] for k in order][:max_det]
            ious[-1].append(bb_iou([x["bbox"] for x in ds], [x["bbox"] for x in g],
                                   [int(x["iscrowd"]) for x in g]).tolist() if (g or ds) else [])
            g_inst[-1].append([mod.InstanceAnnotation(int(x["id"]), x.get("score", 0.0), x["area"],
                                                      bool(x.get("iscrowd", 0)), bool(x.get("ignore", 0))) for x in g])
            d_inst[-1].append([mod.InstanceAnnotation(int(x["id"]), x["score"], x["area"],
                                                      bool(x.get("iscrowd", 0)), bool(x.get("ignore", 0))) for x in d])
    evals = mod.COCOevalEvaluateImages(p.areaRng, max_det, p.iouThrs, ious, g_inst, d_inst)
    prm = types.SimpleNamespace(recThrs=p.recThrs, maxDets=sorted(p.maxDets), iouThrs=p.iouThrs, useCats=1,
                                catIds=cat_ids, areaRng=p.areaRng, imgIds=img_ids)
    ev = mod.COCOevalAccumulate(prm, evals)
    counts = ev["counts"]
    return {"precision": np.array(ev["precision"]).reshape(counts),
            "recall": np.array(ev["recall"]).reshape(counts[:1] + counts[2:]),
            "scores": np.array(ev["scores"]).reshape(counts)}


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_bbox_eval_identical_to_reference_cocoeval(seed):
    from yolox_amd.evaluators import COCOParams, coco_bbox_eval, summarize
    mod = ref_module()
    gt, dets = synthetic(seed)
    p = COCOParams()
    ours = coco_bbox_eval(gt, dets, p)
    ref = reference_eval(mod, gt, dets, p)
    for k in ("precision", "recall", "scores"):
        assert ours[k].shape == ref[k].shape
        np.testing.assert_array_equal(ours[k], ref[k], err_msg=k)
    np.testing.assert_array_equal(ours["stats"], summarize(ref, p))
    assert 0.0 < ours["stats"][0] < 1.0


def test_bbox_eval_other_settings_identical_to_reference():
    """Non-default max-dets (cut below the per-image detection count) and two IoU thresholds."""
    from yolox_amd.evaluators import COCOParams, coco_bbox_eval
    mod = ref_module()
    gt, dets = synthetic(5, n_img=6, dets_per_img=60)
    p = COCOParams(iouThrs=np.array([0.3, 0.5]), maxDets=[5, 20, 50])
    ours = coco_bbox_eval(gt, dets, p)
    ref = reference_eval(mod, gt, dets, p)
    for k in ("precision", "recall", "scores"):
        np.testing.assert_array_equal(ours[k], ref[k], err_msg=k)


def test_known_answers():
    """Perfect detections give AP = AR = 1 on every populated setting; a lone false
    positive ranked first caps precision; crowd GTs neither count nor penalise."""
    from yolox_amd.evaluators import coco_bbox_eval
    gt = {"images": [{"id": 1}, {"id": 2}], "categories": [{"id": 5}],
          "annotations": [{"id": 1, "image_id": 1, "category_id": 5, "bbox": [10, 10, 100, 100], "area": 10000,
                           "iscrowd": 0},
                          {"id": 2, "image_id": 2, "category_id": 5, "bbox": [50, 50, 20, 20], "area": 400,
                           "iscrowd": 0},
                          {"id": 3, "image_id": 2, "category_id": 5, "bbox": [200, 200, 50, 50], "area": 2500,
                           "iscrowd": 1}]}
    perfect = [{"image_id": a["image_id"], "category_id": 5, "bbox": a["bbox"], "score": 0.9}
               for a in gt["annotations"] if not a["iscrowd"]]
    ev = coco_bbox_eval(gt, perfect)
    assert ev["stats"][0] == 1.0 and ev["stats"][1] == 1.0 and ev["stats"][8] == 1.0
    on_crowd = perfect + [{"image_id": 2, "category_id": 5, "bbox": [205, 205, 40, 40], "score": 0.95}]
    assert coco_bbox_eval(gt, on_crowd)["stats"][0] == 1.0  # matched to the crowd: ignored
    fp = perfect + [{"image_id": 1, "category_id": 5, "bbox": [400, 400, 30, 30], "score": 0.99}]
    ev = coco_bbox_eval(gt, fp)
    assert ev["precision"][0, 0, 0, 0, 2] == pytest.approx(2 / 3)  # monotone envelope at recall 0
    assert ev["stats"][0] < 1.0
    with pytest.raises(ValueError):
        coco_bbox_eval(gt, [{"image_id": 99, "category_id": 5, "bbox": [0, 0, 1, 1], "score": 1.0}])


def test_convert_to_coco_format():
    """coco_evaluator.py:205-251: boxes / scale, xyxy -> xywh, score = obj * cls (fp32),
    dataset class ids, None images skipped."""
    import torch

    from yolox_amd.evaluators import convert_to_coco_format
    rows = torch.tensor([[10.0, 20.0, 110.0, 60.0, 0.9, 0.5, 2.0], [0.0, 0.0, 64.0, 32.0, 0.8, 0.25, 0.0]])
    out = convert_to_coco_format([rows, None], ([320, 100], [640, 100]), [7, 8], (640, 640), [1, 2, 3])
    assert len(out) == 2 and {o["image_id"] for o in out} == {7}
    assert out[0]["category_id"] == 3 and out[1]["category_id"] == 1
    np.testing.assert_allclose(out[0]["bbox"], [10.0, 20.0, 100.0, 40.0])
    assert out[0]["score"] == float(torch.tensor(0.9) * torch.tensor(0.5))
