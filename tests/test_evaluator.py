"""CocoEvaluator (yolox/evaluators/coco_evaluator.py:78-315) on CPU: the evaluation loop, the COCO
conversion, rank-sharded evaluation gathered on rank 0 (gloo, world size 2) and the summary text.
The model and the device NMS are stubbed (they run on the GPU: tests/test_gpu_processor.py); the
COCOeval core is the native one (pinned to the reference's cocoeval.cpp, tests/test_coco_map.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

IMG = 64
NIMG, BS = 6, 2


def _gt_and_rows():
    """A COCO ground truth (6 images, 3 categories with ids 1, 3, 7) and, per image, the
    postprocess rows [x1, y1, x2, y2, obj, cls_conf, cls_idx] of the network input scale that
    detect every object exactly (image scale = IMG / size, letterbox ratio r)."""
    rng = np.random.default_rng(3)
    cats = [{"id": 1, "name": "a"}, {"id": 3, "name": "b"}, {"id": 7, "name": "c"}]
    images, anns, rows = [], [], {}
    for i in range(NIMG):
        h, w = int(rng.integers(40, 128)), int(rng.integers(40, 128))
        images.append({"id": 100 + i, "height": h, "width": w})
        r = min(IMG / h, IMG / w)
        rr = []
        for _ in range(int(rng.integers(1, 4))):
            x, y = float(rng.uniform(0, w / 2)), float(rng.uniform(0, h / 2))
            bw, bh = float(rng.uniform(8, w / 2)), float(rng.uniform(8, h / 2))
            c = int(rng.integers(0, 3))
            anns.append({"id": len(anns) + 1, "image_id": 100 + i, "category_id": cats[c]["id"],
                         "bbox": [x, y, bw, bh], "area": bw * bh, "iscrowd": 0})
            rr.append([x * r, y * r, (x + bw) * r, (y + bh) * r, 0.9, 0.8 + 0.01 * len(rr), c])
        rows[100 + i] = torch.tensor(rr, dtype=torch.float32)
    return {"images": images, "annotations": anns, "categories": cats}, rows


class _Dataset:
    class_ids = [1, 3, 7]

    def __init__(self, gt):
        self.coco = gt


class _Loader(list):
    def __init__(self, gt, rank=0, world=1):
        super().__init__()
        self.dataset = _Dataset(gt)
        self.batch_size = BS
        ims = gt["images"][rank::world]  # the DistributedSampler's shard
        for k in range(0, len(ims), BS):
            b = ims[k:k + BS]
            self.append((torch.zeros(len(b), 3, IMG, IMG), None,
                         ([im["height"] for im in b], [im["width"] for im in b]), [im["id"] for im in b]))


class _Model(torch.nn.Module):
    """Returns the image ids as its 'output' so the stubbed NMS can look up the rows."""

    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.zeros(1))

    def forward(self, x):
        return x


def _patch(monkeypatch, rows, loader):
    import yolox_amd.utils as U
    ids = iter(i for batch in loader for i in batch[3])

    def postprocess(outputs, num_classes, conf, nms):
        return [rows[next(ids)] for _ in range(outputs.shape[0])]

    monkeypatch.setattr(U, "postprocess", postprocess)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)


def test_coco_evaluator_perfect_detections(monkeypatch):
    from yolox_amd.evaluators import CocoEvaluator
    gt, rows = _gt_and_rows()
    loader = _Loader(gt)
    _patch(monkeypatch, rows, loader)
    ev = CocoEvaluator(loader, IMG, 0.01, 0.65, 3)
    (ap, ap50, info), per_image = ev.evaluate(_Model(), return_outputs=True)
    assert ap == pytest.approx(1.0) and ap50 == pytest.approx(1.0)
    assert "Average Precision  (AP) @[ IoU=0.50:0.95 | area=   all | maxDets=100 ] = 1.000" in info
    assert "per class AP:" in info and "per class AR:" in info
    assert sorted(per_image) == [im["id"] for im in gt["images"]]
    a = next(x for x in gt["annotations"] if x["image_id"] == 100)
    b = per_image[100]["bboxes"][0]
    np.testing.assert_allclose([b[0], b[1], b[2] - b[0], b[3] - b[1]], a["bbox"], rtol=1e-5)


def test_coco_evaluator_misses_lower_ap(monkeypatch):
    from yolox_amd.evaluators import CocoEvaluator
    gt, rows = _gt_and_rows()
    rows[100] = None  # image 100's objects missed
    loader = _Loader(gt)
    _patch(monkeypatch, rows, loader)
    ap, ap50, _ = CocoEvaluator(loader, IMG, 0.01, 0.65, 3, per_class_AP=False, per_class_AR=False).evaluate(
        _Model())
    assert 0.0 < ap < 1.0 and ap50 < 1.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import yolox_amd.utils as U
        from yolox_amd.evaluators import CocoEvaluator
        gt, rows = _gt_and_rows()
        rows[101] = None
        loader = _Loader(gt, rank, world)
        ids = iter(i for batch in loader for i in batch[3])
        U.postprocess = lambda outputs, *a: [rows[next(ids)] for _ in range(outputs.shape[0])]
        torch.cuda.synchronize = lambda *a, **k: None
        res, per_image = CocoEvaluator(loader, IMG, 0.01, 0.65, 3).evaluate(_Model(), distributed=True,
                                                                             return_outputs=True)
        q.put((rank, res[0], res[1], sorted(per_image)))
    finally:
        dist.destroy_process_group()


def test_coco_evaluator_distributed_gloo_world2(monkeypatch):
    """Each rank evaluates its shard; rank 0's AP over the gathered detections equals the
    single-process AP over the whole set; other ranks return (0, 0)."""
    from yolox_amd.evaluators import CocoEvaluator
    gt, rows = _gt_and_rows()
    rows[101] = None
    loader = _Loader(gt)
    _patch(monkeypatch, rows, loader)
    ap_one, ap50_one, _ = CocoEvaluator(loader, IMG, 0.01, 0.65, 3).evaluate(_Model())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (a, a50, ids)) for r, a, a50, ids in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][0] == pytest.approx(ap_one) and got[0][1] == pytest.approx(ap50_one)
    assert got[1][0] == 0 and got[1][1] == 0
    assert got[0][2] == got[1][2] == [im["id"] for im in gt["images"] if im["id"] != 101]


def test_summary_text_format():
    """pycocotools' summarize() lines for the 12 statistics."""
    from yolox_amd.evaluators import summary_text
    t = summary_text(np.array([0.5, 0.7, 0.55, -1, 0.3, 0.6, 0.2, 0.4, 0.45, -1, 0.35, 0.65]))
    lines = t.splitlines()
    assert len(lines) == 12
    assert lines[0] == " Average Precision  (AP) @[ IoU=0.50:0.95 | area=   all | maxDets=100 ] = 0.500"
    assert lines[1] == " Average Precision  (AP) @[ IoU=0.50      | area=   all | maxDets=100 ] = 0.700"
    assert lines[3] == " Average Precision  (AP) @[ IoU=0.50:0.95 | area= small | maxDets=100 ] = -1.000"
    assert lines[6] == " Average Recall     (AR) @[ IoU=0.50:0.95 | area=   all | maxDets=  1 ] = 0.200"


def test_eval_loader_legacy_normalisation(monkeypatch):
    """get_eval_loader(legacy=True) = ValTransform(legacy=True) (data_augment.py:236-240): after the
    letterbox, BGR -> RGB, /255, - mean, / std, rounded as numpy's in-place float32 ops round; the
    default (legacy=False) hands the letterboxed batch over untouched.  The device letterbox is
    stubbed with a seeded float32 batch (its own parity: tests/test_gpu_processor.py)."""
    from yolox_amd.config import named_config
    from yolox_amd.models import processor as P

    rng = np.random.default_rng(5)
    boxed = rng.integers(0, 256, size=(2, 3, IMG, IMG)).astype(np.float32)
    boxed[0, :, :4, :4] = 114.0  # letterbox padding value
    monkeypatch.setattr(P, "letterbox_batch", lambda imgs, size: torch.from_numpy(boxed.copy()))

    class _Items:
        coco, class_ids = {}, [1]

        def __len__(self):
            return 2

        def pull_item(self, i):
            return np.zeros((8, 8, 3), np.uint8), np.zeros((1, 5)), (8, 8), i

    cfg = named_config("yolox_s")
    plain = next(iter(cfg.get_eval_loader(2, False, dataset=_Items())))[0]
    assert torch.equal(plain, torch.from_numpy(boxed))
    got = next(iter(cfg.get_eval_loader(2, False, dataset=_Items(), legacy=True)))[0].numpy()
    want = []
    for img in boxed:  # data_augment.py:236-240 verbatim semantics, per image
        img = img[::-1, :, :].copy()
        img /= 255.0
        img -= np.array([0.485, 0.456, 0.406]).reshape(3, 1, 1)
        img /= np.array([0.229, 0.224, 0.225]).reshape(3, 1, 1)
        want.append(img)
    want = np.stack(want)
    assert got.dtype == np.float32 and np.array_equal(got, want)
    ev = cfg.get_evaluator(2, False, legacy=True, dataset=_Items())
    assert ev.dataloader.legacy
