#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE (pixeltable-yolox) on CPU.

Run in the build container only (needs /root/reference, which never travels to the
GPU box):   python tests/golden/make_golden.py

The reference package cannot be imported as-is (its __init__ reads installed
package metadata; cv2/torchvision/loguru are absent), so this script registers
empty package objects for ``yolox``, ``yolox.models``, ``yolox.utils``,
``yolox.data(.datasets)`` and loads the individual hot-path source files with
importlib.  torchvision.ops is replaced by a *recorder* that captures what the
reference hands to batched_nms/nms (so the pre-NMS filter is pinned) and keeps
everything (NMS itself is unpinned offline).

Outputs (all under tests/golden/ unless stated):
  state_dict_shapes.json keys/shapes of every preset's state_dict (checkpoint contract)
  bn_stats_<model>.npz  -> pixeltable-yolox_amd/yolox_amd/data/  (BN calibration)
  fwd_<model>_<hw>.npz   eval forward: input uint8 NHWC, decoded [B,A,85] output,
                         FPN features (yolox_s only)
  blocks.npz             per-block fixtures (Focus, BaseConv, Bottleneck, SPP, CSP, DWConv)
  train_yolox_s_128.npz  train-mode forward: losses, per-image SimOTA assignment,
                         selected gradients (use_l1 False and True)
  simota_640.npz         get_assignments on synthetic 640 predictions, G=50
  boxes.npz              bboxes_iou (xyxy / cxcywh), IouLoss
  postprocess_pre_nms.npz  the (boxes, scores, idxs) the reference gives batched_nms
"""
from __future__ import annotations

import importlib.util
import logging
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/yolox"
sys.path.insert(0, os.path.join(REPO, "pixeltable-yolox_amd"))

from yolox_amd.weights import (DATA_DIR, anchor_grid, synthetic_head_outputs,  # noqa: E402
                               synthetic_images, synthetic_labels, synthetic_state_dict)

torch.set_num_threads(8)
torch.manual_seed(0)


# --------------------------------------------------------------------------- shim
NMS_CALLS: list = []


def _register(name: str, path: str | None = None) -> types.ModuleType:
    mod = types.ModuleType(name)
    if path is not None:
        mod.__path__ = [path]
    sys.modules[name] = mod
    return mod


def _exec(name: str, rel: str) -> types.ModuleType:
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


# torchvision is absent: "record" keeps every candidate (pins the pre-NMS filter),
# "oracle" substitutes the restated torchvision nms/batched_nms (oracle/postprocess_oracle.c)
# so the reference's processor.postprocess can run end to end.
NMS_MODE = "record"


def _oracle_keep(boxes, scores, idxs, thr):
    sys.path.insert(0, REPO)
    from oracle import reference_cpu as O
    if idxs is None:
        keep = O.nms(boxes.numpy(), scores.numpy(), thr)
    else:
        keep = O.batched_nms(boxes.numpy(), scores.numpy(), idxs.numpy(), thr)
    return torch.from_numpy(keep)


def _recording_batched_nms(boxes, scores, idxs, thr):
    NMS_CALLS.append((boxes.clone(), scores.clone(), idxs.clone(), float(thr)))
    if NMS_MODE == "oracle":
        return _oracle_keep(boxes, scores, idxs, thr)
    return torch.argsort(scores, descending=True, stable=True)


def _recording_nms(boxes, scores, thr):
    NMS_CALLS.append((boxes.clone(), scores.clone(), None, float(thr)))
    if NMS_MODE == "oracle":
        return _oracle_keep(boxes, scores, None, thr)
    return torch.argsort(scores, descending=True, stable=True)


def _identity_resize(img, dsize, interpolation=None):
    """cv2 stub: only the identity resize (r == 1) is reproducible without cv2."""
    if tuple(dsize) != (img.shape[1], img.shape[0]):
        raise NotImplementedError(f"cv2 absent: resize {img.shape[:2]} -> {dsize} cannot be pinned")
    return img.copy()


def load_reference():
    _register("yolox", REF)
    utils = _register("yolox.utils", REF + "/utils")
    models = _register("yolox.models", REF + "/models")
    _register("yolox.data", REF + "/data")
    _register("yolox.data.datasets", REF + "/data/datasets").Dataset = object
    loguru = types.ModuleType("loguru")
    loguru.logger = logging.getLogger("reference")
    sys.modules["loguru"] = loguru
    tv = types.ModuleType("torchvision")
    tv.ops = types.SimpleNamespace(batched_nms=_recording_batched_nms, nms=_recording_nms)
    sys.modules["torchvision"] = tv
    boxes = _exec("yolox.utils.boxes", "utils/boxes.py")
    compat = _exec("yolox.utils.compat", "utils/compat.py")
    utils.bboxes_iou = boxes.bboxes_iou
    utils.cxcywh2xyxy = boxes.cxcywh2xyxy
    utils.meshgrid = compat.meshgrid
    utils.visualize_assign = None
    utils.postprocess = boxes.postprocess
    proc = _register("yolox.models.processor")
    proc.Detections = dict
    proc.YoloxProcessor = object
    ref = types.SimpleNamespace()
    ref.blocks = _exec("yolox.models.network_blocks", "models/network_blocks.py")
    ref.darknet = _exec("yolox.models.darknet", "models/darknet.py")
    ref.pafpn = _exec("yolox.models.yolo_pafpn", "models/yolo_pafpn.py")
    ref.losses = _exec("yolox.models.losses", "models/losses.py")
    ref.head = _exec("yolox.models.yolo_head", "models/yolo_head.py")
    ref.config = _exec("yolox.config", "config.py")
    ref.yolox = _exec("yolox.models.yolox", "models/yolox.py")
    models.YoloPafpn = ref.pafpn.YoloPafpn
    models.YoloxHead = ref.head.YoloxHead
    models.YoloxModule = ref.yolox.YoloxModule
    ref.boxes = boxes
    # the real processor (processor.py) over data_augment.ValTransform with a cv2 stub
    cv2 = types.ModuleType("cv2")
    cv2.INTER_LINEAR = 1
    cv2.resize = _identity_resize
    sys.modules["cv2"] = cv2
    utils.xyxy2cxcywh = boxes.xyxy2cxcywh
    ref.augment = _exec("yolox.data.data_augment", "data/data_augment.py")
    sys.modules["yolox.data"].ValTransform = ref.augment.ValTransform
    sys.modules["yolox"].data = sys.modules["yolox.data"]
    sys.modules["yolox"].utils = utils
    ref.processor = _exec("yolox.models.processor", "models/processor.py")
    return ref


# ------------------------------------------------------------------ helpers
CALIB_SEED = 1234
CALIB_HW = 256


def calibrate_bn(model: nn.Module, x: torch.Tensor) -> None:
    """Set each BN's running stats to the batch statistics of its input (fp64)."""
    hooks = []

    def pre(mod, inp):
        t = inp[0].double()
        mod.running_mean.copy_(t.mean(dim=(0, 2, 3)).float())
        mod.running_var.copy_(t.var(dim=(0, 2, 3), unbiased=False).float())

    for m in model.modules():
        if isinstance(m, nn.BatchNorm2d):
            hooks.append(m.register_forward_pre_hook(pre))
    was = model.training
    model.eval()
    with torch.no_grad():
        model(x)
    model.train(was)
    for h in hooks:
        h.remove()


def nchw(img_u8: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(img_u8).permute(0, 3, 1, 2).float().contiguous()


def build(ref, name: str, calibrated: bool = True) -> nn.Module:
    cfg = ref.config.YoloxConfig.get_named_config(name)
    cfg.model = None  # the named configs are singletons that cache the module
    model = cfg.get_model()
    sd = synthetic_state_dict(model.state_dict(), seed=0)
    model.load_state_dict(sd)
    if calibrated:
        calibrate_bn(model, nchw(synthetic_images(2, CALIB_HW, CALIB_HW, CALIB_SEED)))
    model.eval()
    return model


def save(name: str, **arrays) -> None:
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB)")


# ------------------------------------------------------------------ fixtures
MODELS = ["yolox_s", "yolox_m", "yolox_l", "yolox_x", "yolox_tiny", "yolox_nano"]
FWD_CASES = [("yolox_s", 2, 128), ("yolox_tiny", 1, 416), ("yolox_nano", 1, 128),
             ("yolox_m", 1, 64), ("yolox_l", 1, 96), ("yolox_x", 1, 64)]


def gen_bn_stats(ref) -> None:
    os.makedirs(DATA_DIR, exist_ok=True)
    for name in MODELS:
        model = build(ref, name)
        stats = {k: v.numpy() for k, v in model.state_dict().items()
                 if k.endswith("running_mean") or k.endswith("running_var")}
        path = os.path.join(DATA_DIR, f"bn_stats_{name}.npz")
        np.savez_compressed(path, **stats)
        print(f"wrote {path} ({len(stats)} tensors)")


def gen_shapes(ref) -> None:
    """state_dict keys/shapes per preset: the checkpoint-compatibility contract."""
    import json
    out = {}
    for name in MODELS:
        cfg = ref.config.YoloxConfig.get_named_config(name)
        cfg.model = None
        sd = cfg.get_model().state_dict()
        out[name] = [[k, list(v.shape)] for k, v in sd.items()]
    path = os.path.join(HERE, "state_dict_shapes.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print(f"wrote {path}")


def gen_forward(ref) -> None:
    for name, batch, hw in FWD_CASES:
        model = build(ref, name)
        img = synthetic_images(batch, hw, hw, seed=7)
        x = nchw(img)
        with torch.no_grad():
            feats = model.backbone(x)
            out = model(x)
        extra = {}
        if name == "yolox_s":
            extra = {f"fpn{i}": f.numpy() for i, f in enumerate(feats)}
        save(f"fwd_{name}_{hw}.npz", input_u8=img, output=out.numpy(), **extra)


def _block_params(mod: nn.Module, seed: int) -> dict:
    sd = synthetic_state_dict(mod.state_dict(), seed=seed)
    mod.load_state_dict(sd)
    return sd


def gen_blocks(ref) -> None:
    B = ref.blocks
    rng = np.random.default_rng(11)
    cases = {
        "focus": (B.Focus(3, 32, ksize=3), (2, 3, 32, 32), 255.0),
        "conv3s1": (B.BaseConv(32, 48, 3, 1), (2, 32, 16, 16), 1.0),
        "conv3s2": (B.BaseConv(32, 64, 3, 2), (2, 32, 17, 15), 1.0),
        "conv1": (B.BaseConv(64, 32, 1, 1), (2, 64, 16, 16), 1.0),
        "conv1_lrelu": (B.BaseConv(32, 32, 1, 1, act="lrelu"), (2, 32, 8, 8), 1.0),
        "conv3_relu": (B.BaseConv(32, 32, 3, 1, act="relu"), (2, 32, 8, 8), 1.0),
        "bottleneck": (B.Bottleneck(32, 32, True, 1.0), (2, 32, 16, 16), 1.0),
        "spp": (B.SPPBottleneck(64, 64), (2, 64, 20, 20), 1.0),
        "csp_short": (B.CspLayer(64, 64, n=2, shortcut=True), (2, 64, 16, 16), 1.0),
        "csp_noshort": (B.CspLayer(128, 64, n=1, shortcut=False), (2, 128, 8, 8), 1.0),
        "dwconv3s1": (B.DWConv(32, 48, 3, 1), (2, 32, 16, 16), 1.0),
        "dwconv3s2": (B.DWConv(32, 64, 3, 2), (2, 32, 16, 16), 1.0),
    }
    arrays = {}
    for i, (key, (mod, shape, scale)) in enumerate(cases.items()):
        params = _block_params(mod, seed=100 + i)
        x = torch.from_numpy(rng.uniform(-1, 1, shape).astype(np.float32)) * scale
        if key == "focus":
            x = torch.round(x.abs())
        calibrate_bn(mod, x)
        mod.eval()
        with torch.no_grad():
            y = mod(x)
        arrays[f"{key}.x"] = x.numpy()
        arrays[f"{key}.y"] = y.numpy()
        for k, v in mod.state_dict().items():
            arrays[f"{key}.p.{k}"] = v.numpy()
    save("blocks.npz", **arrays)


def gen_train(ref) -> None:
    arrays = {}
    for use_l1 in (False, True):
        model = build(ref, "yolox_s")
        model.train()
        model.head.use_l1 = use_l1
        head = model.head
        records = []
        orig = head.get_assignments

        def wrapped(*args, **kw):
            res = orig(*args, **kw)
            gt_cls, fg_mask, pred_ious, matched, num_fg = res
            records.append((fg_mask.clone(), matched.clone(), pred_ious.clone(), gt_cls.clone(), num_fg))
            return res

        head.get_assignments = wrapped
        img = synthetic_images(2, 128, 128, seed=21)
        labels = synthetic_labels(2, 128, 128, max_gt=12, seed=22)
        x = nchw(img)
        out = model(x, torch.from_numpy(labels))
        loss = out["total_loss"]
        loss.backward()
        tag = "l1" if use_l1 else "nol1"
        if use_l1:
            arrays["input_u8"] = img
            arrays["labels"] = labels
        for k in ("total_loss", "iou_loss", "l1_loss", "conf_loss", "cls_loss", "num_fg"):
            v = out[k]
            arrays[f"{tag}.{k}"] = np.float64(v.item() if torch.is_tensor(v) else v)
        for b, (fg, matched, piou, gcls, nfg) in enumerate(records):
            arrays[f"{tag}.img{b}.fg_mask"] = fg.numpy()
            arrays[f"{tag}.img{b}.matched_gt_inds"] = matched.numpy()
            arrays[f"{tag}.img{b}.pred_ious"] = piou.detach().numpy()
            arrays[f"{tag}.img{b}.gt_matched_classes"] = gcls.numpy()
            arrays[f"{tag}.img{b}.num_fg"] = np.int64(nfg)
        for pname in ("backbone.backbone.stem.conv.conv.weight", "backbone.backbone.stem.conv.bn.weight",
                      "backbone.C3_n4.conv3.conv.weight", "head.cls_preds.0.weight", "head.cls_preds.0.bias",
                      "head.reg_preds.1.weight", "head.obj_preds.2.bias", "head.stems.0.conv.weight"):
            p = dict(model.named_parameters())[pname]
            arrays[f"{tag}.grad.{pname}"] = p.grad.numpy()
    save("train_yolox_s_128.npz", **arrays)


def gen_simota(ref) -> None:
    """get_assignments on synthetic 640 head outputs (A=8400, G<=50).

    Inputs are regenerated from seeds by ``synthetic_head_outputs`` / ``synthetic_labels``;
    only labels and the reference's assignment outputs are stored.
    """
    head = ref.head.YoloxHead(80, width=0.5)
    x_s, y_s, st = (torch.from_numpy(a) for a in anchor_grid(640, 640))
    bbox, cls, obj = (torch.from_numpy(a) for a in synthetic_head_outputs(2, 640, 640, seed=31))
    labels = synthetic_labels(2, 640, 640, max_gt=50, seed=32)
    arrays = {"labels": labels}
    lab = torch.from_numpy(labels)
    for b in range(2):
        num_gt = int((lab[b].sum(1) > 0).sum())
        res = head.get_assignments(b, num_gt, lab[b, :num_gt, 1:5], lab[b, :num_gt, 0], bbox[b],
                                   st, x_s, y_s, cls, obj)
        gt_cls, fg_mask, pred_ious, matched, num_fg = res
        arrays[f"img{b}.fg_mask"] = fg_mask.numpy()
        arrays[f"img{b}.matched_gt_inds"] = matched.numpy()
        arrays[f"img{b}.pred_ious"] = pred_ious.numpy()
        arrays[f"img{b}.gt_matched_classes"] = gt_cls.numpy()
        arrays[f"img{b}.num_fg"] = np.int64(num_fg)
    save("simota_640.npz", **arrays)


def gen_boxes(ref) -> None:
    rng = np.random.default_rng(41)
    a = rng.uniform(0, 100, (13, 4)).astype(np.float32)
    b = rng.uniform(0, 100, (29, 4)).astype(np.float32)
    a_xyxy = np.concatenate([np.minimum(a[:, :2], a[:, 2:]), np.maximum(a[:, :2], a[:, 2:])], 1)
    b_xyxy = np.concatenate([np.minimum(b[:, :2], b[:, 2:]), np.maximum(b[:, :2], b[:, 2:])], 1)
    a_c = np.concatenate([a[:, :2], np.abs(a[:, 2:] - 50) + 1], 1).astype(np.float32)
    b_c = np.concatenate([b[:, :2], np.abs(b[:, 2:] - 50) + 1], 1).astype(np.float32)
    iou_xyxy = ref.boxes.bboxes_iou(torch.from_numpy(a_xyxy), torch.from_numpy(b_xyxy), True)
    iou_c = ref.boxes.bboxes_iou(torch.from_numpy(a_c), torch.from_numpy(b_c), False)
    p = torch.from_numpy(np.abs(rng.normal(30, 10, (64, 4))).astype(np.float32))
    t = torch.from_numpy(np.abs(rng.normal(30, 10, (64, 4))).astype(np.float32))
    loss = ref.losses.IouLoss(reduction="none")(p, t)
    save("boxes.npz", a_xyxy=a_xyxy, b_xyxy=b_xyxy, iou_xyxy=iou_xyxy.numpy(), a_c=a_c, b_c=b_c,
         iou_c=iou_c.numpy(), iouloss_p=p.numpy(), iouloss_t=t.numpy(), iouloss=loss.numpy())


def gen_postprocess(ref) -> None:
    """Pin the reference's pre-NMS filter: what it hands to batched_nms."""
    d = np.load(os.path.join(HERE, "fwd_yolox_s_128.npz"))
    arrays = {"prediction": d["output"]}
    for conf in (0.01, 0.3):
        NMS_CALLS.clear()
        pred = torch.from_numpy(d["output"].copy())
        ref.boxes.postprocess(pred, 80, conf, 0.65, class_agnostic=False)
        arrays[f"c{conf}.xyxy_inplace"] = pred.numpy()
        for i, (bx, sc, ix, thr) in enumerate(NMS_CALLS):
            arrays[f"c{conf}.call{i}.boxes"] = bx.numpy()
            arrays[f"c{conf}.call{i}.scores"] = sc.numpy()
            arrays[f"c{conf}.call{i}.idxs"] = ix.numpy()
        arrays[f"c{conf}.ncalls"] = np.int64(len(NMS_CALLS))
    save("postprocess_pre_nms.npz", **arrays)


IMAGE_FILES = [os.path.join(HERE, "images", f"{n}.jpg") for n in ("000000000001", "000000000009", "000000000016")]
PROC_THRESHOLDS = (0.65, 0.3)


def gen_processor(ref) -> None:
    """End to end through the reference's own Yolox / YoloxProcessor / ValTransform /
    YoloxModule / utils.postprocess (tests/test_detections.py:7-45 call patterns) on the
    reference's test images (copied to tests/golden/images; all give r == 1 at 640, so the
    cv2 stub's identity resize is exact).  NMS is the restated torchvision (oracle)."""
    import hashlib

    from PIL import Image

    global NMS_MODE
    NMS_MODE = "oracle"
    model = build(ref, "yolox_s")
    proc = ref.processor.YoloxProcessor("yolox_s")
    yolox = ref.yolox.Yolox(model, proc)
    images = [Image.open(f) for f in IMAGE_FILES]
    arrays = {}
    for i, im in enumerate(images):
        arrays[f"img{i}.sha256"] = np.array(hashlib.sha256(np.asarray(im).tobytes()).hexdigest())
        arrays[f"img{i}.size"] = np.array(im.size, np.int64)
    with torch.no_grad():
        tensor = proc(images)
        arrays["tensor.sha256"] = np.array(hashlib.sha256(tensor.numpy().tobytes()).hexdigest())
        arrays["tensor.shape"] = np.array(tensor.shape, np.int64)
        for thr in PROC_THRESHOLDS:
            patterns = {
                "files": yolox(IMAGE_FILES, threshold=thr),
                "images": yolox(images, threshold=thr),
                "separate": proc.postprocess(images, model(tensor.clone()), threshold=thr),
                "deprecated": proc.postprocess(images, yolox(tensor.clone()), threshold=thr),
            }
            dets = patterns["files"]
            for name, got in patterns.items():
                assert got == dets, f"call pattern {name} differs"
            for i, d in enumerate(dets):
                arrays[f"t{thr}.img{i}.bboxes"] = np.array(d["bboxes"], np.float64).reshape(-1, 4)
                arrays[f"t{thr}.img{i}.scores"] = np.array(d["scores"], np.float64)
                arrays[f"t{thr}.img{i}.labels"] = np.array(d["labels"], np.int64)
            print(f"threshold {thr}: detections per image {[len(d['labels']) for d in dets]}")
    NMS_MODE = "record"
    save("processor_yolox_s_640.npz", **arrays)


def tiny_416_image():
    """BASELINE configs[0] input: one 416x416 RGB image (r == 1 at yolox_tiny's 416 test size, so
    the cv2 stub's identity resize is exact) -- the top-left 416x416 crop of the reference's first
    test image."""
    from PIL import Image
    return Image.open(IMAGE_FILES[0]).convert("RGB").crop((0, 0, 416, 416))


def gen_processor_tiny(ref) -> None:
    """configs[0]: yolox_tiny single-image inference through the reference's own Yolox.__call__
    (yolox.py:41-52 -> YoloxProcessor (416) -> YoloxModule -> postprocess), seeded weights."""
    import hashlib

    global NMS_MODE
    NMS_MODE = "oracle"
    model = build(ref, "yolox_tiny")
    proc = ref.processor.YoloxProcessor("yolox_tiny")
    yolox = ref.yolox.Yolox(model, proc)
    im = tiny_416_image()
    arrays = {"img.sha256": np.array(hashlib.sha256(np.asarray(im).tobytes()).hexdigest())}
    with torch.no_grad():
        tensor = proc([im])
        arrays["tensor.sha256"] = np.array(hashlib.sha256(tensor.numpy().tobytes()).hexdigest())
        arrays["tensor.shape"] = np.array(tensor.shape, np.int64)
        for thr in (0.5, 0.3):
            (d,) = yolox([im], threshold=thr)
            arrays[f"t{thr}.bboxes"] = np.array(d["bboxes"], np.float64).reshape(-1, 4)
            arrays[f"t{thr}.scores"] = np.array(d["scores"], np.float64)
            arrays[f"t{thr}.labels"] = np.array(d["labels"], np.int64)
            print(f"tiny 416 threshold {thr}: {len(d['labels'])} detections")
    NMS_MODE = "record"
    save("processor_yolox_tiny_416.npz", **arrays)


MOSAIC_HW = (64, 96)
# (h, w) of the fixture's pull_item images: exact copies, 2x up, exact 2x down (INTER_AREA), odd
# bilinear factors in both directions, tall and wide
MOSAIC_SHAPES = [(64, 96), (32, 48), (128, 192), (50, 70), (200, 90), (41, 96), (64, 33), (97, 131), (20, 150),
                 (64, 96)]
MOSAIC_CASES = {  # name -> MosaicDetection kwargs (config.py defaults; the nano preset; close_mosaic)
    "default": dict(mosaic=True, mosaic_scale=(0.1, 2), mixup_scale=(0.5, 1.5), enable_mixup=True,
                    mosaic_prob=1.0, mixup_prob=1.0),
    "nano": dict(mosaic=True, mosaic_scale=(0.5, 1.5), mixup_scale=(0.5, 1.5), enable_mixup=False,
                 mosaic_prob=0.5, mixup_prob=1.0),
    "no_aug": dict(mosaic=False, mosaic_scale=(0.1, 2), mixup_scale=(0.5, 1.5), enable_mixup=True,
                   mosaic_prob=1.0, mixup_prob=1.0),
}
MOSAIC_SEEDS = 12


def mosaic_dataset():
    """Fixture dataset: seeded BGR images of MOSAIC_SHAPES with structured content and 0-5
    boxes (x1, y1, x2, y2, cls) each (image 3 has none)."""
    rng = np.random.default_rng(77)
    images, labels = [], []
    for i, (h, w) in enumerate(MOSAIC_SHAPES):
        yy, xx = np.mgrid[0:h, 0:w]
        img = np.stack([xx * 255 // max(w - 1, 1), yy * 255 // max(h - 1, 1), (xx * yy) % 256], -1)
        img = (img + rng.integers(-30, 31, (h, w, 3))).clip(0, 255).astype(np.uint8)
        n = 0 if i == 3 else int(rng.integers(1, 6))
        lab = np.zeros((n, 5))
        for k in range(n):
            bw, bh = rng.uniform(1.5, w), rng.uniform(1.5, h)
            x1, y1 = rng.uniform(0, w - bw), rng.uniform(0, h - bh)
            lab[k] = (x1, y1, x1 + bw, y1 + bh, int(rng.integers(0, 80)))
            img[int(y1):int(y1 + bh), int(x1):int(x1 + bw)] = rng.integers(0, 256, 3)
        images.append(img)
        labels.append(lab)
    return images, labels


def gen_mosaic(ref) -> None:
    """The reference's own MosaicDetection.__getitem__ / mixup / TrainTransform(max_labels=120)
    (mosaicdetection.py:76-232, data_augment.py:19-208) over mosaic_dataset(), with the oracle's
    cv2 restatement (oracle/augment_oracle.py) in place of cv2: pins the random-draw order, the
    label arithmetic and the image-operation order; pixel values of cv2's kernels stay pinned only
    to the restatement.  Each sample seeds random / np.random with its seed first."""
    import random as pyrandom

    sys.path.insert(0, REPO)
    from oracle import augment_oracle as A
    cv2 = sys.modules["cv2"]
    for k in ("INTER_LINEAR", "COLOR_BGR2HSV", "COLOR_HSV2BGR", "resize", "warpAffine", "cvtColor",
              "getRotationMatrix2D"):
        setattr(cv2, k, getattr(A.CV2, k))
    utils = sys.modules["yolox.utils"]
    utils.adjust_box_anns = ref.boxes.adjust_box_anns
    utils.get_local_rank = lambda: 0
    wrapper = _exec("yolox.data.datasets.datasets_wrapper", "data/datasets/datasets_wrapper.py")
    mosaic = _exec("yolox.data.datasets.mosaicdetection", "data/datasets/mosaicdetection.py")
    images, labels = mosaic_dataset()

    class FixtureDataset(wrapper.Dataset):
        def __init__(self):
            super().__init__(MOSAIC_HW)

        def __len__(self):
            return len(images)

        def load_anno(self, i):
            return labels[i]

        def pull_item(self, i):
            return images[i].copy(), labels[i].copy(), images[i].shape[:2], np.array([i])

    arrays = {"input_hw": np.array(MOSAIC_HW, np.int64), "shapes": np.array(MOSAIC_SHAPES, np.int64),
              "pixels": np.concatenate([im.reshape(-1) for im in images]),
              "label_counts": np.array([len(l) for l in labels], np.int64),
              "labels": np.concatenate(labels, 0).astype(np.float64)}
    for case, kw in MOSAIC_CASES.items():
        ds = mosaic.MosaicDetection(FixtureDataset(), MOSAIC_HW,
                                    preproc=ref.augment.TrainTransform(max_labels=120, flip_prob=0.5, hsv_prob=1.0),
                                    degrees=10.0, translate=0.1, shear=2.0, **kw)
        for s in range(MOSAIC_SEEDS):
            idx = s % len(images)
            pyrandom.seed(1000 + s)
            np.random.seed(1000 + s)
            img, lab, info, img_id = ds[idx]
            assert img.dtype == np.float32 and np.all(img == np.round(img)), "image not integral"
            arrays[f"{case}.{s}.image"] = img.astype(np.uint8)
            arrays[f"{case}.{s}.labels"] = lab
            arrays[f"{case}.{s}.info"] = np.array(info, np.int64)
            arrays[f"{case}.{s}.id"] = np.array(img_id, np.int64).reshape(-1)
        print(f"mosaic {case}: {MOSAIC_SEEDS} samples")
    # the close_mosaic boundary (trainer.py:217-230 -> YoloBatchSampler(mosaic=False)): ONE seed,
    # MOSAIC_SEEDS samples drawn with mosaic on, then MOSAIC_SEEDS with it off -- pins which
    # random draws each mode consumes across the switch
    ds = mosaic.MosaicDetection(FixtureDataset(), MOSAIC_HW,
                                preproc=ref.augment.TrainTransform(max_labels=120, flip_prob=0.5, hsv_prob=1.0),
                                degrees=10.0, translate=0.1, shear=2.0, **MOSAIC_CASES["default"])
    pyrandom.seed(4242)
    np.random.seed(4242)
    for s in range(2 * MOSAIC_SEEDS):
        _, lab, _, _ = ds[(s < MOSAIC_SEEDS, (3 * s + 1) % len(images))]
        arrays[f"boundary.{s}.labels"] = lab
    print(f"mosaic boundary: {2 * MOSAIC_SEEDS} samples")
    save("mosaic_aug.npz", **arrays)


def gen_resize(ref) -> None:
    """The reference's own YoloxConfig.preprocess (config.py:296-305: F.interpolate bilinear,
    align_corners False, + the label scaling) on CPU over a seeded 160x160 batch (a copy of the
    yolox_s config with input_size 160, so the fixture stays small) at down / up / non-square
    sizes; float32.  The device kernel is bit-exact to ATen's bilinear on the GPU
    (tests/test_gpu_augment.py); against this CPU run it is held to a few ulps (ATen's CPU
    kernel contracts the same expression differently)."""
    import copy
    cfg = copy.copy(ref.config.YoloxConfig.get_named_config("yolox_s"))
    cfg.input_size = (160, 160)
    g = torch.Generator().manual_seed(77)
    x = (torch.rand(2, 3, 160, 160, generator=g) * 255).round()
    t = torch.rand(2, 6, 5, generator=g) * 150
    arrays = {"input_u8": x.to(torch.uint8).numpy(), "targets": t.numpy()}
    for size in ((128, 128), (192, 192), (224, 160), (96, 200)):
        y, t2 = cfg.preprocess(x.clone(), t.clone(), size)
        arrays[f"{size[0]}x{size[1]}.image"] = y.numpy()
        arrays[f"{size[0]}x{size[1]}.targets"] = t2.numpy()
    save("resize_preprocess.npz", **arrays)


def main() -> None:
    if not os.path.isdir(REF):
        sys.exit("reference not present: fixtures can only be generated in the build container")
    ref = load_reference()
    if len(sys.argv) > 1:  # generate only the named fixtures, e.g. `make_golden.py processor`
        for name in sys.argv[1:]:
            globals()[f"gen_{name}"](ref)
        return
    gen_shapes(ref)
    gen_bn_stats(ref)
    gen_forward(ref)
    gen_blocks(ref)
    gen_train(ref)
    gen_simota(ref)
    gen_boxes(ref)
    gen_postprocess(ref)
    gen_processor(ref)


if __name__ == "__main__":
    main()
