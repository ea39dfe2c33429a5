"""The oracle (CPU restatement) against the reference's own outputs.

Every fixture under tests/golden/ was produced by running the reference model
files in the build container (tests/golden/make_golden.py).  These tests pin the
oracle before it is trusted as the checker for the HIP path.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

torch.set_num_threads(min(8, os.cpu_count() or 1))

FWD = [("yolox_s", 128), ("yolox_tiny", 416), ("yolox_nano", 128), ("yolox_m", 64),
       ("yolox_l", 96), ("yolox_x", 64)]


def shapes(name):
    with open(os.path.join(GOLDEN, "state_dict_shapes.json")) as f:
        return {k: s for k, s in json.load(f)[name]}


def weights(name):
    from yolox_amd.weights import synthetic_state_dict
    return synthetic_state_dict(shapes(name), seed=0, bn_stats=name)


@pytest.mark.parametrize("name,hw", FWD)
def test_forward_eval_matches_reference(oracle, golden, name, hw):
    d = golden(f"fwd_{name}_{hw}.npz")
    x = torch.from_numpy(oracle.letterbox_identity(d["input_u8"]))
    out = oracle.forward_eval(weights(name), oracle.ARCHS[name], x).numpy()
    ref = d["output"]
    assert out.shape == ref.shape
    # fp32 on both sides; differences come only from CPU thread-count reduction order
    np.testing.assert_allclose(out, ref, rtol=2e-4, atol=2e-4)


def test_fpn_features_match_reference(oracle, golden):
    d = golden("fwd_yolox_s_128.npz")
    x = torch.from_numpy(oracle.letterbox_identity(d["input_u8"]))
    with torch.no_grad():
        feats = oracle.backbone(weights("yolox_s"), oracle.ARCHS["yolox_s"], x)
    for i, f in enumerate(feats):
        np.testing.assert_allclose(f.numpy(), d[f"fpn{i}"], rtol=1e-4, atol=1e-4)


def _block_sd(d, key):
    pre = f"{key}.p."
    return {k[len(pre):]: torch.from_numpy(v) for k, v in d.items() if k.startswith(pre)}


@pytest.mark.parametrize("key", ["focus", "conv3s1", "conv3s2", "conv1", "conv1_lrelu", "conv3_relu",
                                 "bottleneck", "spp", "csp_short", "csp_noshort", "dwconv3s1",
                                 "dwconv3s2"])
def test_blocks_match_reference(oracle, golden, key):
    d = golden("blocks.npz")
    x = torch.from_numpy(d[f"{key}.x"])
    sd = _block_sd(d, key)
    eps = 1e-5  # blocks built outside config.get_model keep torch's default BN eps
    A = oracle.Arch(0.33, 0.5, bn_eps=eps)
    with torch.no_grad():
        if key == "focus":
            y = oracle.base_conv(sd, "conv", oracle.focus(x), 3, 1, "silu", eps)
        elif key.startswith("conv"):
            k = 1 if key.startswith("conv1") else 3
            s = 2 if key.endswith("s2") else 1
            act = "lrelu" if "lrelu" in key else "relu" if "relu" in key else "silu"
            y = oracle.base_conv({f"c.{k_}": v for k_, v in sd.items()}, "c", x, k, s, act, eps)
        elif key == "bottleneck":
            y = oracle.bottleneck({f"b.{k_}": v for k_, v in sd.items()}, "b", x, True, A, False)
        elif key == "spp":
            y = oracle.spp({f"s.{k_}": v for k_, v in sd.items()}, "s", x, A, False)
        elif key.startswith("csp"):
            n = 2 if key == "csp_short" else 1
            y = oracle.csp({f"c.{k_}": v for k_, v in sd.items()}, "c", x, n, key == "csp_short", A, False)
        else:
            s = 2 if key.endswith("s2") else 1
            Adw = oracle.Arch(0.33, 0.5, depthwise=True, bn_eps=eps)
            y = oracle.conv({f"c.{k_}": v for k_, v in sd.items()}, "c", x, 3, s, Adw, False)
    np.testing.assert_allclose(y.numpy(), d[f"{key}.y"], rtol=1e-5, atol=1e-5)


def test_bboxes_iou_and_iou_loss(oracle, golden):
    d = golden("boxes.npz")
    t = torch.from_numpy
    np.testing.assert_array_equal(oracle.bboxes_iou(t(d["a_xyxy"]), t(d["b_xyxy"]), True).numpy(),
                                  d["iou_xyxy"])
    np.testing.assert_array_equal(oracle.bboxes_iou(t(d["a_c"]), t(d["b_c"]), False).numpy(), d["iou_c"])
    np.testing.assert_array_equal(oracle.iou_loss(t(d["iouloss_p"]), t(d["iouloss_t"])).numpy(),
                                  d["iouloss"])
    with pytest.raises(IndexError):
        oracle.bboxes_iou(torch.zeros(2, 5), torch.zeros(3, 4))


def test_simota_matches_reference(oracle, golden):
    from yolox_amd.weights import anchor_grid, synthetic_head_outputs
    d = golden("simota_640.npz")
    xs, ys, st = (torch.from_numpy(a)[0] for a in anchor_grid(640, 640))
    bbox, cls, obj = (torch.from_numpy(a) for a in synthetic_head_outputs(2, 640, 640, seed=31))
    lab = torch.from_numpy(d["labels"])
    for b in range(2):
        G = int((lab[b].sum(1) > 0).sum())
        fg, matched, piou, gcls, nfg = oracle.simota_assign(
            lab[b, :G, 1:5], lab[b, :G, 0], bbox[b], cls[b], obj[b], xs, ys, st)
        assert nfg == int(d[f"img{b}.num_fg"])
        np.testing.assert_array_equal(fg.numpy(), d[f"img{b}.fg_mask"])
        np.testing.assert_array_equal(matched.numpy(), d[f"img{b}.matched_gt_inds"])
        np.testing.assert_array_equal(gcls.numpy(), d[f"img{b}.gt_matched_classes"])
        np.testing.assert_allclose(piou.numpy(), d[f"img{b}.pred_ious"], rtol=0, atol=0)


@pytest.mark.parametrize("tag", ["nol1", "l1"])
def test_train_losses_and_grads_match_reference(oracle, golden, tag):
    d = golden("train_yolox_s_128.npz")
    sd = {k: v.requires_grad_(v.is_floating_point() and "running" not in k)
          for k, v in weights("yolox_s").items()}
    x = torch.from_numpy(oracle.letterbox_identity(d["input_u8"]))
    out = oracle.forward_train(sd, oracle.ARCHS["yolox_s"], x, torch.from_numpy(d["labels"]),
                               use_l1=(tag == "l1"))
    for k in ("total_loss", "iou_loss", "l1_loss", "conf_loss", "cls_loss", "num_fg"):
        v = out[k]
        v = v.item() if torch.is_tensor(v) else v
        assert v == pytest.approx(float(d[f"{tag}.{k}"]), rel=1e-4, abs=1e-6), k
    out["total_loss"].backward()
    for key in [k for k in d if k.startswith(f"{tag}.grad.")]:
        pname = key[len(f"{tag}.grad."):]
        g = sd[pname].grad.numpy()
        ref = d[key]
        scale = np.abs(ref).max() + 1e-12
        assert np.abs(g - ref).max() / scale < 1e-3, pname


def test_postprocess_filter_matches_reference(oracle, golden):
    """The reference's pre-NMS candidates (recorded at its batched_nms call) are
    reproduced bit-exactly, and so is the in-place xyxy conversion."""
    d = golden("postprocess_pre_nms.npz")
    for conf in (0.01, 0.3):
        pred = d["prediction"].copy()
        oracle.xyxy_inplace(pred)
        np.testing.assert_array_equal(pred, d[f"c{conf}.xyxy_inplace"])
        nonempty = [r for r in (oracle.filter_candidates(p, 80, conf) for p in pred) if len(r)]
        assert len(nonempty) == int(d[f"c{conf}.ncalls"])
        for i, r in enumerate(nonempty):
            np.testing.assert_array_equal(r[:, :4], d[f"c{conf}.call{i}.boxes"])
            np.testing.assert_array_equal(r[:, 4] * r[:, 5], d[f"c{conf}.call{i}.scores"])
            np.testing.assert_array_equal(r[:, 6], d[f"c{conf}.call{i}.idxs"])


def _fixture_images(d):
    import hashlib

    from PIL import Image
    files = [os.path.join(GOLDEN, "images", f"{n}.jpg") for n in ("000000000001", "000000000009", "000000000016")]
    arrays = [np.asarray(Image.open(f)) for f in files]
    for i, a in enumerate(arrays):  # same decoder output as where the fixture was made
        assert hashlib.sha256(a.tobytes()).hexdigest() == str(d[f"img{i}.sha256"])
    return arrays


def test_processor_end_to_end_matches_reference(oracle, golden):
    """The reference's Yolox / YoloxProcessor / ValTransform / YoloxModule /
    utils.postprocess on its own test images (tests/test_detections.py:7-45 call
    patterns, all four identical; NMS = restated torchvision) vs the oracle chain:
    letterbox (bit-exact tensor), fp32 forward, C NMS, processor formatting.  Bars are
    the reference test's own: boxes 1e-2, scores 1e-4, labels exact."""
    import hashlib
    d = golden("processor_yolox_s_640.npz")
    arrays = _fixture_images(d)
    x = np.stack([oracle.letterbox(a, (640, 640)) for a in arrays])
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(d["tensor.sha256"])
    out = oracle.forward_eval(weights("yolox_s"), oracle.ARCHS["yolox_s"], torch.from_numpy(x)).numpy()
    for thr in (0.65, 0.3):
        rows = oracle.postprocess(out.copy(), 80, thr, 0.65)
        for i, a in enumerate(arrays):
            det = oracle.detections(rows[i], a.shape[:2], (640, 640))
            assert det["labels"] == d[f"t{thr}.img{i}.labels"].tolist()
            np.testing.assert_allclose(np.array(det["bboxes"]).reshape(-1, 4), d[f"t{thr}.img{i}.bboxes"],
                                       atol=1e-2, rtol=0)
            np.testing.assert_allclose(det["scores"], d[f"t{thr}.img{i}.scores"], atol=1e-4, rtol=0)


def test_oracle_letterbox_resize_paths(oracle):
    """The restated resize: r == 1 copy, exact 2x area path, generic bilinear within one
    LSB of float bilinear (cv2 itself is absent: parity unpinned beyond r == 1)."""
    import torch.nn.functional as F
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (64, 96, 3), dtype=np.uint8)
    out = oracle.letterbox(a, (32, 48))
    ref = (a[0::2, 0::2].astype(int) + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2] + 2) >> 2
    np.testing.assert_array_equal(out, ref.transpose(2, 0, 1).astype(np.float32))
    b = rng.integers(0, 256, (100, 150, 3), dtype=np.uint8)
    out = oracle.letterbox(b, (64, 64))
    r = min(64 / 100, 64 / 150)
    rh, rw = int(100 * r), int(150 * r)
    assert (out[:, rh:, :] == 114).all() and (out[:, :, rw:] == 114).all()
    fl = F.interpolate(torch.from_numpy(b).permute(2, 0, 1)[None].float(), size=(rh, rw), mode="bilinear",
                       align_corners=False)[0].numpy()
    assert np.abs(out[:, :rh, :rw] - fl).max() <= 1.01
    c = rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)
    out = oracle.letterbox(c, (640, 640))
    np.testing.assert_array_equal(out[:, :480], c.transpose(2, 0, 1).astype(np.float32))
    assert (out[:, 480:] == 114).all()


def test_processor_tiny_416_matches_reference(oracle, golden):
    """BASELINE configs[0] (yolox_tiny 416, one image) pinned: the reference's Yolox.__call__ on
    a 416x416 crop of its first test image (tests/golden/make_golden.py gen_processor_tiny) vs
    the oracle chain (letterbox r == 1, fp32 forward, C NMS, processor formatting)."""
    import hashlib

    from PIL import Image
    d = golden("processor_yolox_tiny_416.npz")
    a = np.asarray(Image.open(os.path.join(GOLDEN, "images", "000000000001.jpg")).convert("RGB")
                   .crop((0, 0, 416, 416)))
    assert hashlib.sha256(a.tobytes()).hexdigest() == str(d["img.sha256"])
    x = oracle.letterbox(a, (416, 416))[None]
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(d["tensor.sha256"])
    out = oracle.forward_eval(weights("yolox_tiny"), oracle.ARCHS["yolox_tiny"], torch.from_numpy(x)).numpy()
    for thr in (0.5, 0.3):
        (rows,) = oracle.postprocess(out.copy(), 80, thr, 0.65)
        det = oracle.detections(rows, a.shape[:2], (416, 416))
        assert det["labels"] == d[f"t{thr}.labels"].tolist()
        np.testing.assert_allclose(np.array(det["bboxes"]).reshape(-1, 4), d[f"t{thr}.bboxes"], atol=1e-2, rtol=0)
        np.testing.assert_allclose(det["scores"], d[f"t{thr}.scores"], atol=1e-4, rtol=0)
