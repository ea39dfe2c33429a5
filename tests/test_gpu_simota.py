"""On-device SimOTA assignment + YOLOX losses (yxh_yolox_loss) vs the reference.

* simota_640 fixture (reference get_assignments on synthetic 640 head outputs,
  G <= 50): fg mask, matched GT indices and num_fg exact; pred IoUs bit-exact.
* train fixture (reference train-mode forward of yolox_s at 128): the oracle
  (pinned to the same fixture) produces the head outputs; the device losses must
  match the reference's loss values within 1e-4 relative (north_star: 1e-3).
* random batches incl. images without labels vs the oracle's simota_assign.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def run(outputs, labels, hw, origin=None):
    from yolox_amd.models.losses import yolox_losses
    losses, assign = yolox_losses(outputs.cuda(), labels.cuda(), hw, origin_reg=None if origin is None else origin.cuda())
    torch.cuda.synchronize()
    return {k: v.item() for k, v in losses.items()}, {k: v.cpu() for k, v in assign.items()}


def check_image(assign, b, fg_ref, matched_ref, piou_ref, nfg_ref, iou_rtol=0.0):
    """Assignment exact; pred IoUs bit-exact when the head outputs are the reference's
    own, within iou_rtol when they come from the oracle (equal to fp32 rounding)."""
    fg = assign["fg_mask"][b].numpy()
    np.testing.assert_array_equal(fg, fg_ref)
    assert int(assign["num_fg"][b]) == int(nfg_ref)
    np.testing.assert_array_equal(assign["matched_gt_inds"][b].numpy()[fg], matched_ref)
    if iou_rtol:
        np.testing.assert_allclose(assign["pred_ious"][b].numpy()[fg], piou_ref, rtol=iou_rtol, atol=0)
    else:
        np.testing.assert_array_equal(assign["pred_ious"][b].numpy()[fg], piou_ref)


def test_simota_640_fixture(golden):
    from yolox_amd.weights import synthetic_head_outputs
    d = golden("simota_640.npz")
    bbox, cls, obj = synthetic_head_outputs(2, 640, 640, seed=31)
    outputs = torch.from_numpy(np.concatenate([bbox, obj, cls], -1))
    _, assign = run(outputs, torch.from_numpy(d["labels"]), [(80, 80), (40, 40), (20, 20)])
    for b in range(2):
        check_image(assign, b, d[f"img{b}.fg_mask"], d[f"img{b}.matched_gt_inds"], d[f"img{b}.pred_ious"],
                    d[f"img{b}.num_fg"])


@pytest.mark.parametrize("tag", ["nol1", "l1"])
def test_losses_match_reference_train_step(oracle, golden, tag):
    from yolox_amd.weights import synthetic_state_dict
    d = golden("train_yolox_s_128.npz")
    with open(os.path.join(GOLDEN, "state_dict_shapes.json")) as f:
        shapes = {k: s for k, s in json.load(f)["yolox_s"]}
    sd = synthetic_state_dict(shapes, seed=0, bn_stats="yolox_s")
    x = torch.from_numpy(oracle.letterbox_identity(d["input_u8"]))
    with torch.no_grad():
        outputs, origin, hw = oracle.train_outputs(sd, oracle.ARCHS["yolox_s"], x)
    losses, assign = run(outputs, torch.from_numpy(d["labels"]), hw, origin if tag == "l1" else None)
    names = {"total_loss": "total_loss", "iou_loss": "iou_loss", "conf_loss": "conf_loss", "cls_loss": "cls_loss",
             "l1_loss": "l1_loss", "num_fg": "num_fg"}
    for k, ref_k in names.items():
        assert losses[k] == pytest.approx(float(d[f"{tag}.{ref_k}"]), rel=1e-4, abs=1e-6), k
    for b in range(2):
        # head outputs from the oracle (not bit-identical to the reference's): IoUs to 1e-6
        check_image(assign, b, d[f"{tag}.img{b}.fg_mask"], d[f"{tag}.img{b}.matched_gt_inds"],
                    d[f"{tag}.img{b}.pred_ious"], d[f"{tag}.img{b}.num_fg"], iou_rtol=1e-6)


@pytest.mark.parametrize("seed", [0, 1])
def test_random_batches_vs_oracle(oracle, seed):
    from yolox_amd.weights import anchor_grid, synthetic_head_outputs, synthetic_labels
    B, S = 4, 320
    bbox, cls, obj = synthetic_head_outputs(B, S, S, seed=100 + seed)
    labels = synthetic_labels(B, S, S, max_gt=30, seed=200 + seed)
    labels[2] = 0.0  # an image without ground truth
    outputs = torch.from_numpy(np.concatenate([bbox, obj, cls], -1))
    _, assign = run(outputs, torch.from_numpy(labels), [(S // 8, S // 8), (S // 16, S // 16), (S // 32, S // 32)])
    xs, ys, st = (torch.from_numpy(a)[0] for a in anchor_grid(S, S))
    lab = torch.from_numpy(labels)
    for b in range(B):
        G = int((lab[b].sum(1) > 0).sum())
        if G == 0:
            assert int(assign["num_fg"][b]) == 0 and not assign["fg_mask"][b].any()
            continue
        fg, matched, piou, _, nfg = oracle.simota_assign(
            lab[b, :G, 1:5], lab[b, :G, 0], torch.from_numpy(bbox[b]), torch.from_numpy(cls[b]),
            torch.from_numpy(obj[b]), xs, ys, st)
        check_image(assign, b, fg.numpy(), matched.numpy(), piou.numpy(), nfg)
