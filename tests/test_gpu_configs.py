"""Parity at the BASELINE.json workloads themselves (not scaled-down stand-ins).

configs[1]  yolox_s 640 bf16 batch 32: the autotuned, graph-captured plan bench.py
            times; all 32 images vs the oracle's fp32 forward, within bounds derived from
            the oracle itself run with bf16 storage (weights and every stored map rounded,
            oracle.stored_as: DESIGN.md §7), device NMS on the whole replayed batch
            bit-exact vs the oracle's NMS on the same output, and BOX mAP of the device's
            detections (the benched step: conf 0.5, nms 0.65) scored by the COCO harness with
            the fp32 oracle's detections as ground truth (BASELINE's "box mAP parity").
configs[2]  yolox_s 640 train step batch 8 in fp32 (the reference's default precision):
            the six loss values and every parameter gradient within 1e-3 of the
            oracle's autograd (north_star tolerance).
configs[0]  yolox_tiny 416 single image through Yolox.from_pretrained (a local checkpoint of
            the seeded weights) and Yolox.__call__: Detections vs the reference-run fixture
            (processor_yolox_tiny_416.npz; the reference test's bars) and == the oracle NMS +
            formatting on the same device output.
configs[3]  yolox_l 640 fp16 batch 16 (bench plan): all 16 images vs the oracle's fp32 forward
            (bounds derived from the oracle with fp16 storage) and device NMS on the whole batch bit-exact vs the oracle's NMS on the
            same output.
configs[4]  yolox_x 1280 --fp16 train: on-device SimOTA at A = 33600 anchors with up to
            120 GTs exact vs the oracle (fg mask, matched GT, num_fg; IoUs to fp32
            rounding) plus the loss values; a yolox_x 1280 train step at the per-GPU batch of
            -d 8 -b 64 (8 images) in fp32 whose losses (rel 1e-3) and named parameter gradients
            (1e-3 of the tensor's max) match the oracle's autograd; and the --fp16 step (batch 8,
            the bench's) against the same oracle within bounds derived from the oracle run with
            fp16 storage.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def probs_close(out, ref, pmax, p99, xy):
    dp = np.abs(out[..., 4:] - ref[..., 4:])
    assert dp.max() < pmax and np.quantile(dp, 0.99) < p99, (dp.max(), np.quantile(dp, 0.99))
    assert np.abs(out[..., :2] - ref[..., :2]).max() < xy


def oracle_forward(oracle, name, images_u8, stored=None):
    """The oracle's fp32 forward, or (stored = bf16 / f16) the same with the device's storage
    precision emulated (oracle.stored_as)."""
    from yolox_amd.config import named_config
    from yolox_amd.weights import synthetic_state_dict
    sd = synthetic_state_dict(named_config(name).get_model().state_dict(), seed=0, bn_stats=name)
    x = torch.from_numpy(oracle.letterbox_identity(images_u8))
    with torch.no_grad(), oracle.stored_as(stored):
        return oracle.forward_eval(sd, oracle.ARCHS[name], x).numpy()


def derived_bounds_hold(dev, ref, emu, factor):
    """dev (device, 16-bit) vs ref (oracle fp32) within ``factor`` x the distance of emu (the
    oracle with 16-bit storage) from ref: max and p99 of the probabilities, max of the box
    centres -- a faithful 16-bit implementation differs from emu only in summation order."""
    stats = {}
    for name, sl in (("prob", np.s_[..., 4:]), ("xy", np.s_[..., :2])):
        d_dev, d_emu = np.abs(dev[sl] - ref[sl]), np.abs(emu[sl] - ref[sl])
        stats[name] = (float(d_dev.max()), float(d_emu.max()), float(np.quantile(d_dev, 0.99)),
                       float(np.quantile(d_emu, 0.99)))
    pm, pe, p99m, p99e = stats["prob"]
    assert pm <= factor * pe and p99m <= factor * p99e, stats
    assert stats["xy"][0] <= factor * stats["xy"][1] + 0.25, stats
    return stats


def bench_plan(name, batch, size, dtype):
    """bench.py's inference plan: uint8 NHWC resident input, autotune, hipGraph."""
    from yolox_amd import _native as N
    from yolox_amd.models import YoloxModule
    from yolox_amd.weights import synthetic_images
    model = YoloxModule.synthetic(name, seed=0, device="cuda", dtype=dtype)
    plan = model.plan_for(batch, size, size, N.NHWC, torch.uint8)
    imgs = synthetic_images(batch, size, size, seed=1000)
    plan.static_input().copy_(torch.from_numpy(imgs).cuda())
    plan.autotune()
    plan.capture()
    return model, plan, imgs


@pytest.mark.parametrize("name,batch,dtype", [("yolox_s", 32, torch.bfloat16), ("yolox_l", 16, torch.float16)])
def test_every_candidate_tile_is_deterministic(name, batch, dtype):
    """Race detector at the benched shapes: every conv op of the configs[1] / configs[3] plan, under
    EVERY 16-bit tile the autotuner may pick for it, writes the same bytes on three runs over the
    same inputs.  (Round 5: a K-split exchange overlapping a row buffer still in flight made three
    conv_ws1 variants nondeterministic only where a block walks several pixel tiles -- the bench's
    shapes -- while the small-shape op tests passed.)  In-place ops (output = residual input) are
    skipped; every other op's written buffers are compared whole."""
    import ctypes as C
    from yolox_amd import _native as N
    from yolox_amd.engine import TILE_CANDIDATES_16, op_buffers
    model, plan, _ = bench_plan(name, batch, 640, dtype)
    L, st = plan.lib, N.stream_ptr(plan.device)
    N.check(L.yxh_run_ops(plan._ops, plan._nops, st), "forward")
    checked = 0
    for i, rec in enumerate(plan.ctx.ops):
        if rec.kind != N.OP_CONV or rec.args["groups"] != 1:
            continue
        reads, writes = op_buffers(rec)
        if not writes or any(w is r for w in writes for r in reads):
            continue
        op = plan._ops[i]
        keep, ptr = op.u.conv.tile, C.pointer(op)
        regions = [plan.arena[w.offset:w.offset + plan.chunk * w.h * w.w * w.c * w.esize] for w in writes]
        for tile in TILE_CANDIDATES_16:
            op.u.conv.tile = tile
            if L.yxh_run_ops(ptr, 1, st) != N.OK:  # variant not applicable
                continue
            first = [r.clone() for r in regions]
            for _ in range(2):
                N.check(L.yxh_run_ops(ptr, 1, st), "op")
                assert all(torch.equal(a, r) for a, r in zip(first, regions)), (name, i, tile >> 1, tile & 1)
            checked += 1
        op.u.conv.tile = keep
    torch.cuda.synchronize()
    print(f"{name}: {checked} (op, tile) pairs deterministic")
    assert checked > 100


def box_map_vs_oracle(dets, ref_dets, size):
    """(AP@[.5:.95], AP@.5) of detections ``dets`` (per image [N, 7] rows: x1, y1, x2, y2, obj,
    cls_conf, cls) scored by the COCO harness (yolox_amd.evaluators.coco: the reference's
    COCOeval_opt, pinned in tests/test_coco_map.py) against ``ref_dets`` (the fp32 oracle's
    detections of the same images) as the ground truth: 1.0 / 1.0 means the same boxes."""
    from yolox_amd.evaluators.coco import coco_bbox_eval, convert_to_coco_format
    n = len(dets)
    images, anns = [], []
    for i, r in enumerate(ref_dets):
        images.append({"id": i, "height": size, "width": size})
        for row in np.asarray(r).reshape(-1, 7):
            x1, y1, x2, y2 = (float(v) for v in row[:4])
            w, h = x2 - x1, y2 - y1
            anns.append({"id": len(anns) + 1, "image_id": i, "category_id": int(row[6]), "bbox": [x1, y1, w, h],
                         "area": w * h, "iscrowd": 0})
    gt = {"images": images, "annotations": anns, "categories": [{"id": c, "name": str(c)} for c in range(80)]}
    res = convert_to_coco_format([torch.from_numpy(np.asarray(d).reshape(-1, 7)) for d in dets],
                                 ([size] * n, [size] * n), list(range(n)), (size, size), list(range(80)))
    st = coco_bbox_eval(gt, res)["stats"]
    return float(st[0]), float(st[1])


def map_parity(host, ref, emu, dev_dets, size, tag):
    """Box-mAP parity at the benched precision: the device's detections vs the fp32 oracle's
    (ground truth) may lose at most MAP_FACTOR x the AP that the oracle run with the device's
    16-bit storage loses (+ 0.01), and stay above an absolute floor.  AP50 == AP50:95 on these
    synthetic nets: a box the device keeps is the oracle's box to IoU > 0.95; what costs AP is
    detections whose confidence sits at the 0.5 threshold or whose NMS partner flips (the ~150
    detections per image of a random-weight net crowd the threshold far more than a trained
    net's).  The AP of a faithful 16-bit implementation depends on its summation order: oracle
    emulations that differ only in that score 0.909-0.951 on configs[1] (tools/map_noise.py,
    profiles/r06/map_noise.txt).  Measured on MI355X (round 6, printed with -s): configs[1] bf16
    device 0.917 vs the emulation's 0.951, configs[3] fp16 0.964 vs 0.974.  (Round 5's 0.867 came
    from folding BatchNorm from bf16-rounded parameters, fixed by the fp32 fold masters,
    models/yolox.py.)  Returns the numbers."""
    from oracle import reference_cpu as O
    ref_dets = O.postprocess(ref.copy(), 80, 0.5, 0.65)
    emu_dets = O.postprocess(emu.copy(), 80, 0.5, 0.65)
    self_ap = box_map_vs_oracle(ref_dets, ref_dets, size)
    dev_ap = box_map_vs_oracle(dev_dets, ref_dets, size)
    emu_ap = box_map_vs_oracle(emu_dets, ref_dets, size)
    print(f"{tag} box mAP vs the fp32 oracle's detections (AP50:95, AP50): device {dev_ap}, "
          f"oracle with 16-bit storage {emu_ap}, oracle self {self_ap}")
    assert self_ap[0] > 0.99 and self_ap[1] > 0.99  # the harness scores identical boxes as 1
    for k in (0, 1):
        assert 1.0 - dev_ap[k] <= MAP_FACTOR * (1.0 - emu_ap[k]) + 0.01, (dev_ap, emu_ap)
    assert dev_ap[0] >= MAP_FLOOR[tag][0] and dev_ap[1] >= MAP_FLOOR[tag][1], (dev_ap, MAP_FLOOR[tag])
    return dev_ap, emu_ap


# absolute floors (AP50:95, AP50) of the device detections vs the fp32 oracle's, and the factor on
# the 16-bit-storage emulation's AP loss (measured round 6: configs[1] 0.917 = 1.7x, configs[3] 0.964 = 1.4x;
# emulations differing only in summation order: 0.909-0.951 = up to 1.9x, tools/map_noise.py)
MAP_FLOOR = {"configs1": (0.90, 0.90), "configs3": (0.93, 0.93)}
MAP_FACTOR = 2.0
# the device's probability / box-centre distance from the fp32 oracle over the emulation's (measured
# round 6 with the fp32 fold masters: max 1.06x, p99 1.00x on configs[1]; 0.95x / 0.99x on configs[3])
DERIVED_FACTOR = 1.25


def test_configs1_yolox_s_640_bf16_batch32(oracle):
    from yolox_amd.utils.boxes import postprocess_device
    model, plan, imgs = bench_plan("yolox_s", 32, 640, torch.bfloat16)
    out = plan.replay()
    out2 = plan.replay().clone()
    torch.cuda.synchronize()
    assert torch.equal(out, out2)  # replays are deterministic
    host = out.cpu().numpy()
    # all 32 images.  The factor covers the summation order: the device's fp32 accumulations
    # run in another order than the oracle's, which flips the bf16 rounding of values near a
    # rounding boundary in every stored map.  Measured on MI355X (round 6, stats printed with -s):
    # max 1.06x, p99 1.00x the storage-only distance (round 5: 1.68x / 1.56x -- BN folded from
    # bf16-rounded parameters, see YoloxModule.fp32_master)
    ref = oracle_forward(oracle, "yolox_s", imgs)
    emu = oracle_forward(oracle, "yolox_s", imgs, torch.bfloat16)
    print("configs1 bf16 vs fp32 oracle (dev max, emu max, dev p99, emu p99):",
          derived_bounds_hold(host, ref, emu, DERIVED_FACTOR))
    # device NMS (bench step: conf 0.5, nms 0.65) on the replayed output == oracle NMS
    pred = out.clone()
    det, counts = postprocess_device(pred, 80, 0.5, 0.65)
    n = counts.cpu().numpy()
    want = oracle.postprocess(host.copy(), 80, 0.5, 0.65)
    np.testing.assert_array_equal(pred.cpu().numpy(), oracle_xyxy(host))
    dets = det.cpu().numpy()
    assert (n > 0).all()
    for b in range(32):
        np.testing.assert_array_equal(dets[b, :n[b]], want[b])
    map_parity(host, ref, emu, [dets[b, :n[b]] for b in range(32)], 640, "configs1")


def oracle_xyxy(host):
    x = host.copy()
    from oracle import reference_cpu as O
    O.xyxy_inplace(x)
    return x


def test_configs2_yolox_s_640_train_fp32_batch8(oracle, monkeypatch):
    """One fp32 train step at the configs[2] per-GPU workload.  SPP's max pools route
    gradients to one argmax per window; the device forward differs from the CPU's by fp32
    rounding (1.6e-5 absolute at the SPP input here), which flips the argmax of 4 of
    819200 near-tied 5x5 windows and moves upstream gradients by ~1e-2 -- a discrete
    effect any non-bit-identical forward has (tools/spp_argmax_check.py).  The oracle
    therefore takes the pooling ROUTING (which element is the max) from the device
    forward, its values from its own; everything else is independent."""
    import torch.nn.functional as F

    import yolox_amd.train as T
    from yolox_amd.models import YoloxModule
    from yolox_amd.weights import synthetic_images, synthetic_labels
    m = YoloxModule.synthetic("yolox_s", seed=0, device="cuda").train()
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    x = torch.from_numpy(synthetic_images(8, 640, 640, seed=1000)).permute(0, 3, 1, 2).float()
    labels = torch.from_numpy(synthetic_labels(8, 640, 640, seed=2000))
    spp_conv1, seen = m.backbone.backbone.dark5[1].conv1, {}
    base_conv = T.TrainGraph.base_conv

    def recording(self, mod, inputs, out=None, residual=None, cin_store=None):
        r = base_conv(self, mod, inputs, out, residual, cin_store)
        if mod is spp_conv1:
            seen["act"] = r
        return r

    monkeypatch.setattr(T.TrainGraph, "base_conv", recording)
    out = m(x.cuda(), labels.cuda())
    out["total_loss"].backward()
    torch.cuda.synchronize()
    a = seen["act"]
    gpu_pool_in = a.t[..., a.coff:a.coff + a.ch].permute(0, 3, 1, 2).cpu().float()
    max_pool2d = F.max_pool2d

    def pool_routed_like_device(t, k, stride=None, padding=0, **kw):
        _, idx = max_pool2d(gpu_pool_in, k, 1, k // 2, return_indices=True)
        return t.flatten(2).gather(2, idx.flatten(2)).view_as(idx)

    monkeypatch.setattr(F, "max_pool2d", pool_routed_like_device)
    sdo = {k: v.float().requires_grad_(v.is_floating_point() and "running" not in k and "num_batches" not in k)
           for k, v in sd.items()}
    torch.set_num_threads(16)
    ref = oracle.forward_train(sdo, oracle.ARCHS["yolox_s"], x, labels)
    ref["total_loss"].backward()
    for k in ("total_loss", "iou_loss", "conf_loss", "cls_loss", "num_fg"):
        assert float(out[k]) == pytest.approx(float(ref[k]), rel=1e-3, abs=1e-6), k
    worst = []
    for name, p in m.named_parameters():
        g, gr = p.grad.cpu(), sdo[name].grad
        e = float((g - gr).abs().max() / (gr.abs().max() + 1e-12))
        worst.append((e, name))
        assert e < 1e-3, (name, e)
    print("worst gradient rel err", max(worst))


def test_configs3_yolox_l_640_fp16_batch16(oracle):
    from yolox_amd.utils.boxes import postprocess_device
    model, plan, imgs = bench_plan("yolox_l", 16, 640, torch.float16)
    out = plan.replay()
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    torch.set_num_threads(16)
    ref = oracle_forward(oracle, "yolox_l", imgs)
    emu = oracle_forward(oracle, "yolox_l", imgs, torch.float16)
    print("configs3 fp16 vs fp32 oracle (dev max, emu max, dev p99, emu p99):",
          derived_bounds_hold(host, ref, emu, DERIVED_FACTOR))
    # device NMS (processor defaults conf 0.5, nms 0.65) on the replayed fp16-plan output
    pred = out.clone()
    det, counts = postprocess_device(pred, 80, 0.5, 0.65)
    n = counts.cpu().numpy()
    want = oracle.postprocess(host.copy(), 80, 0.5, 0.65)
    np.testing.assert_array_equal(pred.cpu().numpy(), oracle_xyxy(host))
    dets = det.cpu().numpy()
    assert (n > 0).all()
    for b in range(16):
        np.testing.assert_array_equal(dets[b, :n[b]], want[b])
    map_parity(host, ref, emu, [dets[b, :n[b]] for b in range(16)], 640, "configs3")


@pytest.mark.parametrize("seed", [0, 1])
def test_configs4_simota_1280_max_labels(oracle, seed):
    """yolox_x at 1280: A = 160^2 + 80^2 + 40^2 = 33600 anchors, G up to the 120-label cap."""
    from yolox_amd.models.losses import yolox_losses
    from yolox_amd.weights import synthetic_head_outputs, synthetic_labels
    B, S = 2, 1280
    bbox, cls, obj = synthetic_head_outputs(B, S, S, seed=300 + seed)
    labels = synthetic_labels(B, S, S, max_gt=120, seed=400 + seed)
    labels[0, :120, 0] = np.arange(120) % 80  # image 0: exactly 120 GTs
    rng = np.random.default_rng(seed)
    labels[0, :120, 1:3] = rng.uniform(100, 1180, (120, 2))
    labels[0, :120, 3:5] = rng.uniform(20, 320, (120, 2))
    out = torch.from_numpy(np.concatenate([bbox, obj, cls], -1))
    hw = [(160, 160), (80, 80), (40, 40)]
    losses, assign = yolox_losses(out.cuda(), torch.from_numpy(labels).cuda(), hw)
    torch.cuda.synchronize()
    xs, ys, st = oracle.level_grid(hw)
    lab = torch.from_numpy(labels)
    for b in range(B):
        G = int((lab[b].sum(1) > 0).sum())
        fg, matched, piou, _, nfg = oracle.simota_assign(lab[b, :G, 1:5], lab[b, :G, 0], out[b, :, :4],
                                                          out[b, :, 5:], out[b, :, 4:5], xs, ys, st)
        gfg = assign["fg_mask"][b].cpu().numpy()
        np.testing.assert_array_equal(gfg, fg.numpy())
        assert int(assign["num_fg"][b]) == nfg
        np.testing.assert_array_equal(assign["matched_gt_inds"][b].cpu().numpy()[gfg], matched.numpy())
        np.testing.assert_allclose(assign["pred_ious"][b].cpu().numpy()[gfg], piou.numpy(), rtol=1e-6, atol=0)
    ref = oracle.losses(out, None, lab, xs, ys, st)
    for k in ("total_loss", "iou_loss", "conf_loss", "cls_loss", "num_fg"):
        assert float(losses[k]) == pytest.approx(float(ref[k]), rel=1e-4, abs=1e-6), k


def _f(v) -> float:
    """A loss-dict value as a float (tensors may require grad; num_fg is a float)."""
    return float(v.detach()) if torch.is_tensor(v) else float(v)


def _oracle_train_step(oracle, monkeypatch, m, name, x, labels, spp_in, assign=None, flips=None):
    """The oracle's fp32 autograd train step on the module's own weights, with SPP's pooling
    ROUTING taken from the device forward (see configs[2]); returns (losses, sd).

    ``assign`` (the device's SimOTA result, TrainGraph.assign): the oracle's losses use the
    device's fg anchors and matched ground truths (their IoU targets from the oracle's own boxes)
    -- SimOTA's top-k / min-cost matching is discrete, so where the 16-bit forward moves a cost
    across a tie the two runs train different anchors and the losses differ by whole terms; the
    assignment itself is pinned exactly elsewhere (tests/test_gpu_train.py SimOTA vs the
    reference fixture, A = 33 600).  ``flips`` collects, per image, how many fg anchors the
    oracle's own assignment would change."""
    import torch.nn.functional as F
    sd = {k: v.detach().cpu().float().clone() for k, v in m.state_dict().items()}
    max_pool2d = F.max_pool2d

    def pool_routed_like_device(t, k, stride=None, padding=0, **kw):
        _, idx = max_pool2d(spp_in, k, 1, k // 2, return_indices=True)
        return t.flatten(2).gather(2, idx.flatten(2)).view_as(idx)

    monkeypatch.setattr(F, "max_pool2d", pool_routed_like_device)
    simota = oracle.simota_assign
    if assign is not None:
        fg_all = assign["fg_mask"].bool().cpu()
        matched_all = assign["matched_gt_inds"].long().cpu()
        imgs = [b for b in range(labels.shape[0]) if int((labels[b].sum(1) > 0).sum()) > 0]
        order = iter(imgs)

        def simota_routed_like_device(gt_boxes, gt_classes, pred_boxes, *rest):
            b = next(order)
            fg = fg_all[b]
            matched = matched_all[b][fg]
            ious = oracle.bboxes_iou(gt_boxes, pred_boxes[fg], False)
            piou = ious[matched, torch.arange(matched.numel())]
            if flips is not None:
                own_fg = simota(gt_boxes, gt_classes, pred_boxes, *rest)[0]
                flips.append(int((own_fg != fg).sum()))
            return fg, matched, piou, gt_classes[matched], int(fg.sum())

        monkeypatch.setattr(oracle, "simota_assign", simota_routed_like_device)
    sdo = {k: v.requires_grad_("running" not in k and "num_batches" not in k) for k, v in sd.items()}
    torch.set_num_threads(16)
    ref = oracle.forward_train(sdo, oracle.ARCHS[name], x, labels)
    ref["total_loss"].backward()
    monkeypatch.setattr(F, "max_pool2d", max_pool2d)
    monkeypatch.setattr(oracle, "simota_assign", simota)
    return ref, sdo


def _device_train_step(monkeypatch, m, x, labels, amp_dtype=None):
    import yolox_amd.train as T
    spp_conv1, seen = m.backbone.backbone.dark5[1].conv1, {}
    base_conv = T.TrainGraph.base_conv

    def recording(self, mod, inputs, out=None, residual=None, cin_store=None):
        r = base_conv(self, mod, inputs, out, residual, cin_store)
        if mod is spp_conv1:
            seen["act"] = r
        return r

    monkeypatch.setattr(T.TrainGraph, "base_conv", recording)
    m.zero_grad(set_to_none=True)
    if amp_dtype is None:
        out = m(x.cuda(), labels.cuda())
    else:
        with torch.autocast("cuda", dtype=amp_dtype):
            out = m(x.cuda().to(amp_dtype), labels.cuda())
    out["total_loss"].backward()
    torch.cuda.synchronize()
    monkeypatch.setattr(T.TrainGraph, "base_conv", base_conv)
    a = seen["act"]
    spp_in = a.t[..., a.coff:a.coff + a.ch].permute(0, 3, 1, 2).cpu().float()
    return out, spp_in


@pytest.mark.parametrize("name,size,dtype", [("yolox_s", 640, None), ("yolox_x", 1280, torch.float16)])
def test_every_training_candidate_tile_is_deterministic(monkeypatch, name, size, dtype):
    """Race detector for the training tuner's candidates at the benched shapes (configs[2]: yolox_s fp32
    batch 8; configs[4]: yolox_x 1280 --fp16 batch 8): the first step tunes every forward conv, data
    gradient and weight gradient shape, and with the check on every applicable candidate tile runs twice
    more into a zeroed sink and must write the same bytes both times (split-K partial sums are reduced in
    a fixed order, so even the accumulating forms are bit-stable)."""
    import yolox_amd.train as T
    from yolox_amd.models import YoloxModule
    from yolox_amd.weights import synthetic_images, synthetic_labels
    monkeypatch.setattr(T, "_TRAIN_TILES", {})
    monkeypatch.setattr(T, "_CHECK_DET", True)
    monkeypatch.setattr(T, "TUNE_DET_FAILURES", [])
    monkeypatch.setattr(T, "TUNE_DET_CHECKED", [0])
    B = 8
    m = YoloxModule.synthetic(name, seed=0, device="cuda").train()
    x = torch.from_numpy(synthetic_images(B, size, size, seed=5)).permute(0, 3, 1, 2).float().cuda()
    labels = torch.from_numpy(synthetic_labels(B, size, size, max_gt=120, seed=6)).cuda()
    m.zero_grad(set_to_none=True)
    if dtype is None:
        out = m(x, labels)
    else:
        with torch.autocast("cuda", dtype=dtype):
            out = m(x.to(dtype), labels)
    out["total_loss"].backward()
    torch.cuda.synchronize()
    print(f"{name}: {T.TUNE_DET_CHECKED[0]} (shape, tile) pairs checked, failures {T.TUNE_DET_FAILURES}")
    assert not T.TUNE_DET_FAILURES
    assert T.TUNE_DET_CHECKED[0] > 100


GRAD_NAMES = ("backbone.backbone.stem.conv.conv.weight", "backbone.backbone.dark2.0.conv.weight",
              "backbone.backbone.dark5.1.conv2.conv.weight", "backbone.C3_n4.conv3.conv.weight",
              "head.stems.0.conv.weight", "head.cls_convs.0.1.conv.weight", "head.cls_preds.0.weight",
              "head.reg_preds.1.weight", "head.obj_preds.2.bias", "head.stems.2.bn.weight")


def test_configs4_yolox_x_1280_train_step_fp32_batch8_vs_oracle(oracle, monkeypatch):
    """configs[4]'s model and image size (yolox_x, 1280x1280, up to 120 labels) at its per-GPU
    batch (-d 8 -b 64: 8 images per rank; the loss is per rank, trainer.py:168-169): fp32 losses
    within 1e-3 of the oracle (north_star tolerance) and named gradients within 1e-3 of each
    tensor's max.  The oracle's fp32 autograd at batch 8 holds ~25 GB of host memory and runs
    ~1 min on the box's 16 threads."""
    from yolox_amd.models import YoloxModule
    from yolox_amd.weights import synthetic_images, synthetic_labels
    B = 8
    m = YoloxModule.synthetic("yolox_x", seed=0, device="cuda").train()
    x = torch.from_numpy(synthetic_images(B, 1280, 1280, seed=5)).permute(0, 3, 1, 2).float()
    labels = torch.from_numpy(synthetic_labels(B, 1280, 1280, max_gt=120, seed=6))
    labels[0, :120, 0] = torch.arange(120) % 80  # image 0 at the 120-label cap
    g = torch.Generator().manual_seed(7)
    labels[0, :120, 1:3] = torch.rand(120, 2, generator=g) * 1080 + 100
    labels[0, :120, 3:5] = torch.rand(120, 2, generator=g) * 300 + 20
    out, spp_in = _device_train_step(monkeypatch, m, x, labels)
    grads = {n: p.grad.cpu().clone() for n, p in m.named_parameters() if n in GRAD_NAMES}
    ref, sdo = _oracle_train_step(oracle, monkeypatch, m, "yolox_x", x, labels, spp_in)
    for k in ("total_loss", "iou_loss", "conf_loss", "cls_loss", "num_fg"):
        assert float(out[k]) == pytest.approx(_f(ref[k]), rel=1e-3, abs=1e-6), k
    assert float(out["num_fg"]) > 0
    worst = []
    for name in GRAD_NAMES:
        g, gr = grads[name], sdo[name].grad
        e = float((g - gr).abs().max() / (gr.abs().max() + 1e-12))
        worst.append((e, name))
        assert e < 1e-3, (name, e)
    print("configs4 fp32 batch 8: worst gradient rel err", max(worst))


def test_configs4_yolox_x_1280_train_step_fp16_derived_bound(oracle, monkeypatch):
    """The --fp16 (autocast) step of configs[4] at the benched per-GPU batch (yolox_x 1280, batch 8
    = -d 8 -b 64, with the tiles the training tuner picks for it, as the bench's: the nine-tap
    16-bit weight gradient wgrad9t_h and its 64 MiB partials cap) against the oracle's fp32
    autograd, within bounds DERIVED from the oracle itself run with 16-bit storage
    (oracle.stored_as(float16) in train mode: fp16 image, conv weights, conv outputs and block
    outputs, fp32 sums and BN statistics): each loss and each named gradient may be off the fp32
    oracle by at most FACTOR x the emulation's own distance from it (+ 1e-3 of the tensor's max,
    the fp32 noise floor), both oracle runs on the device's SimOTA assignment (it is discrete:
    _oracle_train_step).  The factor covers what the emulation does not model -- 16-bit
    backward maps and the device's summation order; measured on MI355X at batch 2 (round 4,
    printed with -s): 1.9x at worst (the stem weight's gradient, 0.147 vs 0.077 of its max;
    obj_preds.2.bias 2.8x of a 4e-5 distance, under the floor), losses within 0.1x.  Host memory:
    the two oracle runs (fp32, fp16 storage) at batch 8 hold ~25 GB each, one after the other."""
    from yolox_amd.models import YoloxModule
    from yolox_amd.weights import synthetic_images, synthetic_labels
    FACTOR = 3.0
    B = 8
    m = YoloxModule.synthetic("yolox_x", seed=0, device="cuda").train()
    x = torch.from_numpy(synthetic_images(B, 1280, 1280, seed=5)).permute(0, 3, 1, 2).float()
    labels = torch.from_numpy(synthetic_labels(B, 1280, 1280, max_gt=120, seed=6))
    out16, spp_in = _device_train_step(monkeypatch, m, x, labels, torch.float16)
    assign = {k: v.clone() for k, v in m._train_graph.assign.items()}
    grads = {n: p.grad.cpu().float().clone() for n, p in m.named_parameters() if n in GRAD_NAMES}
    for n, p in m.named_parameters():
        assert torch.isfinite(p.grad).all(), n
    flips = []
    ref, sdo = _oracle_train_step(oracle, monkeypatch, m, "yolox_x", x, labels, spp_in, assign, flips)
    ref_grads = {n: sdo[n].grad.clone() for n in GRAD_NAMES}
    nfg = int(assign["fg_mask"].bool().sum())
    # the device's assignment agrees with the fp32 oracle's own on all but a few anchors (a swapped anchor
    # counts twice; measured on MI355X: 15 of 577 fg anchors over the 8 images)
    assert sum(flips) <= 0.05 * nfg, (flips, nfg)
    with oracle.stored_as(torch.float16):
        emu, sde = _oracle_train_step(oracle, monkeypatch, m, "yolox_x", x, labels, spp_in, assign)
    stats = {}
    for k in ("total_loss", "iou_loss", "conf_loss", "cls_loss"):
        r = _f(ref[k])
        d_dev, d_emu = abs(float(out16[k]) - r), abs(_f(emu[k]) - r)
        stats[k] = (d_dev / abs(r), d_emu / abs(r))
        assert d_dev <= FACTOR * d_emu + 1e-3 * abs(r), (k, stats[k])
    for name in GRAD_NAMES:
        gr = ref_grads[name]
        scale = float(gr.abs().max()) + 1e-12
        d_dev = float((grads[name] - gr).abs().max()) / scale
        d_emu = float((sde[name].grad - gr).abs().max()) / scale
        stats[name] = (d_dev, d_emu)
        assert d_dev <= FACTOR * d_emu + 1e-3, (name, stats[name], stats)
    print("configs4 fp16 (dev, emulation) distances from the fp32 oracle:", stats,
          f"(SimOTA routed from the device; the oracle's own assignment differs on {flips} of {nfg} fg anchors)")


def test_configs0_yolox_tiny_416_single_image(golden, oracle, tmp_path):
    """BASELINE configs[0]: Yolox.from_pretrained(<local checkpoint>, config) + Yolox.__call__
    on one 416x416 image (r == 1), against the reference's own run (fixture) and the oracle."""
    from PIL import Image

    from yolox_amd.config import YoloxConfig
    from yolox_amd.models import Yolox, YoloxModule
    d = golden("processor_yolox_tiny_416.npz")
    ckpt = tmp_path / "yolox_tiny.pth"
    syn = YoloxModule.synthetic("yolox_tiny", seed=0, device="cuda")
    torch.save({"model": {k: v.cpu() for k, v in syn.state_dict().items()}}, ckpt)
    yolox = Yolox.from_pretrained(str(ckpt), config=YoloxConfig.get_named_config("yolox_tiny"), device="cuda")
    im = Image.open(os.path.join(GOLDEN, "images", "000000000001.jpg")).convert("RGB").crop((0, 0, 416, 416))
    for thr in (0.5, 0.3):
        (det,) = yolox([im], threshold=thr)
        assert det["labels"] == d[f"t{thr}.labels"].tolist()
        np.testing.assert_allclose(np.array(det["bboxes"]).reshape(-1, 4), d[f"t{thr}.bboxes"], atol=1e-2, rtol=0)
        np.testing.assert_allclose(det["scores"], d[f"t{thr}.scores"], atol=1e-4, rtol=0)
    # the same device output through the oracle's NMS + the reference formatting: identical
    out = yolox.module(yolox.processor([im]))
    (rows,) = oracle.postprocess(out.cpu().numpy().copy(), 80, 0.5, 0.65)
    assert yolox.processor.postprocess([im], out, threshold=0.5) == [
        oracle.detections(rows, (416, 416), (416, 416))]
