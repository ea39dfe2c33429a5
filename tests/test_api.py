"""Host-side API surface (no GPU): configs, module tree, loaders, planner."""
import json
import os

import pytest
import torch

from conftest import GOLDEN


def test_named_configs_are_singletons_and_accept_dash():
    from yolox_amd.config import YoloxConfig
    a = YoloxConfig.get_named_config("yolox-s")
    assert a is YoloxConfig.get_named_config("yolox_s")
    assert (a.depth, a.width) == (0.33, 0.50)
    assert YoloxConfig.get_named_config("nope") is None
    t = YoloxConfig.get_named_config("yolox_tiny")
    assert t.test_size == (416, 416) and t.width == 0.375
    assert YoloxConfig.get_named_config("yolox_nano").depthwise


def test_config_update_coercion():
    from yolox_amd.config import named_config
    c = named_config("yolox_s")
    c.update({"max_epoch": "10", "test_size": "(320, 320)", "seed": "7", "nmsthre": "0.5"})
    assert c.max_epoch == 10 and c.test_size == (320, 320) and c.seed == 7 and c.nmsthre == 0.5
    with pytest.raises(AttributeError):
        c.update({"bogus": "1"})


@pytest.mark.parametrize("name", ["yolox_s", "yolox_m", "yolox_l", "yolox_x", "yolox_tiny", "yolox_nano"])
def test_state_dict_matches_reference_checkpoint_layout(name):
    from yolox_amd.config import named_config
    with open(os.path.join(GOLDEN, "state_dict_shapes.json")) as f:
        ref = {k: tuple(s) for k, s in json.load(f)[name]}
    m = named_config(name).get_model()
    mine = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert mine == ref


def test_get_model_initialisation():
    from yolox_amd.config import named_config
    m = named_config("yolox_s").get_model()
    bns = [x for x in m.modules() if isinstance(x, torch.nn.BatchNorm2d)]
    assert bns and all(b.eps == 1e-3 and b.momentum == 0.03 for b in bns)
    assert torch.allclose(m.head.cls_preds[0].bias, torch.full((80,), -4.59511985))
    assert m.training


def test_from_pretrained_errors(tmp_path):
    from yolox_amd.models import YoloxModule
    with pytest.raises(ValueError, match="Unknown model"):
        YoloxModule.from_pretrained("yolox_q")
    f = tmp_path / "w.pth"
    f.write_bytes(b"0")
    with pytest.raises(ValueError, match="config must be provided"):
        YoloxModule.from_pretrained(str(f))
    os.environ["YOLOX_HOME"] = str(tmp_path)
    with pytest.raises(FileNotFoundError):
        YoloxModule.from_pretrained("yolox_s")


def test_from_pretrained_loads_local_checkpoint(tmp_path):
    from yolox_amd.config import named_config
    from yolox_amd.models import YoloxModule
    from yolox_amd.weights import synthetic_state_dict
    cfg = named_config("yolox_nano")
    sd = synthetic_state_dict(cfg.get_model().state_dict(), seed=3)
    torch.save({"model": sd}, tmp_path / "nano.pth")
    # the HIP path has no CPU execution: a CPU device is refused at load, not at the first forward
    with pytest.raises(RuntimeError, match="ROCm device"):
        YoloxModule.from_pretrained(str(tmp_path / "nano.pth"), named_config("yolox_nano"), device="cpu")
    m = YoloxModule.load_checkpoint(str(tmp_path / "nano.pth"), named_config("yolox_nano"))
    assert not m.training
    assert torch.equal(m.state_dict()["head.cls_preds.1.weight"], sd["head.cls_preds.1.weight"])
    with pytest.raises(RuntimeError, match="ROCm device"):
        m(torch.zeros(1, 3, 64, 64))


def test_processor_rejects_bad_config():
    from yolox_amd.models import YoloxProcessor
    with pytest.raises(ValueError, match="string or YoloxConfig"):
        YoloxProcessor(3)
    assert YoloxProcessor("yolox-tiny").config.test_size == (416, 416)


def test_bboxes_iou_matches_reference_fixture(golden):
    from yolox_amd.utils import bboxes_iou
    d = golden("boxes.npz")
    t = torch.from_numpy
    assert torch.equal(bboxes_iou(t(d["a_xyxy"]), t(d["b_xyxy"]), True), t(d["iou_xyxy"]))
    assert torch.equal(bboxes_iou(t(d["a_c"]), t(d["b_c"]), False), t(d["iou_c"]))
    with pytest.raises(IndexError):
        bboxes_iou(torch.zeros(2, 3), torch.zeros(2, 4))


@pytest.mark.parametrize("name,hw,gflop,anchors", [
    ("yolox_s", 640, 26.69, 8400), ("yolox_tiny", 416, 6.41, 3549), ("yolox_nano", 416, 1.05, 3549),
    ("yolox_l", 640, 155.29, 8400), ("yolox_x", 1280, 1125.64, 33600)])
def test_planner_topology_and_flops(name, hw, gflop, anchors):
    """The plan covers every conv of the reference (SURVEY.md Appendix A counts)."""
    from yolox_amd.config import named_config
    from yolox_amd.engine import OutBuffer, PlanCtx
    m = named_config(name).get_model()
    ctx = PlanCtx(1, torch.bfloat16, torch.device("cpu"))
    feats = m.backbone.plan(ctx, ctx.image(hw, hw))
    A = sum(f.lh * f.lw for f in feats)
    m.head.plan(ctx, feats, OutBuffer(A, 85))
    assert A == anchors
    assert round(ctx.flops / 1e9, 2) == gflop
    n_bn_convs = sum(1 for x in m.modules() if x.__class__.__name__ == "BaseConv")
    n_csp = sum(1 for x in m.modules() if x.__class__.__name__ == "CspLayer")
    fused_head = 0 if m.backbone.backbone.stem.conv.conv.groups != 1 or name == "yolox_nano" else 3
    # every BaseConv is planned; CSP conv1|conv2 and head cls0|reg0 are stacked into one
    # launch each; + (reg|obj, cls) preds x 3 levels
    # ... and Focus + stem conv is one fused op (kind 3) when the stem width allows; a
    # level's three preds + decode are one head op (kind 4) when its rows are 16-byte
    # aligned and the head width is 64/128/256 (else two decode convs: reg|obj, cls)
    # ... and with the uint8 NHWC input the default context assumes, yolox_s's Focus stem +
    # dark2[0] are one yxh_stem_s2 op (kind 5) instead (stem 32 -> 64 channels only)
    kinds = [o.kind for o in ctx.ops]
    s2 = kinds.count(5)
    assert s2 == (1 if name == "yolox_s" else 0)
    assert kinds.count(3) + s2 == 1
    heads = kinds.count(4)
    # ... and with 128-channel head convs (yolox_s) each level's preds ride in its two-group
    # cls_convs[k][1] | reg_convs[k][1] launch instead (conv_ws head form)
    n_head_post = sum(1 for o in ctx.ops if o.args.get("head_post") is not None)
    from yolox_amd import engine as E  # YOLOX_AMD_HEAD_FUSION: the levels planned in the head form
    assert n_head_post == (len(E._HEAD_FUSION & {0, 1, 2}) if name == "yolox_s" else 0)
    if name in ("yolox_s", "yolox_l"):  # head widths 128 / 256 (yolox_x: 320, unfused)
        assert heads + n_head_post == 3
    # ... and a 16-bit plan folds each fusable Bottleneck's conv1 into its 3x3 (one op)
    n_fused_bneck = sum(1 for o in ctx.ops if o.args.get("pre_spec") is not None)
    n_bneck = sum(1 for x in m.modules() if x.__class__.__name__ == "Bottleneck")
    assert n_fused_bneck == sum(1 for x in m.modules() if x.__class__.__name__ == "Bottleneck"
                                and ctx.bottleneck_fusable(x)) <= n_bneck
    # ... and a 16-bit plan runs cls_convs[k][1] | reg_convs[k][1] as one two-group launch
    n_grouped = sum(1 for o in ctx.ops if o.args.get("grouped2"))
    assert n_grouped == (3 if name in ("yolox_s", "yolox_l") else n_grouped)
    # ... and yolox_s's dark2 CspLayer conv1 | conv2 and first Bottleneck conv1 ride in the
    # stem_s2 launch (its CSP form: two conv ops fewer)
    n_stem_csp = sum(1 for o in ctx.ops if o.kind == 5 and o.args.get("dst") is None)
    assert n_stem_csp == (1 if name == "yolox_s" else 0)
    # ... and 16-bit convs followed by a 1x1 that fits a conv_ws post tile (a Bottleneck 3x3 +
    # CspLayer.conv3, a stride-2 stage conv + its CspLayer conv1 | conv2, a Bottleneck 3x3 + the
    # next Bottleneck's conv1: dark3's and dark4's chains of three) are one op each
    n_post = sum(1 for o in ctx.ops if o.args.get("post_spec") is not None)
    n_chain = sum(1 for o in ctx.ops if o.args.get("post_store_out") is not None)
    assert n_post == (8 if name == "yolox_s" else n_post)
    assert n_chain == (4 if name == "yolox_s" else n_chain)
    assert (kinds.count(0) == n_bn_convs - n_csp - fused_head + 2 * (3 - heads - n_head_post) - 1 - n_fused_bneck
            - n_grouped
            - s2 - 2 * n_stem_csp - n_post)


def test_planner_fused_bottleneck_ping_pong():
    """Plan(fuse_bottleneck=True): every fusable Bottleneck (C 32/64/128, 3x3 s1 conv2) is one
    conv op carrying conv1 as pre_spec; no fused op writes the buffer it reads (neighbouring
    tiles read its halo), and after an odd chain CspLayer.conv3 reads [last | x_2] as two
    sources."""
    from yolox_amd.config import named_config
    from yolox_amd.engine import OutBuffer, PlanCtx
    m = named_config("yolox_s").get_model()
    ctx = PlanCtx(1, torch.bfloat16, torch.device("cpu"), fuse_bottleneck=True)
    feats = m.backbone.plan(ctx, ctx.image(640, 640))
    m.head.plan(ctx, feats, OutBuffer(sum(f.lh * f.lw for f in feats), 85))
    fused = [o for o in ctx.ops if o.args.get("pre_spec") is not None]
    assert len(fused) == 10 and {o.args["cin"] for o in fused} == {32, 64, 128}
    for o in fused:
        src, out = o.args["srcs"][0], o.args["out"]
        assert o.args["k"] == 3 and o.args["stride"] == 1 and len(o.args["srcs"]) == 1
        assert not (out.buf is src.buf and out.coff < src.coff + src.ch and src.coff < out.coff + out.ch)
        if o.args["residual"] is not None:
            assert o.args["residual"] is src
    two_src_1x1 = [o for o in ctx.ops if o.kind == 0 and o.args["k"] == 1 and len(o.args["srcs"]) == 2
                   and not any(s.up for s in o.args["srcs"])]
    assert len(two_src_1x1) == 6  # dark2/3/4, C3_p4, C3_p3, C3_n3: n = 1 or 3, odd
    assert round(ctx.flops / 1e9, 2) == 26.69  # same algorithmic work as the split plan
    fp32 = PlanCtx(1, torch.float32, torch.device("cpu"), fuse_bottleneck=True)
    feats = m.backbone.plan(fp32, fp32.image(640, 640))
    assert not any(o.args.get("pre_spec") is not None for o in fp32.ops)  # 16-bit only


def test_synthetic_weights_are_deterministic():
    from yolox_amd.weights import synthetic_state_dict
    shapes = {"a.conv.weight": (4, 3, 3, 3), "a.bn.weight": (4,), "head.cls_preds.0.bias": (80,)}
    a = synthetic_state_dict(shapes, seed=1)
    b = synthetic_state_dict(dict(reversed(list(shapes.items()))), seed=1)
    for k in shapes:
        assert torch.equal(a[k], b[k])
    assert not torch.equal(a["a.conv.weight"], synthetic_state_dict(shapes, seed=2)["a.conv.weight"])


def test_fp32_fold_masters_survive_the_16bit_cast():
    """Perf mode (.to(bfloat16)) keeps each parameter's / BN statistic's float32 value as the fold
    master (models/yolox.py: the plan folds BN from it, so packed weights are rounded once); a moved
    module keeps them, an edited parameter or a float32 module has none, and a float32 state dict
    loaded into a 16-bit module becomes the masters."""
    from yolox_amd.config import named_config
    from yolox_amd.weights import synthetic_state_dict
    m = named_config("yolox_nano").get_model()
    sd = synthetic_state_dict(m.state_dict(), seed=0, bn_stats="yolox_nano")
    m.load_state_dict(sd)
    conv, bn = m.backbone.backbone.stem.conv.conv, m.backbone.backbone.stem.conv.bn
    assert m.fp32_master(conv.weight) is None  # float32 module: folds from the parameters themselves
    m = m.to(torch.bfloat16)
    assert conv.weight.dtype == torch.bfloat16
    for t, k in ((conv.weight, "backbone.backbone.stem.conv.conv.weight"),
                 (bn.running_var, "backbone.backbone.stem.conv.bn.running_var"),
                 (bn.bias, "backbone.backbone.stem.conv.bn.bias")):
        assert torch.equal(m.fp32_master(t), sd[k].float()), k
    m = m.to(torch.float16)  # 16 -> 16 bit: the float32 masters carry over
    assert torch.equal(m.fp32_master(conv.weight), sd["backbone.backbone.stem.conv.conv.weight"])
    with torch.no_grad():
        conv.weight.mul_(2)  # an edit: the plan must fold from the edited value
    assert m.fp32_master(conv.weight) is None
    assert m.fp32_master(bn.weight) is not None
    m.load_state_dict(sd)  # float32 values into the 16-bit module: masters again
    assert torch.equal(m.fp32_master(conv.weight), sd["backbone.backbone.stem.conv.conv.weight"])
    m = m.float()
    assert m.fp32_master(conv.weight) is None
