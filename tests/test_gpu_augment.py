"""GPU parity of the training augmentation kernels (csrc/augment.hip via yxh_augment_batch):
bit-exact against tests/golden/mosaic_aug.npz (the reference's own MosaicDetection /
TrainTransform code over the oracle's cv2 restatement) and against the oracle's composition
(oracle/augment_oracle.py render) at the training sizes (640 default config, 416 nano
config, close_mosaic).  Pixels are integers in float32, so every comparison is exact."""
import random

import numpy as np
import pytest
import torch

from augment_common import CASES, SEEDS, ArrayDataset, load_fixture
from oracle import augment_oracle as A
from yolox_amd.data import mosaic as M

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", list(CASES))
def test_fixture_batch_bit_exact(case):
    g, images, labels = load_fixture()
    H, W = (int(v) for v in g["input_hw"])
    ds = M.GpuMosaicDetection(ArrayDataset(images, labels), (H, W), preproc=M.TrainTransform(max_labels=120),
                              device="cuda", **CASES[case])
    drawn = []
    for s in range(SEEDS):
        random.seed(1000 + s)
        np.random.seed(1000 + s)
        drawn.append(ds.draw(s % len(ds)))
    out = ds.render([p for p, _ in drawn]).cpu().numpy()
    for s, (_, lab) in enumerate(drawn):
        np.testing.assert_array_equal(out[s].astype(np.uint8), g[f"{case}.{s}.image"], err_msg=f"{case} seed {s}")
        np.testing.assert_array_equal(out[s], np.round(out[s]))
        np.testing.assert_array_equal(lab, g[f"{case}.{s}.labels"])


def test_getitem_matches_reference_item():
    """__getitem__ returns the reference's 4-tuple: image, padded labels, img_info, img_id."""
    g, images, labels = load_fixture()
    H, W = (int(v) for v in g["input_hw"])
    ds = M.GpuMosaicDetection(ArrayDataset(images, labels), (H, W), preproc=M.TrainTransform(max_labels=120),
                              device="cuda", **CASES["nano"])
    for s in range(SEEDS):
        random.seed(1000 + s)
        np.random.seed(1000 + s)
        img, lab, info, img_id = ds[s % len(ds)]
        np.testing.assert_array_equal(img.cpu().numpy().astype(np.uint8), g[f"nano.{s}.image"])
        np.testing.assert_array_equal(lab, g[f"nano.{s}.labels"])
        np.testing.assert_array_equal(np.array(info, np.int64), g[f"nano.{s}.info"])
        np.testing.assert_array_equal(np.array(img_id, np.int64).reshape(-1), g[f"nano.{s}.id"])


@pytest.mark.parametrize("hw,case,batch", [((640, 640), "default", 8), ((416, 416), "nano", 8),
                                           ((640, 640), "no_aug", 6), ((384, 640), "default", 4)])
def test_training_sizes_vs_oracle(hw, case, batch):
    H, W = hw
    src = M.SyntheticDetectionDataset(24, hw, seed=11, min_side=40, max_side=1100)
    ds = M.GpuMosaicDetection(src, hw, preproc=M.TrainTransform(max_labels=120), device="cuda", **CASES[case])
    rnd, nrnd = random.Random(5), np.random.RandomState(5)
    ds.random, ds.np_random = rnd, nrnd
    drawn = [ds.draw(i) for i in range(batch)]
    out = ds.render([p for p, _ in drawn]).cpu().numpy()
    images = [src.pull_item(i)[0] for i in range(len(src))]
    for b, (p, _) in enumerate(drawn):
        ref = A.render(p, images, H, W)
        diff = np.argwhere(out[b] != ref)
        assert diff.size == 0, f"sample {b} ({p.mosaic=}, {p.mix=}): {len(diff)} px differ, first {diff[:4]}"


def test_mosaic_batches_loader():
    """The trainer's loader: InfiniteSampler indices -> device images + targets."""
    from yolox_amd.trainer import InfiniteSampler
    src = M.SyntheticDetectionDataset(40, (320, 320), seed=2)
    ds = M.GpuMosaicDetection(src, (320, 320), preproc=M.TrainTransform(max_labels=120), device="cuda")
    loader = M.MosaicBatches(ds, InfiniteSampler(len(ds), seed=0), batch_size=6)
    imgs, targets = loader.next()
    assert imgs.shape == (6, 3, 320, 320) and imgs.dtype == torch.float32 and imgs.is_cuda
    assert targets.shape == (6, 120, 5) and targets.is_cuda
    assert float(imgs.min()) >= 0 and float(imgs.max()) <= 255
    loader.close_mosaic()
    imgs2, _ = loader.next()
    assert imgs2.shape == imgs.shape and not ds.enable_mosaic


def test_rejects_bad_output():
    g, images, labels = load_fixture()
    H, W = (int(v) for v in g["input_hw"])
    ds = M.GpuMosaicDetection(ArrayDataset(images, labels), (H, W), device="cuda")
    p, _ = ds.draw(0)
    with pytest.raises(ValueError):
        ds.render([p], out=torch.empty((1, 3, H, W + 1), device="cuda"))


# ------------------------------------------------------------------ multiscale resize
def test_preprocess_resize_matches_reference_fixture(golden):
    """YoloxConfig.preprocess (config.py:296-305) with the HIP resize (yxh_resize_bilinear) vs the
    reference's own preprocess run on CPU (tests/golden/resize_preprocess.npz): labels exact;
    pixels within a few fp32 ulps of the CPU run (ATen's CPU kernel contracts the bilinear sum
    differently from its GPU kernel, to which the device result is bit-exact -- next test)."""
    from yolox_amd.config import named_config
    d = golden("resize_preprocess.npz")
    cfg = named_config("yolox_s")
    cfg.input_size = (160, 160)
    x = torch.from_numpy(d["input_u8"]).float().cuda()
    for key in [k[:-6] for k in d if k.endswith(".image")]:
        size = tuple(int(v) for v in key.split("x"))
        y, t = cfg.preprocess(x.clone(), torch.from_numpy(d["targets"]).cuda(), size)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(t.cpu().numpy(), d[f"{key}.targets"])
        want = d[f"{key}.image"]
        assert y.shape == want.shape and y.dtype == torch.float32
        np.testing.assert_allclose(y.cpu().numpy(), want, rtol=0, atol=1e-4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_resize_bilinear_bit_exact_vs_aten_on_device(dtype):
    """The reference's call itself, F.interpolate(bilinear, align_corners=False), on this GPU
    (ATen's HIP kernel) against yxh_resize_bilinear: bit-identical over the yolox_s multiscale
    range at the training batch shape (640 -> 480..800 in steps of 32, trainer.py:83 + config.py:
    275-294), non-square sizes, odd sizes and the same-size copy; fp32, and fp16 / bf16 (--fp16
    resizes the half batch)."""
    import torch.nn.functional as F
    from yolox_amd.utils.resize import resize_bilinear
    g = torch.Generator().manual_seed(3)
    x = (torch.rand(2, 3, 640, 640, generator=g) * 255).round().to(dtype).cuda()
    sizes = [(s, s) for s in range(480, 801, 32)] + [(640, 640), (608, 672), (353, 517), (17, 23), (1, 1)]
    for size in sizes:
        got = resize_bilinear(x, size)
        want = F.interpolate(x, size=size, mode="bilinear", align_corners=False)
        assert got.shape == want.shape
        assert torch.equal(got, want), (size, float((got.float() - want.float()).abs().max()))
    small = torch.rand(1, 5, 7, 9, generator=g).to(dtype).cuda()  # C != 3, upsample from tiny maps
    for size in [(14, 18), (3, 4), (21, 5)]:
        assert torch.equal(resize_bilinear(small, size),
                           F.interpolate(small, size=size, mode="bilinear", align_corners=False)), size
