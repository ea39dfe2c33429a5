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
