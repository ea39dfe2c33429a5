"""CPU tests of the training augmentation pipeline (§8(f)-4): the host half of
yolox_amd.data.mosaic (random draws in the reference's order + label arithmetic) and the
oracle's image composition (oracle/augment_oracle.py) against tests/golden/mosaic_aug.npz --
samples produced by the reference's own MosaicDetection.__getitem__ / mixup / TrainTransform
with the oracle's cv2 restatement substituted for cv2 (parity vs cv2's pixels is unpinned:
cv2 is absent).  The device kernels are checked against the same fixture in
test_gpu_augment.py."""
import random

import numpy as np
import pytest

from augment_common import CASES, SEEDS, ArrayDataset, load_fixture
from oracle import augment_oracle as A
from yolox_amd.data import mosaic as M


@pytest.fixture(scope="module")
def fixture():
    return load_fixture()


def _dataset(fixture, case):
    g, images, labels = fixture
    ds = ArrayDataset(images, labels)
    res = M.ResidentImages(ds, device="cpu")
    H, W = (int(v) for v in g["input_hw"])
    return M.GpuMosaicDetection(ds, (H, W), preproc=M.TrainTransform(max_labels=120), resident=res,
                                **CASES[case]), images, H, W


@pytest.mark.parametrize("case", list(CASES))
def test_draws_and_labels_match_reference(fixture, case):
    g = fixture[0]
    ds, _, _, _ = _dataset(fixture, case)
    for s in range(SEEDS):
        random.seed(1000 + s)
        np.random.seed(1000 + s)
        _, lab = ds.draw(s % len(ds))
        np.testing.assert_array_equal(lab, g[f"{case}.{s}.labels"], err_msg=f"{case} seed {s}")


@pytest.mark.parametrize("case", list(CASES))
def test_oracle_render_matches_reference(fixture, case):
    g = fixture[0]
    ds, images, H, W = _dataset(fixture, case)
    kinds = set()
    for s in range(SEEDS):
        random.seed(1000 + s)
        np.random.seed(1000 + s)
        p, _ = ds.draw(s % len(ds))
        kinds.add((p.mosaic, p.mix, p.flip, p.do_hsv))
        img = A.render(p, images, H, W)
        np.testing.assert_array_equal(img.astype(np.uint8), g[f"{case}.{s}.image"], err_msg=f"{case} seed {s}")
    assert len(kinds) >= 2  # the seeds exercise more than one branch


def test_fixture_covers_branches(fixture):
    """The fixture exercises mosaic + mixup, mosaic without mixup, the letterbox path, both
    mirror states, HSV on/off and the empty-label image."""
    seen = set()
    for case in CASES:
        ds, _, _, _ = _dataset(fixture, case)
        for s in range(SEEDS):
            random.seed(1000 + s)
            np.random.seed(1000 + s)
            p, lab = ds.draw(s % len(ds))
            seen |= {("mosaic", p.mosaic), ("mix", p.mix), ("flip", p.flip), ("hsv", p.do_hsv),
                     ("empty", not lab.any())}
    for k in ("mosaic", "mix", "flip", "hsv"):
        assert (k, True) in seen and (k, False) in seen, k
    assert ("empty", True) in seen


def test_getitem_index_pair_sets_mosaic(fixture):
    """mosaic_getitem (datasets_wrapper.py:98-122): an (enable_mosaic, index) pair switches mosaic."""
    ds, _, _, _ = _dataset(fixture, "default")
    ds.enable_mosaic = True
    with pytest.raises(ValueError):  # rendering needs the device pool: no CPU image path
        ds[(False, 0)]
    assert ds.enable_mosaic is False


# ----------------------------------------------------------------- cv2 restatement properties
def test_resize_paths():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (20, 30, 3), dtype=np.uint8)
    np.testing.assert_array_equal(A.resize(img, (30, 20)), img)  # same size: copy
    half = A.resize(img, (15, 10))  # exact 2x down: INTER_AREA mean with rounding
    exp = ((img[0::2, 0::2].astype(int) + img[0::2, 1::2] + img[1::2, 0::2] + img[1::2, 1::2] + 2) >> 2)
    np.testing.assert_array_equal(half, exp.astype(np.uint8))
    flat = np.full((7, 9, 3), 77, np.uint8)
    np.testing.assert_array_equal(A.resize(flat, (23, 11)), np.full((11, 23, 3), 77, np.uint8))


def test_warp_affine_identity_and_shift():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (12, 17, 3), dtype=np.uint8)
    eye = np.array([[1.0, 0, 0], [0, 1.0, 0]])
    np.testing.assert_array_equal(A.warpAffine(img, eye, (17, 12)), img)
    shift = np.array([[1.0, 0, 3], [0, 1.0, -2]])  # integer translation: shifted copy, border 114
    out = A.warpAffine(img, shift, (17, 12))
    np.testing.assert_array_equal(out[:10, 3:], img[2:, :14])
    assert (out[:, :3] == 114).all() and (out[10:] == 114).all()


def test_hsv_known_colours():
    bgr = np.array([[[0, 0, 255], [0, 255, 0], [255, 0, 0], [255, 255, 255], [0, 0, 0], [128, 128, 128]]],
                   np.uint8)
    hsv = A.bgr2hsv(bgr)
    np.testing.assert_array_equal(hsv[0], [[0, 255, 255], [60, 255, 255], [120, 255, 255], [0, 0, 255], [0, 0, 0],
                                           [0, 0, 128]])
    np.testing.assert_array_equal(A.hsv2bgr(hsv), bgr)
    np.testing.assert_array_equal(A.apply_hsv(bgr, (0, 0, 0)), bgr)  # zero gains: exact for these


def test_hsv_roundtrip_close():
    """8-bit HSV round trip is lossy in cv2 too; it stays within a few levels."""
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (32, 32, 3), dtype=np.uint8)
    back = A.hsv2bgr(A.bgr2hsv(img))
    assert np.abs(back.astype(int) - img).max() <= 6


def test_synthetic_detection_dataset():
    ds = M.SyntheticDetectionDataset(16, (96, 128), seed=3)
    shapes = set()
    for i in range(len(ds)):
        img, lab, info, img_id = ds.pull_item(i)
        assert img.dtype == np.uint8 and img.shape[2] == 3
        assert img.shape[0] <= 96 and img.shape[1] <= 128
        assert lab.shape[1] == 5 and (lab[:, 2] > lab[:, 0]).all() and (lab[:, 3] > lab[:, 1]).all()
        np.testing.assert_array_equal(ds.load_anno(i), lab)
        shapes.add(img.shape)
    assert len(shapes) > 4


def test_training_loader_is_the_mosaic_pipeline_across_close_mosaic(fixture):
    """config.get_data_loader (config.py:203-273) builds the device MosaicDetection pipeline
    with the config's augmentation parameters; across close_mosaic (trainer.py:217-230) the
    random draws follow the reference's order: the fixture's `boundary` samples are the
    reference's MosaicDetection seeded ONCE, 12 samples with mosaic on, then 12 with it off."""
    from yolox_amd.config import named_config
    g, images, labels = fixture
    cfg = named_config("yolox_s")
    cfg.input_size = tuple(int(v) for v in g["input_hw"])
    loader = cfg.get_data_loader(batch_size=4, is_distributed=False, dataset=ArrayDataset(images, labels),
                                 device="cpu")
    ds = loader.dataset
    assert isinstance(ds, M.GpuMosaicDetection) and ds.enable_mosaic
    assert (ds.degrees, ds.translate, ds.shear, tuple(ds.scale), ds.enable_mixup) == (
        cfg.degrees, cfg.translate, cfg.shear, tuple(cfg.mosaic_scale), cfg.enable_mixup)
    random.seed(4242)
    np.random.seed(4242)
    n = len(images)
    kinds = []
    for s in range(2 * SEEDS):
        if s == SEEDS:
            loader.close_mosaic()
        p, lab = ds.draw((3 * s + 1) % n)
        kinds.append(p.mosaic)
        np.testing.assert_array_equal(lab, g[f"boundary.{s}.labels"], err_msg=f"boundary sample {s}")
    assert kinds == [True] * SEEDS + [False] * SEEDS


def test_trainer_closes_mosaic_at_the_reference_epoch():
    """Trainer.before_epoch (trainer.py:217-230): mosaic off and the L1 loss on from epoch
    max_epoch - no_aug_epochs - 1 (0-based) onwards, or from the start with no_aug."""
    import types

    from yolox_amd.trainer import Trainer
    cfg = types.SimpleNamespace(max_epoch=5, no_aug_epochs=2, ema=False, input_size=(64, 64))
    for no_aug, first_closed in ((False, 2), (True, 0)):
        tr = Trainer.__new__(Trainer)
        tr.exp, tr.max_epoch, tr.no_aug, tr.is_distributed = cfg, cfg.max_epoch, no_aug, False
        closed = []
        tr.train_loader = types.SimpleNamespace(close_mosaic=lambda: closed.append(tr.epoch))
        tr.model = types.SimpleNamespace(head=types.SimpleNamespace(use_l1=False))
        for tr.epoch in range(cfg.max_epoch):
            tr.before_epoch()
        assert closed[0] == first_closed and tr.model.head.use_l1


def test_resident_images_ids_of_repeated_items():
    """Items that repeat a stored image (``source_index``) are uploaded once; their ids come from
    the dataset (``image_id(i)``: what its pull_item(i) returns), not from the item index."""

    class _Repeating:
        def __len__(self):
            return 6

        def source_index(self, i):
            return i % 2

        def image_id(self, i):
            return np.array([1000 + 7 * i])

        def load_anno(self, i):
            return np.zeros((1, 5)) + i

        def pull_item(self, i):
            return np.full((4, 6, 3), i, np.uint8), self.load_anno(i), (4, 6), self.image_id(i)

    ds = _Repeating()
    res = M.ResidentImages(ds, device="cpu")
    assert [int(np.asarray(v).reshape(-1)[0]) for v in res.ids] == [1000 + 7 * i for i in range(6)]
    assert int(res.pool.numel()) >= 2 * 4 * 6 * 3 and res.offsets[2] == res.offsets[0]
    syn = M.SyntheticDetectionDataset(5, (64, 64), distinct=2)
    r2 = M.ResidentImages(syn, device="cpu")
    assert [int(v[0]) for v in r2.ids] == [int(syn.pull_item(i)[3][0]) for i in range(5)]
