"""Shared helpers of the augmentation tests: the golden fixture's dataset (tests/golden/
mosaic_aug.npz, made by make_golden.py gen_mosaic from the reference's own MosaicDetection /
TrainTransform code) and the MosaicDetection configurations it was drawn with."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mosaic_aug.npz")

# make_golden.py MOSAIC_CASES (config.py defaults; nano preset; close_mosaic)
CASES = {
    "default": dict(mosaic=True, mosaic_scale=(0.1, 2), mixup_scale=(0.5, 1.5), enable_mixup=True, mosaic_prob=1.0,
                    mixup_prob=1.0),
    "nano": dict(mosaic=True, mosaic_scale=(0.5, 1.5), mixup_scale=(0.5, 1.5), enable_mixup=False, mosaic_prob=0.5,
                 mixup_prob=1.0),
    "no_aug": dict(mosaic=False, mosaic_scale=(0.1, 2), mixup_scale=(0.5, 1.5), enable_mixup=True, mosaic_prob=1.0,
                   mixup_prob=1.0),
}
SEEDS = 12


def load_fixture():
    g = np.load(GOLDEN)
    images, labels = [], []
    o = lo = 0
    for (h, w), c in zip(g["shapes"], g["label_counts"]):
        images.append(g["pixels"][o:o + h * w * 3].reshape(h, w, 3))
        o += h * w * 3
        labels.append(g["labels"][lo:lo + c])
        lo += c
    return g, images, labels


class ArrayDataset:
    """pull_item / load_anno over in-memory images (uint8 HxWx3 BGR) and labels [n, 5]."""

    def __init__(self, images, labels):
        self.images, self.labels = images, labels

    def __len__(self):
        return len(self.images)

    def load_anno(self, i):
        return self.labels[i]

    def pull_item(self, i):
        return self.images[i].copy(), self.labels[i].copy(), self.images[i].shape[:2], np.array([i])
