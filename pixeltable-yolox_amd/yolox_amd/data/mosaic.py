"""Training-time augmentation on device: MosaicDetection + TrainTransform for whole batches.

The reference builds every training sample in DataLoader worker processes with cv2 on the
CPU (datasets/mosaicdetection.py:76-232, data_augment.py:19-208): four pull_item images are
resized and pasted into a 2H x 2W mosaic canvas, warped by a random affine, mixed with a
jittered copy-paste image, HSV-jittered, mirrored and transposed to float32 CHW.  Here:

* the dataset's pull_item images stay RESIDENT in HBM (``ResidentImages``: one byte pool,
  uploaded once -- the analogue of the reference's ``cache=True``, sized for 288 GB);
* the host draws each sample's random parameters with Python ``random`` / ``np.random`` in
  exactly the reference's call order (so a seeded run draws the same augmentation as the
  reference) and computes the labels in numpy with the reference's arithmetic;
* ONE ``yxh_augment_batch`` call (csrc/augment.hip, two kernels) renders the whole batch's
  float32 [B, 3, H, W] tensor from the pool -- the mosaic canvas, the resized images and the
  mixup copy are never materialised.

``GpuMosaicDetection`` mirrors the reference class's constructor and ``__getitem__``;
``MosaicBatches`` is the loader the trainer pulls batches from.  There is no CPU image path:
rendering needs libyoloxhip.so on a ROCm device.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from .. import _native as N

__all__ = ["AugParams", "TrainTransform", "ResidentImages", "GpuMosaicDetection", "MosaicBatches",
           "SyntheticDetectionDataset", "xyxy2cxcywh", "adjust_box_anns", "get_mosaic_coordinate"]


# ----------------------------------------------------------------- box helpers (reference semantics)
def xyxy2cxcywh(b: np.ndarray) -> np.ndarray:
    """utils/boxes.py:129-134, in place."""
    b[:, 2] = b[:, 2] - b[:, 0]
    b[:, 3] = b[:, 3] - b[:, 1]
    b[:, 0] = b[:, 0] + b[:, 2] * 0.5
    b[:, 1] = b[:, 1] + b[:, 3] * 0.5
    return b


def adjust_box_anns(b: np.ndarray, ratio: float, padw: float, padh: float, w_max: float, h_max: float):
    """utils/boxes.py:117-120, in place."""
    b[:, 0::2] = np.clip(b[:, 0::2] * ratio + padw, 0, w_max)
    b[:, 1::2] = np.clip(b[:, 1::2] * ratio + padh, 0, h_max)
    return b


def get_mosaic_coordinate(i: int, xc: int, yc: int, w: int, h: int, input_h: int, input_w: int):
    """Canvas rectangle and source crop of mosaic tile ``i`` (mosaicdetection.py:14-32)."""
    if i == 0:
        l = (max(xc - w, 0), max(yc - h, 0), xc, yc)
        return l, (w - (l[2] - l[0]), h - (l[3] - l[1]), w, h)
    if i == 1:
        l = (xc, max(yc - h, 0), min(xc + w, input_w * 2), yc)
        return l, (0, h - (l[3] - l[1]), min(w, l[2] - l[0]), h)
    if i == 2:
        l = (max(xc - w, 0), yc, xc, min(input_h * 2, yc + h))
        return l, (w - (l[2] - l[0]), 0, w, min(l[3] - l[1], h))
    l = (xc, yc, min(xc + w, input_w * 2), min(input_h * 2, yc + h))
    return l, (0, 0, min(w, l[2] - l[0]), min(l[3] - l[1], h))


def _aug_param(rnd: random.Random, value, center: float = 0.0) -> float:
    """get_aug_params (data_augment.py:32-41)."""
    if isinstance(value, float):
        return rnd.uniform(center - value, center + value)
    if len(value) == 2:
        return rnd.uniform(value[0], value[1])
    raise ValueError(f"Affine params should be either a sequence containing two values or single float values. "
                     f"Got {value}")


def affine_matrix(rnd: random.Random, target_size, degrees, translate, scales, shear):
    """get_affine_matrix (data_augment.py:44-77); cv2.getRotationMatrix2D about (0, 0)."""
    twidth, theight = target_size
    angle = _aug_param(rnd, degrees)
    scale = _aug_param(rnd, scales, center=1.0)
    if scale <= 0.0:
        raise ValueError("Argument scale should be positive")
    a = angle * math.pi / 180.0
    alpha, beta = math.cos(a) * scale, math.sin(a) * scale
    R = np.array([[alpha, beta, 0.0], [-beta, alpha, 0.0]], np.float64)
    M = np.ones([2, 3])
    shear_x = math.tan(_aug_param(rnd, shear) * math.pi / 180)
    shear_y = math.tan(_aug_param(rnd, shear) * math.pi / 180)
    M[0] = R[0] + shear_y * R[1]
    M[1] = R[1] + shear_x * R[0]
    M[0, 2] = _aug_param(rnd, translate) * twidth
    M[1, 2] = _aug_param(rnd, translate) * theight
    return M, scale


def affine_boxes(targets: np.ndarray, target_size, M: np.ndarray) -> np.ndarray:
    """apply_affine_to_bboxes (data_augment.py:80-109): corners through M, enclosing box, clip."""
    n = len(targets)
    twidth, theight = target_size
    pts = np.ones((4 * n, 3))
    pts[:, :2] = targets[:, [0, 1, 2, 3, 0, 3, 2, 1]].reshape(4 * n, 2)
    pts = (pts @ M.T).reshape(n, 8)
    xs, ys = pts[:, 0::2], pts[:, 1::2]
    nb = np.concatenate((xs.min(1), ys.min(1), xs.max(1), ys.max(1))).reshape(4, n).T
    nb[:, 0::2] = nb[:, 0::2].clip(0, twidth)
    nb[:, 1::2] = nb[:, 1::2].clip(0, theight)
    targets[:, :4] = nb
    return targets


def invert_affine(M: np.ndarray) -> list:
    """cv2.invertAffineTransform: the output -> canvas map warpAffine samples with."""
    m = M.reshape(-1)
    D = m[0] * m[4] - m[1] * m[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22, A12, A21 = m[4] * D, m[0] * D, -m[1] * D, -m[3] * D
    return [A11, A12, -A11 * m[2] - A12 * m[5], A21, A22, -A21 * m[2] - A22 * m[5]]


# ----------------------------------------------------------------- parameters
@dataclass
class TrainTransform:
    """data_augment.py:159-208's parameters (the image half runs in ``yxh_augment_batch``,
    the label half in ``GpuMosaicDetection._transform``)."""
    max_labels: int = 50
    flip_prob: float = 0.5
    hsv_prob: float = 1.0


@dataclass
class AugParams:
    """One sample's drawn augmentation (what the reference's random calls decided)."""
    mosaic: bool
    indices: list
    xc: int = 0
    yc: int = 0
    M: Optional[np.ndarray] = None
    mix: bool = False
    cp_index: int = -1
    jit: float = 1.0
    cp_flip: bool = False
    x_off: int = 0
    y_off: int = 0
    do_hsv: bool = False
    hsv: tuple = (0, 0, 0)
    flip: bool = False
    extra: dict = field(default_factory=dict)


# ----------------------------------------------------------------- resident images
class ResidentImages:
    """Every pull_item image of ``dataset`` (uint8 HWC BGR) in one device byte pool, plus the
    host copy of its labels.  Images are uploaded once, through pinned staging, in chunks."""

    def __init__(self, dataset, device="cuda", chunk_bytes: int = 256 << 20):
        self.device = torch.device(device)
        n = len(dataset)
        self.shapes = np.zeros((n, 2), np.int64)
        self.offsets = np.zeros(n, np.int64)
        self.labels: list = []
        self.infos: list = []
        self.ids: list = []
        images = []
        off = 0
        # a dataset whose items repeat stored images (source_index) uploads each image once; the
        # repeated item's id is the dataset's own (``image_id(i)``, what its pull_item(i) would
        # return), or the item index when the dataset has no such method
        src_of = getattr(dataset, "source_index", None)
        id_of = getattr(dataset, "image_id", None)
        first: dict = {}
        for i in range(n):
            src = src_of(i) if src_of is not None else i
            if src in first:
                j = first[src]
                self.shapes[i], self.offsets[i] = self.shapes[j], self.offsets[j]
                lab = dataset.load_anno(i) if hasattr(dataset, "load_anno") else self.labels[j]
                self.labels.append(np.array(lab, copy=True))
                self.infos.append(self.infos[j])
                self.ids.append(np.asarray(id_of(i)) if id_of is not None else np.array([i]))
                continue
            first[src] = i
            img, lab, info, img_id = dataset.pull_item(i)
            img = np.ascontiguousarray(img, dtype=np.uint8)
            if img.ndim != 3 or img.shape[2] != 3:
                raise ValueError(f"pull_item({i}) must give an HxWx3 uint8 image, got {img.shape}")
            self.shapes[i] = img.shape[:2]
            self.offsets[i] = off
            off += (img.nbytes + 15) & ~15
            images.append((i, img))
            self.labels.append(np.array(lab, copy=True))
            self.infos.append(info)
            self.ids.append(img_id)
        self.pool = torch.empty(max(off, 16), dtype=torch.uint8, device=self.device)
        staging = torch.empty(min(max(off, 16), chunk_bytes), dtype=torch.uint8)
        if self.device.type == "cuda":
            staging = staging.pin_memory()
        i, m = 0, len(images)
        while i < m:  # pack a chunk of whole images, copy it in one H2D transfer
            j, start = i, int(self.offsets[images[i][0]])
            while j < m and int(self.offsets[images[j][0]]) + images[j][1].nbytes - start <= staging.numel():
                j += 1
            if j == i:
                raise ValueError(f"image {images[i][0]} ({images[i][1].nbytes} bytes) exceeds the staging chunk")
            view = staging.numpy()
            for k in range(i, j):
                o = int(self.offsets[images[k][0]]) - start
                view[o:o + images[k][1].nbytes] = images[k][1].reshape(-1)
            end = int(self.offsets[images[j - 1][0]]) + images[j - 1][1].nbytes
            self.pool[start:end].copy_(staging[:end - start], non_blocking=False)
            i = j

    def __len__(self) -> int:
        return len(self.shapes)

    @property
    def nbytes(self) -> int:
        return self.pool.numel()


# ----------------------------------------------------------------- the dataset wrapper
class GpuMosaicDetection:
    """MosaicDetection (mosaicdetection.py:35-232) + TrainTransform on device.

    ``dataset`` is a detection dataset with the reference's interface: ``__len__``,
    ``pull_item(i) -> (uint8 HxWx3 BGR image, labels [n, 5] (x1, y1, x2, y2, cls), info, id)``
    and ``load_anno(i) -> labels``.  Random draws use Python ``random`` and ``np.random`` (the
    module-level generators, as the reference does) unless ``rng`` / ``np_rng`` are given."""

    def __init__(self, dataset, img_size, mosaic: bool = True, preproc: Optional[TrainTransform] = None,
                 degrees: float = 10.0, translate: float = 0.1, mosaic_scale=(0.5, 1.5), mixup_scale=(0.5, 1.5),
                 shear: float = 2.0, enable_mixup: bool = True, mosaic_prob: float = 1.0, mixup_prob: float = 1.0,
                 device="cuda", rng: Optional[random.Random] = None, np_rng=None, resident: Optional[ResidentImages] = None):
        self._dataset = dataset
        self._input_dim = tuple(img_size[:2])
        self.enable_mosaic = mosaic
        self.preproc = preproc if preproc is not None else TrainTransform(max_labels=120)
        self.degrees, self.translate, self.scale, self.shear = degrees, translate, mosaic_scale, shear
        self.mixup_scale = mixup_scale
        self.enable_mixup = enable_mixup
        self.mosaic_prob, self.mixup_prob = mosaic_prob, mixup_prob
        self.random = rng if rng is not None else random
        self.np_random = np_rng if np_rng is not None else np.random
        self.images = resident if resident is not None else ResidentImages(dataset, device)
        self.device = self.images.device

    def __len__(self) -> int:
        return len(self._dataset)

    @property
    def input_dim(self):
        return self._input_dim

    @input_dim.setter
    def input_dim(self, dim) -> None:
        self._input_dim = tuple(dim[:2])

    def close_mosaic(self) -> None:
        """The last no_aug_epochs (trainer.py before_epoch): plain TrainTransform."""
        self.enable_mosaic = False

    # ------------------------------------------------------------ host: draws + labels
    def _labels(self, i: int) -> np.ndarray:
        return self.images.labels[i].copy()

    def _shape(self, i: int):
        h, w = self.images.shapes[i]
        return int(h), int(w)

    def draw(self, idx: int):
        """The reference's random draws and label arithmetic for sample ``idx`` -> (AugParams,
        padded labels float32 [max_labels, 5] (cls, cx, cy, w, h))."""
        rnd = self.random
        input_h, input_w = self._input_dim
        if self.enable_mosaic and rnd.random() < self.mosaic_prob:
            yc = int(rnd.uniform(0.5 * input_h, 1.5 * input_h))
            xc = int(rnd.uniform(0.5 * input_w, 1.5 * input_w))
            indices = [idx] + [rnd.randint(0, len(self._dataset) - 1) for _ in range(3)]
            p = AugParams(mosaic=True, indices=indices, xc=xc, yc=yc)
            mosaic_labels = []
            for i_mosaic, index in enumerate(indices):
                h0, w0 = self._shape(index)
                scale = min(1.0 * input_h / h0, 1.0 * input_w / w0)
                h, w = int(h0 * scale), int(w0 * scale)
                (l_x1, l_y1, _, _), (s_x1, s_y1, _, _) = get_mosaic_coordinate(i_mosaic, xc, yc, w, h, input_h,
                                                                               input_w)
                padw, padh = l_x1 - s_x1, l_y1 - s_y1
                _labels = self._labels(index)
                labels = _labels.copy()
                if _labels.size > 0:
                    labels[:, 0] = scale * _labels[:, 0] + padw
                    labels[:, 1] = scale * _labels[:, 1] + padh
                    labels[:, 2] = scale * _labels[:, 2] + padw
                    labels[:, 3] = scale * _labels[:, 3] + padh
                mosaic_labels.append(labels)
            mosaic_labels = np.concatenate(mosaic_labels, 0)
            np.clip(mosaic_labels[:, 0], 0, 2 * input_w, out=mosaic_labels[:, 0])
            np.clip(mosaic_labels[:, 1], 0, 2 * input_h, out=mosaic_labels[:, 1])
            np.clip(mosaic_labels[:, 2], 0, 2 * input_w, out=mosaic_labels[:, 2])
            np.clip(mosaic_labels[:, 3], 0, 2 * input_h, out=mosaic_labels[:, 3])
            p.M, _ = affine_matrix(rnd, (input_w, input_h), self.degrees, self.translate, self.scale, self.shear)
            if len(mosaic_labels) > 0:
                mosaic_labels = affine_boxes(mosaic_labels, (input_w, input_h), p.M)
            if self.enable_mixup and not len(mosaic_labels) == 0 and rnd.random() < self.mixup_prob:
                mosaic_labels = self._mixup(p, mosaic_labels)
            labels = self._transform(p, mosaic_labels, (input_h, input_w), 1.0)
            return p, labels
        p = AugParams(mosaic=False, indices=[idx])
        h0, w0 = self._shape(idx)
        r = min(input_h / h0, input_w / w0)
        return p, self._transform(p, self._labels(idx), (h0, w0), r)

    def _mixup(self, p: AugParams, origin_labels: np.ndarray) -> np.ndarray:
        """mosaicdetection.py:160-232, label half; the image half is p's mix fields."""
        rnd = self.random
        input_h, input_w = self._input_dim
        jit = rnd.uniform(*self.mixup_scale)
        flip = rnd.uniform(0, 1) > 0.5
        cp_labels = []
        while len(cp_labels) == 0:
            cp_index = rnd.randint(0, len(self) - 1)
            cp_labels = self._dataset.load_anno(cp_index)
        cp_labels = self._labels(cp_index)
        h0, w0 = self._shape(cp_index)
        ratio = min(input_h / h0, input_w / w0)
        origin_h, origin_w = int(input_h * jit), int(input_w * jit)
        ratio *= jit
        ph, pw = max(origin_h, input_h), max(origin_w, input_w)
        x_off = y_off = 0
        if ph > input_h:
            y_off = rnd.randint(0, ph - input_h - 1)
        if pw > input_w:
            x_off = rnd.randint(0, pw - input_w - 1)
        boxes = adjust_box_anns(cp_labels[:, :4].copy(), ratio, 0, 0, origin_w, origin_h)
        if flip:
            boxes[:, 0::2] = origin_w - boxes[:, 0::2][:, ::-1]
        t = boxes.copy()
        t[:, 0::2] = np.clip(t[:, 0::2] - x_off, 0, input_w)
        t[:, 1::2] = np.clip(t[:, 1::2] - y_off, 0, input_h)
        labels = np.hstack((t, cp_labels[:, 4:5].copy()))
        p.mix, p.cp_index, p.jit, p.cp_flip, p.x_off, p.y_off = True, cp_index, jit, flip, x_off, y_off
        return np.vstack((origin_labels, labels))

    def _transform(self, p: AugParams, targets: np.ndarray, image_hw, r: float) -> np.ndarray:
        """TrainTransform.__call__ (data_augment.py:165-208), label half: draws hsv / mirror,
        returns the padded (cls, cx, cy, w, h) labels; sets p.do_hsv / p.hsv / p.flip to what
        the returned image shows (the no-surviving-box fallback shows the untouched image)."""
        tt = self.preproc
        boxes = targets[:, :4].copy()
        labels = targets[:, 4].copy()
        if len(boxes) == 0:
            return np.zeros((tt.max_labels, 5), dtype=np.float32)
        targets_o = targets.copy()
        boxes_o = xyxy2cxcywh(targets_o[:, :4])
        labels_o = targets_o[:, 4]
        if self.random.random() < tt.hsv_prob:
            gains = self.np_random.uniform(-1, 1, 3) * [5, 30, 30]
            gains *= self.np_random.randint(0, 2, 3)
            p.do_hsv, p.hsv = True, tuple(int(g) for g in gains.astype(np.int16))
        width = image_hw[1]
        if self.random.random() < tt.flip_prob:
            p.flip = True
            boxes[:, 0::2] = width - boxes[:, 2::-2]
        boxes = xyxy2cxcywh(boxes)
        boxes *= r
        mask_b = np.minimum(boxes[:, 2], boxes[:, 3]) > 1
        boxes_t = boxes[mask_b]
        labels_t = labels[mask_b]
        if len(boxes_t) == 0:
            p.do_hsv, p.flip = False, False
            boxes_o *= r
            boxes_t, labels_t = boxes_o, labels_o
        targets_t = np.hstack((np.expand_dims(labels_t, 1), boxes_t))
        padded = np.zeros((tt.max_labels, 5))
        padded[range(len(targets_t))[:tt.max_labels]] = targets_t[:tt.max_labels]
        return np.ascontiguousarray(padded, dtype=np.float32)

    # ------------------------------------------------------------ device: pack + render
    def pack(self, p: AugParams) -> N.AugImage:
        """AugParams -> yxh_aug_image: the geometry the kernels need (sizes, placements, cv2
        scale factors, the inverted affine)."""
        input_h, input_w = self._input_dim
        d = N.AugImage()
        d.mosaic, d.mix, d.flip, d.do_hsv, d.cp_flip = int(p.mosaic), int(p.mix), int(p.flip), int(p.do_hsv), \
            int(p.cp_flip)
        for k in range(3):
            d.hsv[k] = int(p.hsv[k])
        for q, index in enumerate(p.indices):
            h0, w0 = self._shape(index)
            if p.mosaic:
                scale = min(1.0 * input_h / h0, 1.0 * input_w / w0)
            else:
                scale = min(input_h / h0, input_w / w0)
            rh, rw = int(h0 * scale), int(w0 * scale)
            if rh <= 0 or rw <= 0:
                raise ValueError(f"image {index} ({h0}x{w0}) resizes to an empty image at {input_h}x{input_w}")
            d.src_off[q] = int(self.images.offsets[index])
            d.src_h[q], d.src_w[q], d.rh[q], d.rw[q] = h0, w0, rh, rw
            d.rsx[q], d.rsy[q] = 1.0 / (rw / w0), 1.0 / (rh / h0)
            if p.mosaic:
                (l_x1, l_y1, l_x2, l_y2), (s_x1, s_y1, _, _) = get_mosaic_coordinate(q, p.xc, p.yc, rw, rh, input_h,
                                                                                     input_w)
                d.lx1[q], d.ly1[q], d.lx2[q], d.ly2[q], d.sx1[q], d.sy1[q] = l_x1, l_y1, l_x2, l_y2, s_x1, s_y1
        if p.mosaic:
            for k, v in enumerate(invert_affine(p.M)):
                d.minv[k] = v
        if p.mix:
            h0, w0 = self._shape(p.cp_index)
            r = min(input_h / h0, input_w / w0)
            d.cp_off = int(self.images.offsets[p.cp_index])
            d.cp_h, d.cp_w, d.cp_rh, d.cp_rw = h0, w0, int(h0 * r), int(w0 * r)
            if d.cp_rh <= 0 or d.cp_rw <= 0:
                raise ValueError(f"mixup image {p.cp_index} resizes to an empty image")
            d.cp_sx, d.cp_sy = 1.0 / (d.cp_rw / w0), 1.0 / (d.cp_rh / h0)
            d.jit_h, d.jit_w = int(input_h * p.jit), int(input_w * p.jit)
            if d.jit_h <= 0 or d.jit_w <= 0:
                raise ValueError(f"mixup jitter {p.jit} gives an empty image")
            d.jit_sx, d.jit_sy = 1.0 / (d.jit_w / input_w), 1.0 / (d.jit_h / input_h)
            d.x_off, d.y_off = p.x_off, p.y_off
        return d

    def render(self, params: Sequence[AugParams], out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """float32 [B, 3, H, W] images of the drawn samples (one yxh_augment_batch call)."""
        input_h, input_w = self._input_dim
        N.require_device(self.images.pool, "resident image pool")
        B = len(params)
        descs = (N.AugImage * B)(*[self.pack(p) for p in params])
        host = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8)
        dev_desc = host.to(self.device, non_blocking=False)
        if out is None:
            out = torch.empty((B, 3, input_h, input_w), dtype=torch.float32, device=self.device)
        if tuple(out.shape) != (B, 3, input_h, input_w) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError(f"out must be contiguous float32 {(B, 3, input_h, input_w)}")
        ws = torch.empty(B * input_h * input_w * 3, dtype=torch.uint8, device=self.device)
        N.check(N.lib().yxh_augment_batch(self.images.pool.data_ptr(), dev_desc.data_ptr(), B, input_h, input_w,
                                          ws.data_ptr(), out.data_ptr(), N.stream_ptr(self.device)),
                "yxh_augment_batch")
        return out

    def get_batch(self, indices: Sequence[int]):
        """(images float32 [B, 3, H, W], targets float32 [B, max_labels, 5]) on device."""
        drawn = [self.draw(int(i)) for i in indices]
        imgs = self.render([p for p, _ in drawn])
        targets = torch.from_numpy(np.stack([t for _, t in drawn])).to(self.device)
        return imgs, targets

    def __getitem__(self, idx):
        """The reference's item: (image float32 CHW (device), padded labels, img_info, img_id);
        ``idx`` may be the (enable_mosaic, index) pair YoloBatchSampler yields."""
        if not isinstance(idx, (int, np.integer)):
            self.enable_mosaic, idx = idx[0], idx[1]
        p, labels = self.draw(int(idx))
        img = self.render([p])[0]
        if p.mosaic:  # (mix_img.shape[1], mix_img.shape[0]) of the CHW array and the last tile's id, as the reference
            return img, labels, (img.shape[1], img.shape[0]), self.images.ids[p.indices[-1]]
        return img, labels, self.images.infos[int(idx)], self.images.ids[int(idx)]


class MosaicBatches:
    """The training loader over GpuMosaicDetection: per-rank batches of sampler indices
    (YoloBatchSampler over InfiniteSampler), rendered on device."""

    def __init__(self, dataset: GpuMosaicDetection, sampler, batch_size: int):
        self.dataset, self.sampler, self.batch_size = dataset, sampler, batch_size
        self._it = iter(sampler)

    def __len__(self) -> int:
        return (len(self.sampler) + self.batch_size - 1) // self.batch_size

    def next_indices(self) -> list:
        return [next(self._it) for _ in range(self.batch_size)]

    def next(self):
        return self.dataset.get_batch(self.next_indices())

    def close_mosaic(self) -> None:
        self.dataset.close_mosaic()


# ----------------------------------------------------------------- synthetic detection data
class SyntheticDetectionDataset:
    """COCO-like detection items without files (no datasets offline): item i is a seeded
    uint8 BGR image of a seeded size, pre-resized to fit ``img_size`` as COCODataset's
    pull_item gives it (coco.py:131-160 load_resized_img; a plain nearest resample stands in
    for cv2 here, as only the result's shape and content matter to the pipeline), with 0-8
    boxes (x1, y1, x2, y2, cls) scaled alike; smooth gradients + blocks so HSV / resampling
    see structured content."""

    def __init__(self, size: int, img_size=(640, 640), seed: int = 0, num_classes: int = 80,
                 min_side: int = 32, max_side: int = 960, empty_every: int = 7, distinct: Optional[int] = None):
        """``distinct``: item i is item i % distinct (a dataset of ``size`` samples over that
        many different images, so the resident pool stays small for COCO-sized epochs)."""
        self.size, self.img_size, self.seed = size, tuple(img_size), seed
        self.num_classes, self.min_side, self.max_side, self.empty_every = num_classes, min_side, max_side, empty_every
        self.distinct = min(distinct, size) if distinct else None
        self._cache: dict = {}

    def source_index(self, i: int) -> int:
        """The stored image item i shows (ResidentImages uploads each once)."""
        return i % self.distinct if self.distinct else i

    def __len__(self) -> int:
        return self.size

    def _item(self, i: int):
        i = self.source_index(i)
        if i in self._cache:
            return self._cache[i]
        rng = np.random.default_rng((self.seed, i))
        h, w = (int(v) for v in rng.integers(self.min_side, self.max_side + 1, 2))
        r = min(self.img_size[0] / h, self.img_size[1] / w)
        rh, rw = max(int(h * r), 1), max(int(w * r), 1)
        yy, xx = np.mgrid[0:rh, 0:rw]
        base = np.stack([(xx * 255 // max(rw - 1, 1)), (yy * 255 // max(rh - 1, 1)),
                         ((xx + yy) * 127 // max(rw + rh - 2, 1))], -1)
        img = (base + rng.integers(-20, 21, (rh, rw, 3))).clip(0, 255).astype(np.uint8)
        n = 0 if (self.empty_every and i % self.empty_every == self.empty_every - 1) else int(rng.integers(1, 9))
        labels = np.zeros((n, 5))
        for k in range(n):
            bw, bh = rng.uniform(2, rw), rng.uniform(2, rh)
            x1, y1 = rng.uniform(0, rw - bw + 1e-9), rng.uniform(0, rh - bh + 1e-9)
            labels[k] = (x1, y1, x1 + bw, y1 + bh, int(rng.integers(0, self.num_classes)))
            img[int(y1):int(y1 + bh), int(x1):int(x1 + bw)] = rng.integers(0, 256, 3)
        self._cache[i] = (img, labels)
        return img, labels

    def load_anno(self, i: int) -> np.ndarray:
        return self._item(i)[1]

    def image_id(self, i: int) -> np.ndarray:
        """The id pull_item(i) returns (the item index, as the reference's COCODataset ids are
        per item) -- what ResidentImages records for an item it does not pull."""
        return np.array([i])

    def pull_item(self, i: int):
        img, labels = self._item(i)
        return img, labels.copy(), img.shape[:2], self.image_id(i)
