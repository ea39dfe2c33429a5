"""ORACLE -- test infrastructure only (DESIGN.md §Oracle, §8(f)-4 training augmentation).

numpy restatement of the reference's training-time augmentation
(yolox/data/datasets/mosaicdetection.py:76-232, yolox/data/data_augment.py:19-208) and of the
cv2 calls it makes.  cv2 (opencv-python 4.10 per the reference's poetry.lock) is absent from
this image, so ``CV2`` below restates the published fixed-point algorithms of the four calls
the path uses; the checker for the HIP kernels (csrc/augment.hip) is ``render`` -- the
reference's composition of those calls for one sample's drawn parameters.

Pinning: tests/golden/mosaic_aug.npz was produced by running the reference's OWN
MosaicDetection.__getitem__ / mixup / TrainTransform code (make_golden.py gen_mosaic) with
``CV2`` substituted for cv2, so the random-draw order, the label arithmetic and the order of
the image operations are pinned to the reference; the pixel values of cv2's resize /
warpAffine / HSV conversions are pinned only to this restatement (parity unpinned vs cv2).
The product (yolox_amd.data.mosaic) never imports this module.
"""
from __future__ import annotations

import math
import types

import numpy as np

# --------------------------------------------------------------------------- cv2 restated
INTER_LINEAR = 1
COLOR_BGR2HSV = 40
COLOR_HSV2BGR = 54
_AB_BITS, _INTER_BITS = 10, 5
_TAB = 1 << _INTER_BITS


def _coeffs(dst: int, scale: float, ssize: int):
    """cv2 resize INTER_LINEAR source index + 11-bit weights per destination index."""
    f = ((np.arange(dst, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = 0.0, 0
    hi = s >= ssize - 1
    f[hi], s[hi] = 0.0, ssize - 1
    a0 = np.rint((np.float32(1.0) - f) * np.float32(2048.0)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048.0)).astype(np.int64)
    return s, np.minimum(s + 1, ssize - 1), a0, a1


def resize(img: np.ndarray, dsize, interpolation=INTER_LINEAR) -> np.ndarray:
    """cv2.resize(img, (w, h)) for uint8 HxWx3, INTER_LINEAR: same size copies; exact 2x
    downscale takes INTER_AREA's (a+b+c+d+2)>>2; otherwise 11-bit fixed point with
    VResizeLinearVec_32s8u's vertical rounding."""
    rw, rh = int(dsize[0]), int(dsize[1])
    h, w = img.shape[:2]
    if rw == w and rh == h:
        return img.copy()
    sx, sy = 1.0 / (rw / w), 1.0 / (rh / h)
    a = img.astype(np.int64)
    if abs(sx - 2.0) < 2.220446049250313e-16 and abs(sy - 2.0) < 2.220446049250313e-16:
        return ((a[0:2 * rh:2, 0:2 * rw:2] + a[0:2 * rh:2, 1:2 * rw:2] + a[1:2 * rh:2, 0:2 * rw:2]
                 + a[1:2 * rh:2, 1:2 * rw:2] + 2) >> 2).astype(np.uint8)
    x0, x1, ax0, ax1 = _coeffs(rw, sx, w)
    y0, y1, by0, by1 = _coeffs(rh, sy, h)
    h0 = a[y0][:, x0] * ax0[None, :, None] + a[y0][:, x1] * ax1[None, :, None]
    h1 = a[y1][:, x0] * ax0[None, :, None] + a[y1][:, x1] * ax1[None, :, None]
    t = (((h0 >> 4) * by0[:, None, None]) >> 16) + (((h1 >> 4) * by1[:, None, None]) >> 16) + 2
    return np.clip(t >> 2, 0, 255).astype(np.uint8)


def getRotationMatrix2D(center, angle, scale):  # noqa: N802 (cv2 name)
    """cv2.getRotationMatrix2D: [[a, b, (1-a)cx - b cy], [-b, a, b cx + (1-a) cy]]."""
    ang = angle * math.pi / 180.0
    alpha, beta = math.cos(ang) * scale, math.sin(ang) * scale
    cx, cy = center
    return np.array([[alpha, beta, (1 - alpha) * cx - beta * cy], [-beta, alpha, beta * cx + (1 - alpha) * cy]],
                    np.float64)


def invert_affine(M: np.ndarray) -> np.ndarray:
    """cv2.invertAffineTransform (what warpAffine does without WARP_INVERSE_MAP)."""
    m = M.reshape(-1)
    D = m[0] * m[4] - m[1] * m[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22, A12, A21 = m[4] * D, m[0] * D, -m[1] * D, -m[3] * D
    b1 = -A11 * m[2] - A12 * m[5]
    b2 = -A21 * m[2] - A22 * m[5]
    return np.array([A11, A12, b1, A21, A22, b2], np.float64)


def _sat_int(v: np.ndarray) -> np.ndarray:
    return np.clip(np.rint(v), -2147483648.0, 2147483647.0).astype(np.int64)


def warpAffine(img: np.ndarray, M, dsize, borderValue=(114, 114, 114)) -> np.ndarray:  # noqa: N802
    """cv2.warpAffine INTER_LINEAR, BORDER_CONSTANT, uint8 3-channel: inverse map in AB_BITS 10
    fixed point (round_delta 16), INTER_BITS 5 sub-pixel, the exact 15-bit bilinear table,
    (sum + 2^14) >> 15; taps outside the source read the border value."""
    W, H = int(dsize[0]), int(dsize[1])
    sh, sw = img.shape[:2]
    m = invert_affine(np.asarray(M, np.float64))
    scale = float(1 << _AB_BITS)
    rd = (1 << _AB_BITS) // _TAB // 2
    ys = np.arange(H, dtype=np.float64)
    xs = np.arange(W, dtype=np.float64)
    X0 = _sat_int((m[1] * ys + m[2]) * scale) + rd
    Y0 = _sat_int((m[4] * ys + m[5]) * scale) + rd
    adelta = _sat_int(m[0] * xs * scale)
    bdelta = _sat_int(m[3] * xs * scale)
    X = (X0[:, None] + adelta[None, :]) >> (_AB_BITS - _INTER_BITS)
    Y = (Y0[:, None] + bdelta[None, :]) >> (_AB_BITS - _INTER_BITS)
    sx, sy = X >> _INTER_BITS, Y >> _INTER_BITS
    fx, fy = X & (_TAB - 1), Y & (_TAB - 1)
    bv = np.array(borderValue[:3], np.int64)
    src = img.astype(np.int64)

    def tap(ty, tx):
        ok = (tx >= 0) & (tx < sw) & (ty >= 0) & (ty < sh)
        v = src[np.clip(ty, 0, sh - 1), np.clip(tx, 0, sw - 1)]
        return np.where(ok[..., None], v, bv)

    w00 = ((_TAB - fx) * (_TAB - fy) * 32)[..., None]
    w01 = (fx * (_TAB - fy) * 32)[..., None]
    w10 = ((_TAB - fx) * fy * 32)[..., None]
    w11 = (fx * fy * 32)[..., None]
    t = (tap(sy, sx) * w00 + tap(sy, sx + 1) * w01 + tap(sy + 1, sx) * w10 + tap(sy + 1, sx + 1) * w11
         + (1 << 14)) >> 15
    out = np.clip(t, 0, 255)
    far = (sx >= sw) | (sx + 1 < 0) | (sy >= sh) | (sy + 1 < 0)
    out = np.where(far[..., None], bv, out)
    return out.astype(np.uint8)


_SDIV = np.array([0] + [int(np.rint((255 << 12) / i)) for i in range(1, 256)], np.int64)
_HDIV180 = np.array([0] + [int(np.rint((180 << 12) / (6.0 * i))) for i in range(1, 256)], np.int64)
_SECTOR = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]], np.int64)


def bgr2hsv(img: np.ndarray) -> np.ndarray:
    """cv2 RGB2HSV_b (BGR order, hrange 180, hsv_shift 12 division tables)."""
    a = img.astype(np.int64)
    b, g, r = a[..., 0], a[..., 1], a[..., 2]
    v = np.maximum(b, np.maximum(g, r))
    vmin = np.minimum(b, np.minimum(g, r))
    diff = v - vmin
    vr = np.where(v == r, -1, 0)
    vg = np.where(v == g, -1, 0)
    s = (diff * _SDIV[v] + (1 << 11)) >> 12
    h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))))
    h = (h * _HDIV180[diff] + (1 << 11)) >> 12
    h = np.where(h < 0, h + 180, h)
    return np.stack([h, s, v], -1).astype(np.uint8)


def hsv2bgr(hsv: np.ndarray) -> np.ndarray:
    """cv2 HSV2RGB_b (hrange 180): float32 sectors, saturate_cast rounding half to even."""
    f32 = np.float32
    h = hsv[..., 0].astype(f32)
    s = hsv[..., 1].astype(f32) * f32(1.0 / 255.0)
    v = hsv[..., 2].astype(f32) * f32(1.0 / 255.0)
    h = (h * f32(6.0 / 180.0)).astype(f32)
    h = np.fmod(h, f32(6.0)).astype(f32)
    sector = np.floor(h).astype(np.int64)
    h = (h - sector.astype(f32)).astype(f32)
    bad = (sector < 0) | (sector >= 6)
    sector = np.where(bad, 0, sector)
    h = np.where(bad, f32(0.0), h).astype(f32)
    one = f32(1.0)
    tab = np.stack([v, (v * (one - s)).astype(f32), (v * (one - (s * h).astype(f32))).astype(f32),
                    (v * (one - (s * (one - h).astype(f32)).astype(f32))).astype(f32)], -1)
    out = np.take_along_axis(tab, _SECTOR[sector], -1)
    gray = (s == 0)[..., None]
    out = np.where(gray, v[..., None], out).astype(f32)
    return np.clip(np.rint((out * f32(255.0)).astype(f32)), 0, 255).astype(np.uint8)


def cvtColor(img: np.ndarray, code: int, dst=None):  # noqa: N802
    out = bgr2hsv(img) if code == COLOR_BGR2HSV else hsv2bgr(img)
    if dst is not None:
        dst[...] = out
        return dst
    return out


CV2 = types.SimpleNamespace(INTER_LINEAR=INTER_LINEAR, COLOR_BGR2HSV=COLOR_BGR2HSV, COLOR_HSV2BGR=COLOR_HSV2BGR,
                            resize=resize, warpAffine=warpAffine, cvtColor=cvtColor,
                            getRotationMatrix2D=getRotationMatrix2D)


# --------------------------------------------------------------------------- composition
def apply_hsv(img: np.ndarray, gains) -> np.ndarray:
    """augment_hsv (data_augment.py:19-29) with already drawn int16 gains."""
    hsv = bgr2hsv(img).astype(np.int16)
    hsv[..., 0] = (hsv[..., 0] + gains[0]) % 180
    hsv[..., 1] = np.clip(hsv[..., 1] + gains[1], 0, 255)
    hsv[..., 2] = np.clip(hsv[..., 2] + gains[2], 0, 255)
    return hsv2bgr(hsv.astype(np.uint8))


def mosaic_coordinate(i: int, xc: int, yc: int, w: int, h: int, input_h: int, input_w: int):
    """get_mosaic_coordinate (mosaicdetection.py:14-32)."""
    if i == 0:
        x1, y1, x2, y2 = max(xc - w, 0), max(yc - h, 0), xc, yc
        small = w - (x2 - x1), h - (y2 - y1), w, h
    elif i == 1:
        x1, y1, x2, y2 = xc, max(yc - h, 0), min(xc + w, input_w * 2), yc
        small = 0, h - (y2 - y1), min(w, x2 - x1), h
    elif i == 2:
        x1, y1, x2, y2 = max(xc - w, 0), yc, xc, min(input_h * 2, yc + h)
        small = w - (x2 - x1), 0, w, min(y2 - y1, h)
    else:
        x1, y1, x2, y2 = xc, yc, min(xc + w, input_w * 2), min(input_h * 2, yc + h)
        small = 0, 0, min(w, x2 - x1), min(y2 - y1, h)
    return (x1, y1, x2, y2), small


def letterbox_u8(img: np.ndarray, input_h: int, input_w: int) -> np.ndarray:
    """preproc (data_augment.py:140-156) before the CHW float transpose."""
    out = np.full((input_h, input_w, 3), 114, np.uint8)
    r = min(input_h / img.shape[0], input_w / img.shape[1])
    rh, rw = int(img.shape[0] * r), int(img.shape[1] * r)
    out[:rh, :rw] = resize(img, (rw, rh))
    return out


def render(p, images, input_h: int, input_w: int) -> np.ndarray:
    """The image one training sample ends as (float32 CHW), from its drawn parameters ``p``
    (yolox_amd.data.mosaic.AugParams fields) and the dataset's pull_item images: the
    mosaic canvas, random_affine's warp, mixup, augment_hsv, _mirror and preproc in the
    reference's order (mosaicdetection.py:78-152, 160-232; data_augment.py:159-208)."""
    if p.mosaic:
        canvas = None
        for i, index in enumerate(p.indices):
            img = images[index]
            h0, w0 = img.shape[:2]
            scale = min(1.0 * input_h / h0, 1.0 * input_w / w0)
            img = resize(img, (int(w0 * scale), int(h0 * scale)))
            h, w = img.shape[:2]
            if canvas is None:
                canvas = np.full((input_h * 2, input_w * 2, 3), 114, np.uint8)
            (lx1, ly1, lx2, ly2), (sx1, sy1, sx2, sy2) = mosaic_coordinate(i, p.xc, p.yc, w, h, input_h, input_w)
            canvas[ly1:ly2, lx1:lx2] = img[sy1:sy2, sx1:sx2]
        out = warpAffine(canvas, p.M, (input_w, input_h), (114, 114, 114))
        if p.mix:
            img = images[p.cp_index]
            cp = np.full((input_h, input_w, 3), 114, np.uint8)
            r = min(input_h / img.shape[0], input_w / img.shape[1])
            cp[:int(img.shape[0] * r), :int(img.shape[1] * r)] = resize(
                img, (int(img.shape[1] * r), int(img.shape[0] * r)))
            cp = resize(cp, (int(cp.shape[1] * p.jit), int(cp.shape[0] * p.jit)))
            if p.cp_flip:
                cp = cp[:, ::-1, :]
            oh, ow = cp.shape[:2]
            padded = np.zeros((max(oh, input_h), max(ow, input_w), 3), np.uint8)
            padded[:oh, :ow] = cp
            crop = padded[p.y_off:p.y_off + input_h, p.x_off:p.x_off + input_w]
            out = (0.5 * out.astype(np.float32) + 0.5 * crop.astype(np.float32)).astype(np.uint8)
        if p.do_hsv:
            out = apply_hsv(out, p.hsv)
        if p.flip:
            out = out[:, ::-1]
        out = letterbox_u8(out, input_h, input_w)
    else:
        img = images[p.indices[0]]
        if p.do_hsv:
            img = apply_hsv(img, p.hsv)
        if p.flip:
            img = img[:, ::-1]
        out = letterbox_u8(img, input_h, input_w)
    return np.ascontiguousarray(out.transpose(2, 0, 1), dtype=np.float32)
