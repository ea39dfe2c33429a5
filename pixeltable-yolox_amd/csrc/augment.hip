// Training-time augmentation on gfx950 for a whole batch (reference
// yolox/data/datasets/mosaicdetection.py:76-232 MosaicDetection.__getitem__ + mixup, and
// yolox/data/data_augment.py:19-232 augment_hsv / random_affine / _mirror / preproc /
// TrainTransform), as two launches over uint8 HWC (BGR) source images that live in one pool:
//
//   aug_mosaic_affine : per output pixel of the input_h x input_w image, the inverse affine
//       (cv2.warpAffine, INTER_LINEAR, border 114) lands in the 2H x 2W mosaic canvas; each of
//       the four canvas taps is computed on the fly -- 114, or the resized source image the
//       quadrant holds (cv2.resize INTER_LINEAR) -- so neither the canvas nor the resized
//       images are ever materialised;
//   aug_finish : mixup (the copy-paste image: letterbox, jitter resize, flip, pad/crop, then
//       uint8(0.5 a + 0.5 b)), augment_hsv (cv2 BGR<->HSV, 8-bit), the horizontal mirror and
//       the float32 CHW batch tensor the trainer reads; images without mosaic take
//       TrainTransform's letterbox path (HSV and mirror on the source taps, then resize).
//
// cv2 is absent from this image, so its published fixed-point schemes are restated (the
// oracle, oracle/augment_oracle.py, is the same restatement in numpy): resize as in
// preprocess.hip (11-bit coefficients; 2x downscale through INTER_AREA; r == 1 copies);
// warpAffine with AB_BITS 10 / INTER_BITS 5 coordinates and the 15-bit bilinear table
// ((32-fx)(32-fy)*32 ... exact, sum 32768), rounding (v + 2^14) >> 15; the 8-bit HSV
// conversions of RGB2HSV_b (hsv_shift 12 division tables) and HSV2RGB_b (float sectors,
// saturate_cast rounding half to even).  Parity vs cv2 itself is unpinned.
#include "yxh_common.hpp"

namespace yxh {

namespace {

constexpr int kAbBits = 10, kInterBits = 5, kInterTab = 1 << kInterBits;

struct Rs {  // one cv2.resize(src (sh x sw) -> (rh x rw)) sampler
    const uint8_t* src;
    int sh, sw, rh, rw, mode;  // mode 0 copy, 1 bilinear, 2 area-2x
    double sx, sy;
};

__device__ __forceinline__ void rs_coeff(int d, double scale, int ssize, int& s0, int& a0, int& a1) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)floorf(f);
    f -= (float)s;
    if (s < 0) { f = 0.0f; s = 0; }
    if (s >= ssize - 1) { f = 0.0f; s = ssize - 1; }
    s0 = s;
    a0 = (int)rintf((1.0f - f) * 2048.0f);
    a1 = (int)rintf(f * 2048.0f);
}

__device__ __forceinline__ Rs make_rs(const uint8_t* pool, long long off, int sh, int sw, int rh, int rw, double sx,
                                      double sy) {
    Rs r;
    r.src = pool + off;
    r.sh = sh; r.sw = sw; r.rh = rh; r.rw = rw; r.sx = sx; r.sy = sy;
    if (rw == sw && rh == sh)
        r.mode = 0;
    else if (fabs(sx - 2.0) < 2.220446049250313e-16 && fabs(sy - 2.0) < 2.220446049250313e-16)
        r.mode = 2;
    else
        r.mode = 1;
    return r;
}

// pixel (y, x) of the resized image, 3 channels (caller guarantees 0 <= y < rh, 0 <= x < rw)
__device__ __forceinline__ void rs_pixel(const Rs& p, int y, int x, int v[3]) {
    if (p.mode == 0) {
        const uint8_t* s = p.src + ((long long)y * p.sw + x) * 3;
        v[0] = s[0]; v[1] = s[1]; v[2] = s[2];
    } else if (p.mode == 2) {
        const uint8_t* s0 = p.src + ((long long)(2 * y) * p.sw + 2 * x) * 3;
        const uint8_t* s1 = s0 + (long long)p.sw * 3;
        for (int c = 0; c < 3; ++c) v[c] = (s0[c] + s0[c + 3] + s1[c] + s1[c + 3] + 2) >> 2;
    } else {
        int sx0, ax0, ax1, sy0, by0, by1;
        rs_coeff(x, p.sx, p.sw, sx0, ax0, ax1);
        rs_coeff(y, p.sy, p.sh, sy0, by0, by1);
        const int sx1 = min(sx0 + 1, p.sw - 1), sy1 = min(sy0 + 1, p.sh - 1);
        const uint8_t* r0 = p.src + (long long)sy0 * p.sw * 3;
        const uint8_t* r1 = p.src + (long long)sy1 * p.sw * 3;
        for (int c = 0; c < 3; ++c) {
            const int h0 = r0[sx0 * 3 + c] * ax0 + r0[sx1 * 3 + c] * ax1;
            const int h1 = r1[sx0 * 3 + c] * ax0 + r1[sx1 * 3 + c] * ax1;
            const int t = (((h0 >> 4) * by0) >> 16) + (((h1 >> 4) * by1) >> 16) + 2;
            v[c] = min(max(t >> 2, 0), 255);
        }
    }
}

// mosaic canvas pixel (cy, cx): the quadrant holding it, or 114
__device__ __forceinline__ void canvas_pixel(const uint8_t* pool, const yxh_aug_image& im, int cy, int cx, int v[3]) {
    for (int q = 0; q < 4; ++q) {
        if (cx >= im.lx1[q] && cx < im.lx2[q] && cy >= im.ly1[q] && cy < im.ly2[q]) {
            const Rs r = make_rs(pool, im.src_off[q], im.src_h[q], im.src_w[q], im.rh[q], im.rw[q], im.rsx[q],
                                 im.rsy[q]);
            rs_pixel(r, cy - im.ly1[q] + im.sy1[q], cx - im.lx1[q] + im.sx1[q], v);
            return;
        }
    }
    v[0] = v[1] = v[2] = 114;
}

__device__ __forceinline__ int sat_int(double v) {
    // saturate_cast<int>(double): round half to even, clamp
    const double r = rint(v);
    return r > 2147483647.0 ? 2147483647 : r < -2147483648.0 ? (int)0x80000000 : (int)r;
}

}  // namespace

// warpAffine of the (virtual) 2H x 2W mosaic canvas into the H x W output (uint8 HWC)
__global__ __launch_bounds__(256) void aug_mosaic_affine(const uint8_t* pool, const yxh_aug_image* images, int H,
                                                         int W, uint8_t* out) {
    const int b = blockIdx.y;
    const int pix = blockIdx.x * 256 + threadIdx.x;
    if (pix >= H * W) return;
    const yxh_aug_image& im = images[b];
    const int y = pix / W, x = pix - y * W;
    uint8_t* o = out + ((long long)b * H * W + pix) * 3;
    if (!im.mosaic) {  // no mosaic: aug_finish reads the source directly
        o[0] = o[1] = o[2] = 0;
        return;
    }
    const double* M = im.minv;  // dst -> canvas, cv2 invertAffineTransform of the sampled M
    const int rd = (1 << kAbBits) / kInterTab / 2;
    const int X0 = sat_int((M[1] * y + M[2]) * (1 << kAbBits)) + rd;
    const int Y0 = sat_int((M[4] * y + M[5]) * (1 << kAbBits)) + rd;
    const int X = (X0 + sat_int(M[0] * x * (1 << kAbBits))) >> (kAbBits - kInterBits);
    const int Y = (Y0 + sat_int(M[3] * x * (1 << kAbBits))) >> (kAbBits - kInterBits);
    const int sx = X >> kInterBits, sy = Y >> kInterBits;
    const int fx = X & (kInterTab - 1), fy = Y & (kInterTab - 1);
    const int CW = 2 * W, CH = 2 * H;
    if (sx >= CW || sx + 1 < 0 || sy >= CH || sy + 1 < 0) {
        o[0] = o[1] = o[2] = 114;
        return;
    }
    const int w00 = (kInterTab - fx) * (kInterTab - fy) * 32, w01 = fx * (kInterTab - fy) * 32;
    const int w10 = (kInterTab - fx) * fy * 32, w11 = fx * fy * 32;
    int v00[3], v01[3], v10[3], v11[3];
    auto tap = [&](int ty, int tx, int v[3]) {
        if ((unsigned)tx < (unsigned)CW && (unsigned)ty < (unsigned)CH)
            canvas_pixel(pool, im, ty, tx, v);
        else
            v[0] = v[1] = v[2] = 114;
    };
    tap(sy, sx, v00);
    tap(sy, sx + 1, v01);
    tap(sy + 1, sx, v10);
    tap(sy + 1, sx + 1, v11);
    for (int c = 0; c < 3; ++c) {
        const int t = (v00[c] * w00 + v01[c] * w01 + v10[c] * w10 + v11[c] * w11 + (1 << 14)) >> 15;
        o[c] = (uint8_t)min(max(t, 0), 255);
    }
}

namespace {

// cv2 RGB2HSV_b tables (hsv_shift 12): saturate_cast<int> of the double quotients
__device__ __forceinline__ int sdiv(int i) { return i ? (int)rint((double)(255 << 12) / i) : 0; }
__device__ __forceinline__ int hdiv180(int i) { return i ? (int)rint((double)(180 << 12) / (6.0 * i)) : 0; }

__device__ __forceinline__ void bgr2hsv(int b, int g, int r, int& h, int& s, int& v) {
    v = max(b, max(g, r));
    const int vmin = min(b, min(g, r));
    const int diff = v - vmin;
    const int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
    s = (diff * sdiv(v) + (1 << 11)) >> 12;
    h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))));
    h = (h * hdiv180(diff) + (1 << 11)) >> 12;
    h += h < 0 ? 180 : 0;
}

__device__ __forceinline__ int sat_u8(float v) { return min(max((int)rintf(v), 0), 255); }

__device__ __forceinline__ void hsv2bgr(int hi, int si, int vi, int& b, int& g, int& r) {
    float h = (float)hi, s = si * (1.f / 255.f), v = vi * (1.f / 255.f);
    float fb, fg, fr;
    if (s == 0.f) {
        fb = fg = fr = v;
    } else {
        const int sector_data[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
        h *= 6.f / 180.f;
        h = fmodf(h, 6.f);
        int sector = (int)floorf(h);
        h -= (float)sector;
        if ((unsigned)sector >= 6u) {
            sector = 0;
            h = 0.f;
        }
        float tab[4];
        tab[0] = v;
        tab[1] = v * (1.f - s);
        tab[2] = v * (1.f - s * h);
        tab[3] = v * (1.f - s * (1.f - h));
        fb = tab[sector_data[sector][0]];
        fg = tab[sector_data[sector][1]];
        fr = tab[sector_data[sector][2]];
    }
    b = sat_u8(fb * 255.f);
    g = sat_u8(fg * 255.f);
    r = sat_u8(fr * 255.f);
}

// augment_hsv on one BGR pixel (data_augment.py:19-30)
__device__ __forceinline__ void hsv_aug(const yxh_aug_image& im, int v[3]) {
    if (!im.do_hsv) return;
    int h, s, vv;
    bgr2hsv(v[0], v[1], v[2], h, s, vv);
    h = ((h + im.hsv[0]) % 180 + 180) % 180;
    s = min(max(s + im.hsv[1], 0), 255);
    vv = min(max(vv + im.hsv[2], 0), 255);
    hsv2bgr(h, s, vv, v[0], v[1], v[2]);
}

// pixel (y, x) of the letterbox canvas (H x W, 114 pad) of the copy-paste image
__device__ __forceinline__ void cp_canvas(const uint8_t* pool, const yxh_aug_image& im, int y, int x, int v[3]) {
    if (y < im.cp_rh && x < im.cp_rw) {
        const Rs r = make_rs(pool, im.cp_off, im.cp_h, im.cp_w, im.cp_rh, im.cp_rw, im.cp_sx, im.cp_sy);
        rs_pixel(r, y, x, v);
    } else {
        v[0] = v[1] = v[2] = 114;
    }
}

}  // namespace

__global__ __launch_bounds__(256) void aug_finish(const uint8_t* pool, const yxh_aug_image* images, const uint8_t* mos,
                                                  int H, int W, float* out) {
    const int b = blockIdx.y;
    const int pix = blockIdx.x * 256 + threadIdx.x;
    if (pix >= H * W) return;
    const yxh_aug_image& im = images[b];
    const int y = pix / W, x = pix - y * W;
    int v[3];
    if (im.mosaic) {
        const int xs = im.flip ? W - 1 - x : x;  // _mirror (data_augment.py:133-138)
        const uint8_t* m = mos + (((long long)b * H + y) * W + xs) * 3;
        v[0] = m[0]; v[1] = m[1]; v[2] = m[2];
        if (im.mix) {  // mixup (mosaicdetection.py:169-232)
            int c[3] = {0, 0, 0};
            const int py = y + im.y_off, px = xs + im.x_off;  // in the zero-padded copy-paste image
            if (py < im.jit_h && px < im.jit_w) {
                const int u = im.cp_flip ? im.jit_w - 1 - px : px;
                // cv2.resize of the H x W letterbox canvas to (jit_w, jit_h), INTER_LINEAR, taps on the fly
                if (im.jit_w == W && im.jit_h == H) {
                    cp_canvas(pool, im, py, u, c);
                } else {
                    int sx0, ax0, ax1, sy0, by0, by1;
                    rs_coeff(u, im.jit_sx, W, sx0, ax0, ax1);
                    rs_coeff(py, im.jit_sy, H, sy0, by0, by1);
                    const int sx1 = min(sx0 + 1, W - 1), sy1 = min(sy0 + 1, H - 1);
                    int t00[3], t01[3], t10[3], t11[3];
                    cp_canvas(pool, im, sy0, sx0, t00);
                    cp_canvas(pool, im, sy0, sx1, t01);
                    cp_canvas(pool, im, sy1, sx0, t10);
                    cp_canvas(pool, im, sy1, sx1, t11);
                    for (int k = 0; k < 3; ++k) {
                        const int h0 = t00[k] * ax0 + t01[k] * ax1, h1 = t10[k] * ax0 + t11[k] * ax1;
                        const int t = (((h0 >> 4) * by0) >> 16) + (((h1 >> 4) * by1) >> 16) + 2;
                        c[k] = min(max(t >> 2, 0), 255);
                    }
                }
            }
            for (int k = 0; k < 3; ++k) v[k] = (v[k] + c[k]) >> 1;  // uint8(0.5 a + 0.5 b), exact in fp32
        }
        hsv_aug(im, v);
    } else {
        // TrainTransform without mosaic: HSV + mirror on the source, then preproc's resize
        if (y < im.rh[0] && x < im.rw[0]) {
            const Rs r = make_rs(pool, im.src_off[0], im.src_h[0], im.src_w[0], im.rh[0], im.rw[0], im.rsx[0],
                                 im.rsy[0]);
            auto src_px = [&](int sy, int sx, int t[3]) {
                const int xx = im.flip ? r.sw - 1 - sx : sx;
                const uint8_t* s = r.src + ((long long)sy * r.sw + xx) * 3;
                t[0] = s[0]; t[1] = s[1]; t[2] = s[2];
                hsv_aug(im, t);
            };
            if (r.mode == 0) {
                src_px(y, x, v);
            } else if (r.mode == 2) {
                int a[3], bb[3], cc[3], d[3];
                src_px(2 * y, 2 * x, a);
                src_px(2 * y, 2 * x + 1, bb);
                src_px(2 * y + 1, 2 * x, cc);
                src_px(2 * y + 1, 2 * x + 1, d);
                for (int k = 0; k < 3; ++k) v[k] = (a[k] + bb[k] + cc[k] + d[k] + 2) >> 2;
            } else {
                int sx0, ax0, ax1, sy0, by0, by1;
                rs_coeff(x, r.sx, r.sw, sx0, ax0, ax1);
                rs_coeff(y, r.sy, r.sh, sy0, by0, by1);
                const int sx1 = min(sx0 + 1, r.sw - 1), sy1 = min(sy0 + 1, r.sh - 1);
                int t00[3], t01[3], t10[3], t11[3];
                src_px(sy0, sx0, t00);
                src_px(sy0, sx1, t01);
                src_px(sy1, sx0, t10);
                src_px(sy1, sx1, t11);
                for (int k = 0; k < 3; ++k) {
                    const int h0 = t00[k] * ax0 + t01[k] * ax1, h1 = t10[k] * ax0 + t11[k] * ax1;
                    const int t = (((h0 >> 4) * by0) >> 16) + (((h1 >> 4) * by1) >> 16) + 2;
                    v[k] = min(max(t >> 2, 0), 255);
                }
            }
        } else {
            v[0] = v[1] = v[2] = 114;
        }
    }
    const long long plane = (long long)H * W;
    float* o = out + (long long)b * 3 * plane + pix;
    o[0] = (float)v[0];
    o[plane] = (float)v[1];
    o[2 * plane] = (float)v[2];
}

int augment_batch_launch(const uint8_t* pool, const yxh_aug_image* images, int B, int H, int W, uint8_t* mosaic_ws,
                         float* out, hipStream_t st) {
    YXH_CHECK_ARG(pool && images && mosaic_ws && out, "null pointer");
    YXH_CHECK_ARG(B > 0 && H > 0 && W > 0 && (long long)H * W < (1LL << 30), "augment sizes B=%d %dx%d", B, H, W);
    const dim3 grid((H * W + 255) / 256, B);
    hipLaunchKernelGGL(aug_mosaic_affine, grid, dim3(256), 0, st, pool, images, H, W, mosaic_ws);
    YXH_CHECK_LAUNCH("aug_mosaic_affine");
    hipLaunchKernelGGL(aug_finish, grid, dim3(256), 0, st, pool, images, mosaic_ws, H, W, out);
    YXH_CHECK_LAUNCH("aug_finish");
    return YXH_OK;
}

}  // namespace yxh
