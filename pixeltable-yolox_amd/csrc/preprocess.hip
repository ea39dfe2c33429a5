// Letterbox pre-processing on gfx950: data_augment.py:140-156 `preproc` /
// ValTransform (processor.py:30-37) for one uint8 HWC RGB image:
//   r = min(th/h, tw/w); resize to (int(w*r), int(h*r)) with cv2 INTER_LINEAR;
//   paste top-left into a 114-filled canvas; emit float32 CHW (the reference's
//   tensor) or uint8 HWC (the fast path consumed directly by yxh_focus_pack).
//
// cv2 (opencv-python 4.10, reference poetry.lock) is absent here, so its published
// fixed-point scheme is restated: 11-bit coefficients (saturate_cast<short>(c*2048),
// round-half-even), source clamp at the borders, horizontal int sums, vertical
// combine as in VResizeLinearVec_32s8u: ((S0>>4)*b0 >> 16) + ((S1>>4)*b1 >> 16) + 2 >> 2;
// exact 2x downscale takes cv2's INTER_AREA fast path ((a+b+c+d+2)>>2); r == 1 is a
// copy.  Only the r == 1 case is pinned (letterbox parity).
#include "yxh_common.hpp"

namespace yxh {

struct LbParams {
    int sh, sw, rh, rw, th, tw, mode;  // mode 0 copy, 1 bilinear, 2 area-2x
    double sx, sy;                     // source/dest scale (cv2 scale_x / scale_y)
    int out_nchw;                      // 1: float32 [3][th][tw]; 0: uint8 [th][tw][3]
};

__device__ __forceinline__ void coeff(int d, double scale, int ssize, int& s0, int& a0, int& a1) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)floorf(f);
    f -= (float)s;
    if (s < 0) { f = 0.0f; s = 0; }
    if (s >= ssize - 1) { f = 0.0f; s = ssize - 1; }
    s0 = s;
    a0 = (int)rintf((1.0f - f) * 2048.0f);
    a1 = (int)rintf(f * 2048.0f);
}

__global__ __launch_bounds__(256) void letterbox(const uint8_t* src, void* dst, LbParams p) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= p.th * p.tw) return;
    const int y = idx / p.tw, x = idx - y * p.tw;
    int v[3] = {114, 114, 114};
    if (y < p.rh && x < p.rw) {
        if (p.mode == 0) {
            const uint8_t* s = src + ((long long)y * p.sw + x) * 3;
            v[0] = s[0]; v[1] = s[1]; v[2] = s[2];
        } else if (p.mode == 2) {
            const uint8_t* s0 = src + ((long long)(2 * y) * p.sw + 2 * x) * 3;
            const uint8_t* s1 = s0 + (long long)p.sw * 3;
            for (int c = 0; c < 3; ++c) v[c] = (s0[c] + s0[c + 3] + s1[c] + s1[c + 3] + 2) >> 2;
        } else {
            int sx0, ax0, ax1, sy0, by0, by1;
            coeff(x, p.sx, p.sw, sx0, ax0, ax1);
            coeff(y, p.sy, p.sh, sy0, by0, by1);
            const int sx1 = min(sx0 + 1, p.sw - 1), sy1 = min(sy0 + 1, p.sh - 1);
            const uint8_t* r0 = src + (long long)sy0 * p.sw * 3;
            const uint8_t* r1 = src + (long long)sy1 * p.sw * 3;
            for (int c = 0; c < 3; ++c) {
                const int h0 = r0[sx0 * 3 + c] * ax0 + r0[sx1 * 3 + c] * ax1;
                const int h1 = r1[sx0 * 3 + c] * ax0 + r1[sx1 * 3 + c] * ax1;
                const int t = (((h0 >> 4) * by0) >> 16) + (((h1 >> 4) * by1) >> 16) + 2;
                v[c] = min(max(t >> 2, 0), 255);
            }
        }
    }
    if (p.out_nchw) {
        float* d = (float*)dst;
        for (int c = 0; c < 3; ++c) d[(long long)c * p.th * p.tw + idx] = (float)v[c];
    } else {
        uint8_t* d = (uint8_t*)dst + (long long)idx * 3;
        d[0] = (uint8_t)v[0]; d[1] = (uint8_t)v[1]; d[2] = (uint8_t)v[2];
    }
}

int letterbox_launch(const uint8_t* src, int sh, int sw, int th, int tw, int out_nchw, void* dst, hipStream_t st) {
    YXH_CHECK_ARG(src && dst, "null pointer");
    YXH_CHECK_ARG(sh > 0 && sw > 0 && th > 0 && tw > 0, "letterbox sizes");
    const double r = fmin((double)th / sh, (double)tw / sw);
    LbParams p;
    p.sh = sh; p.sw = sw; p.th = th; p.tw = tw;
    p.rw = (int)(sw * r);
    p.rh = (int)(sh * r);
    YXH_CHECK_ARG(p.rw > 0 && p.rh > 0, "degenerate resize");
    p.sx = 1.0 / ((double)p.rw / sw);
    p.sy = 1.0 / ((double)p.rh / sh);
    p.out_nchw = out_nchw;
    if (p.rw == sw && p.rh == sh)
        p.mode = 0;
    else if (fabs(p.sx - 2.0) < 2.220446049250313e-16 && fabs(p.sy - 2.0) < 2.220446049250313e-16)
        p.mode = 2;
    else
        p.mode = 1;
    hipLaunchKernelGGL(letterbox, dim3((th * tw + 255) / 256), dim3(256), 0, st, src, dst, p);
    YXH_CHECK_LAUNCH("letterbox");
    return YXH_OK;
}

}  // namespace yxh
