// Letterbox pre-processing on gfx950: data_augment.py:140-156 `preproc` /
// ValTransform (processor.py:30-37) for a whole batch of uint8 HWC RGB images in ONE
// launch:
//   r = min(th/h, tw/w); resize to (int(w*r), int(h*r)) with cv2 INTER_LINEAR;
//   paste top-left into a 114-filled canvas; emit float32 NCHW (the reference's
//   tensor), uint8 NHWC or bf16 NHWC (both read directly by the fused Focus+stem conv).
//
// The source images live in one pool (a single H2D copy from pinned staging); each
// image's descriptor gives its byte offset and size.  Work unit: 4 consecutive output
// pixels of one row per lane, so a wave reads 64 x 12 contiguous source bytes (dword
// loads when aligned) and writes 64 x 16-byte float4 per NCHW plane / 64 x 12 u8 /
// 64 x 24 bf16 bytes -- coalesced on both sides.  Per-image resize parameters are
// computed once per block into LDS.
//
// cv2 (opencv-python 4.10, reference poetry.lock) is absent here, so its published
// fixed-point scheme is restated for r != 1: 11-bit coefficients (saturate_cast<short>
// (c*2048), round-half-even), source clamp at the borders, horizontal int sums,
// vertical combine as in VResizeLinearVec_32s8u: ((S0>>4)*b0 >> 16) + ((S1>>4)*b1 >> 16)
// + 2 >> 2; exact 2x downscale takes cv2's INTER_AREA fast path ((a+b+c+d+2)>>2); r == 1
// is a copy.  Only r == 1 is pinned to the reference; cv2 finishes each row's SIMD
// remainder with the scalar (b0*S0 + b1*S1 + 2^21) >> 22, which can differ by 1 on those
// pixels, so r != 1 is parity-unpinned (letterbox parity).
#include "yxh_common.hpp"

namespace yxh {

namespace {

struct LbParams {
    int sh, sw, rh, rw, mode;  // mode 0 copy, 1 bilinear, 2 area-2x
    double sx, sy;             // source/dest scale (cv2 scale_x / scale_y)
    long long off;
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

__device__ void lb_params(const yxh_lb_image& im, int th, int tw, LbParams& p) {
    p.sh = im.src_h;
    p.sw = im.src_w;
    p.off = im.src_offset;
    const double r = fmin((double)th / p.sh, (double)tw / p.sw);
    p.rw = (int)(p.sw * r);
    p.rh = (int)(p.sh * r);
    p.sx = 1.0 / ((double)p.rw / p.sw);
    p.sy = 1.0 / ((double)p.rh / p.sh);
    if (p.rw == p.sw && p.rh == p.sh)
        p.mode = 0;
    else if (fabs(p.sx - 2.0) < 2.220446049250313e-16 && fabs(p.sy - 2.0) < 2.220446049250313e-16)
        p.mode = 2;
    else
        p.mode = 1;
}

__device__ __forceinline__ void pixel(const uint8_t* src, const LbParams& p, int y, int x, int v[3]) {
    v[0] = v[1] = v[2] = 114;
    if (y >= p.rh || x >= p.rw) return;
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

}  // namespace

__global__ __launch_bounds__(256) void letterbox_batch(const uint8_t* pool, const yxh_lb_image* images, int th,
                                                       int tw, int fmt, void* dst) {
    __shared__ LbParams sp;
    const int b = blockIdx.y;
    if (threadIdx.x == 0) lb_params(images[b], th, tw, sp);
    __syncthreads();
    const LbParams p = sp;
    const int qpr = tw >> 2;  // 4-pixel quads per row
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= th * qpr) return;
    const int y = q / qpr, x0 = (q - y * qpr) * 4;
    const uint8_t* src = pool + p.off;
    uint32_t w[3];  // 12 bytes: 4 RGB pixels
    if (p.mode == 0 && y < p.rh && x0 + 3 < p.rw) {
        const uint8_t* s = src + ((long long)y * p.sw + x0) * 3;
        if (((uintptr_t)s & 3) == 0) {
            w[0] = ((const uint32_t*)s)[0];
            w[1] = ((const uint32_t*)s)[1];
            w[2] = ((const uint32_t*)s)[2];
        } else {
            uint8_t t[12];
#pragma unroll
            for (int i = 0; i < 12; ++i) t[i] = s[i];
            __builtin_memcpy(w, t, 12);
        }
    } else {
        uint8_t t[12];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int v[3];
            pixel(src, p, y, x0 + k, v);
            t[3 * k] = (uint8_t)v[0];
            t[3 * k + 1] = (uint8_t)v[1];
            t[3 * k + 2] = (uint8_t)v[2];
        }
        __builtin_memcpy(w, t, 12);
    }
    const long long pix = ((long long)b * th + y) * tw + x0;  // first output pixel of the quad
    if (fmt == YXH_LB_F32_NCHW) {
        uint8_t t[12];
        __builtin_memcpy(t, w, 12);
        float* d = (float*)dst + (long long)b * 3 * th * tw + (long long)y * tw + x0;
        const long long plane = (long long)th * tw;
#pragma unroll
        for (int c = 0; c < 3; ++c)
            *(float4*)(d + c * plane) = make_float4(t[c], t[3 + c], t[6 + c], t[9 + c]);
    } else if (fmt == YXH_LB_U8_NHWC) {
        uint32_t* d = (uint32_t*)((uint8_t*)dst + pix * 3);
        d[0] = w[0]; d[1] = w[1]; d[2] = w[2];
    } else {  // bf16 NHWC: 12 values -> 24 bytes (exact: integers 0..255)
        uint8_t t[12];
        __builtin_memcpy(t, w, 12);
        uint32_t o[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const bf16 lo = (bf16)(float)t[2 * i], hi = (bf16)(float)t[2 * i + 1];
            o[i] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
        }
        uint2* d = (uint2*)((uint8_t*)dst + pix * 6);
        d[0] = make_uint2(o[0], o[1]);
        d[1] = make_uint2(o[2], o[3]);
        d[2] = make_uint2(o[4], o[5]);
    }
}

int letterbox_batch_launch(const uint8_t* pool, const yxh_lb_image* images, int B, int th, int tw, int fmt,
                           void* dst, hipStream_t st) {
    YXH_CHECK_ARG(pool && images && dst, "null pointer");
    YXH_CHECK_ARG(B > 0 && th > 0 && tw > 0, "letterbox sizes B=%d %dx%d", B, th, tw);
    YXH_CHECK_ARG(tw % 4 == 0, "letterbox canvas width %d must be a multiple of 4", tw);
    YXH_CHECK_ARG(fmt == YXH_LB_F32_NCHW || fmt == YXH_LB_U8_NHWC || fmt == YXH_LB_BF16_NHWC,
                  "letterbox output format %d", fmt);
    YXH_CHECK_ARG(((uintptr_t)dst & 15) == 0, "letterbox dst must be 16-byte aligned");
    const int quads = th * (tw / 4);
    hipLaunchKernelGGL(letterbox_batch, dim3((quads + 255) / 256, B), dim3(256), 0, st, pool, images, th, tw, fmt,
                       dst);
    YXH_CHECK_LAUNCH("letterbox_batch");
    return YXH_OK;
}

// ---------------------------------------------------------------- multiscale resize
// YoloxConfig.preprocess (config.py:296-305): F.interpolate(inputs, size=tsize, mode="bilinear",
// align_corners=False) of the [B, C, H, W] training batch.  The arithmetic is ATen's bilinear
// kernel term for term, in fp32 whatever the storage type (accscalar_t): scale = in / out,
// src = max(scale * (dst + 0.5) - 0.5, 0), i0 = (int)src, i1 = i0 + (i0 < in - 1), l1 = src - i0,
// l0 = 1 - l1, out = l0y * (l0x * a + l1x * b) + l1y * (l0x * c + l1x * d) with ATen's fma
// grouping (measured: tools/resize_probe.hip), rounded once to the storage type -- so the device
// result is bit-identical to the reference's own call on this GPU (tests/test_gpu_augment.py
// compares with torch's F.interpolate on the device).  Same size: a copy.
// One thread per output element, x fastest: each wave reads two input rows of one plane.
template <typename T>
__global__ __launch_bounds__(256) void resize_bilinear(const T* __restrict__ src, int planes, int ih, int iw,
                                                       T* __restrict__ dst, int oh, int ow, float rh, float rw) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long total = (long long)planes * oh * ow;
    if (idx >= total) return;
    const int ox = (int)(idx % ow);
    const long long r = idx / ow;
    const int oy = (int)(r % oh);
    const long long pl = r / oh;
    const T* s = src + pl * ih * iw;
    if (ih == oh && iw == ow) {
        dst[idx] = s[(long long)oy * iw + ox];
        return;
    }
    float hr = rh * ((float)oy + 0.5f) - 0.5f;
    hr = hr < 0.0f ? 0.0f : hr;
    const int h1 = (int)hr;
    const int h1p = h1 < ih - 1 ? 1 : 0;
    const float h1l = hr - (float)h1;
    const float h0l = 1.0f - h1l;
    float wr = rw * ((float)ox + 0.5f) - 0.5f;
    wr = wr < 0.0f ? 0.0f : wr;
    const int w1 = (int)wr;
    const int w1p = w1 < iw - 1 ? 1 : 0;
    const float w1l = wr - (float)w1;
    const float w0l = 1.0f - w1l;
    const T* r0 = s + (long long)h1 * iw + w1;
    const T* r1 = r0 + (long long)h1p * iw;
    // the contraction ATen's kernel gets from the compiler, spelled out (tools/resize_probe.hip: of
    // the fma groupings of this sum only this one matches F.interpolate on gfx950 bit for bit)
    const float v = __builtin_fmaf(h0l, __builtin_fmaf(w0l, to_f32(r0[0]), w1l * to_f32(r0[w1p])),
                                   h1l * __builtin_fmaf(w0l, to_f32(r1[0]), w1l * to_f32(r1[w1p])));
    dst[idx] = from_f32<T>(v);
}

int resize_bilinear_launch(int dt, int B, int C, int ih, int iw, const void* src, int oh, int ow, void* dst,
                           hipStream_t st) {
    YXH_CHECK_ARG(src && dst, "resize: null pointer");
    YXH_CHECK_ARG(B > 0 && C > 0 && ih > 0 && iw > 0 && oh > 0 && ow > 0, "resize sizes");
    YXH_CHECK_ARG(dt == YXH_F32 || dt == YXH_BF16 || dt == YXH_F16, "resize dtype %d", dt);
    const long long total = (long long)B * C * oh * ow;
    YXH_CHECK_ARG(total < (1LL << 40), "resize: too many elements");
    // area_pixel_compute_scale<float>: (float)input_size / output_size
    const float rh = (float)ih / (float)oh, rw = (float)iw / (float)ow;
    dim3 grid((unsigned)((total + 255) / 256));
#define YXH_RS(T) hipLaunchKernelGGL(resize_bilinear<T>, grid, dim3(256), 0, st, (const T*)src, B * C, ih, iw, (T*)dst, \
                                     oh, ow, rh, rw)
    if (dt == YXH_F32) YXH_RS(float);
    else if (dt == YXH_BF16) YXH_RS(bf16);
    else YXH_RS(f16);
#undef YXH_RS
    YXH_CHECK_LAUNCH("resize_bilinear");
    return YXH_OK;
}

}  // namespace yxh
