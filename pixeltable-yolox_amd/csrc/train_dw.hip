// Depthwise convolution training kernels (DWConv.dconv of yolox_nano: network_blocks.py:55-74,
// groups = channels, 3x3, stride 1 or 2) -- the gradients autograd computes for
// F.conv2d(x, w, groups=C) in the reference's train step (trainer.py:104-112).
//
//  dw_wgrad        : dw[c][tap] partial sums over a pixel range per block, into a workspace
//  dw_wgrad_reduce : the partials summed over blocks in a fixed order (deterministic, no atomics)
//  dw_dgrad        : dx[b][iy][ix][c] (+)= sum over taps of dy[b][oy][ox][c] * w[c][tap]
//
// All three are HBM-bound VALU kernels: a depthwise conv does 9 multiply-adds per element, far
// below the MFMA roofline, and nothing here is reshaped into a GEMM.  NHWC activations: a wave
// reads consecutive channels of consecutive pixels (16-byte chunks per lane).
#include "conv_common.hpp"

namespace yxh {

namespace {

constexpr int kDwThreads = 256;

// One block: a range of output pixels x a slice of CS channels (CS <= 64).  Thread t handles
// channel c0 + (t % CS) of pixel slot t / CS (256 / CS slots), walking the block's pixels with
// that stride; per-thread partial sums of the K*K taps, then a fixed-order LDS reduction over the
// slots, one partial per (block, channel, tap) into the workspace.
template <typename T, int K>
__global__ __launch_bounds__(kDwThreads) void dw_wgrad(const T* __restrict__ x, int xcs, long long xbs, int in_h,
                                                        int in_w, const T* __restrict__ dy, int dycs, long long dybs,
                                                        int out_h, int out_w, int batch, int C, int CS, int stride,
                                                        int pad, int pix_per_block, float* __restrict__ part) {
    __shared__ float red[kDwThreads][K * K];
    const int tid = threadIdx.x;
    const int c0 = blockIdx.y * CS;
    const int slots = kDwThreads / CS;
    const int cl = tid % CS, slot = tid / CS;
    const int c = c0 + cl;
    const long long M = (long long)batch * out_h * out_w;
    const long long m0 = (long long)blockIdx.x * pix_per_block;
    const long long m1 = min(M, m0 + pix_per_block);
    float acc[K * K];
#pragma unroll
    for (int t = 0; t < K * K; ++t) acc[t] = 0.0f;
    const int ohw = out_h * out_w;
    if (slot < slots && c < C) {
        for (long long m = m0 + slot; m < m1; m += slots) {
            const int b = (int)(m / ohw), pix = (int)(m - (long long)b * ohw);
            const int oy = pix / out_w, ox = pix - oy * out_w;
            const float g = to_f32(dy[b * dybs + (long long)pix * dycs + c]);
            const T* xb = x + b * xbs + c;
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
                const int iy = oy * stride - pad + ky;
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
                    const int ix = ox * stride - pad + kx;
                    const bool ok = (unsigned)iy < (unsigned)in_h && (unsigned)ix < (unsigned)in_w;
                    const float v = ok ? to_f32(xb[((long long)iy * in_w + ix) * xcs]) : 0.0f;
                    acc[ky * K + kx] += g * v;
                }
            }
        }
    }
#pragma unroll
    for (int t = 0; t < K * K; ++t) red[tid][t] = acc[t];
    __syncthreads();
    // slot s of channel cl lives in thread s * CS + cl: sum the slots in order
    for (int q = tid; q < CS * K * K; q += kDwThreads) {
        const int ch = q % CS, t = q / CS;
        if (c0 + ch < C) {
            float s = 0.0f;
            for (int sl = 0; sl < slots; ++sl) s += red[sl * CS + ch][t];
            part[((long long)blockIdx.x * C + c0 + ch) * (K * K) + t] = s;
        }
    }
}

__global__ __launch_bounds__(kDwThreads) void dw_wgrad_reduce(const float* __restrict__ part, int nsplit, int n,
                                                             float* __restrict__ dw) {
    const int i = blockIdx.x * kDwThreads + threadIdx.x;
    if (i >= n) return;
    float s = 0.0f;
    for (int k = 0; k < nsplit; ++k) s += part[(long long)k * n + i];
    dw[i] = s;
}

// One thread: EPC channels (one 16-byte chunk of dy) of one input pixel.
template <typename T, int K>
__global__ __launch_bounds__(kDwThreads) void dw_dgrad(const T* __restrict__ dy, int dycs, long long dybs, int out_h,
                                                        int out_w, const T* __restrict__ w, int C, int stride, int pad,
                                                        int in_h, int in_w, int batch, float* __restrict__ dx, int dxcs,
                                                        long long dxbs, int accumulate) {
    constexpr int EPC = Chunk<T>::N;
    const int nch = (C + EPC - 1) / EPC;
    const long long idx = (long long)blockIdx.x * kDwThreads + threadIdx.x;
    const long long total = (long long)batch * in_h * in_w * nch;
    if (idx >= total) return;
    const int q = (int)(idx % nch);
    const long long m = idx / nch;
    const int ihw = in_h * in_w;
    const int b = (int)(m / ihw), pix = (int)(m - (long long)b * ihw);
    const int iy = pix / in_w, ix = pix - iy * in_w;
    const int c0 = q * EPC;
    float acc[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) acc[e] = 0.0f;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
        const int ty = iy + pad - ky;  // = oy * stride
        if (ty < 0 || ty % stride) continue;
        const int oy = ty / stride;
        if (oy >= out_h) continue;
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
            const int tx = ix + pad - kx;
            if (tx < 0 || tx % stride) continue;
            const int ox = tx / stride;
            if (ox >= out_w) continue;
            const T* g = dy + b * dybs + ((long long)oy * out_w + ox) * dycs + c0;
            T gv[EPC];
            if (c0 + EPC <= C) {
                const uint4 u = *(const uint4*)g;
                __builtin_memcpy(gv, &u, 16);
            } else {
#pragma unroll
                for (int e = 0; e < EPC; ++e) gv[e] = c0 + e < C ? g[e] : (T)0.0f;
            }
#pragma unroll
            for (int e = 0; e < EPC; ++e)
                if (c0 + e < C) acc[e] += to_f32(gv[e]) * to_f32(w[(c0 + e) * (K * K) + ky * K + kx]);
        }
    }
    float* d = dx + b * dxbs + (long long)pix * dxcs + c0;
#pragma unroll
    for (int e = 0; e < EPC; ++e)
        if (c0 + e < C) d[e] = accumulate ? d[e] + acc[e] : acc[e];
}

int elem_bytes(int dt) { return dt == YXH_F32 ? 4 : 2; }

}  // namespace

size_t dw_wgrad_workspace_bytes(long long pixels, int channels, int k) {
    const long long per = 4096;  // output pixels per block (one partial per block, channel, tap)
    const long long nsplit = (pixels + per - 1) / per;
    return (size_t)(nsplit * channels * k * k * 4);
}

int dw_wgrad_launch(int dt, int B, const yxh_src* x, const yxh_src* dy, int C, int k, int stride, int pad, int out_h,
                    int out_w, float* dw, void* ws, size_t ws_bytes, hipStream_t st) {
    YXH_CHECK_ARG(x && dy && dw && ws && x->ptr && dy->ptr, "dw_wgrad: null pointer");
    YXH_CHECK_ARG(k == 3 && (stride == 1 || stride == 2) && pad == 1, "dw_wgrad: 3x3, stride 1/2, pad 1 only");
    YXH_CHECK_ARG(B > 0 && C > 0 && x->channels == C && dy->channels >= C && !x->upsample && !dy->upsample &&
                      dy->h == out_h && dy->w == out_w && out_h == (x->h + 2 * pad - k) / stride + 1 &&
                      out_w == (x->w + 2 * pad - k) / stride + 1,
                  "dw_wgrad: views do not match a %dx%d s%d conv over %d channels", k, k, stride, C);
    YXH_CHECK_ARG(dt == YXH_F32 || dt == YXH_BF16 || dt == YXH_F16, "dw_wgrad dtype %d", dt);
    const long long M = (long long)B * out_h * out_w;
    const int per = 4096;
    const long long nsplit = (M + per - 1) / per;
    YXH_CHECK_ARG(ws_bytes >= dw_wgrad_workspace_bytes(M, C, k) && nsplit < 65536, "dw_wgrad: workspace too small");
    const int CS = C < 64 ? C : 64;
    dim3 grid((unsigned)nsplit, (unsigned)((C + CS - 1) / CS));
    float* part = (float*)ws;
#define YXH_DWW(T)                                                                                                  \
    hipLaunchKernelGGL((dw_wgrad<T, 3>), grid, dim3(kDwThreads), 0, st, (const T*)x->ptr, x->cstride, x->bstride,   \
                       x->h, x->w, (const T*)dy->ptr, dy->cstride, dy->bstride, out_h, out_w, B, C, CS, stride, pad, \
                       per, part)
    if (dt == YXH_F32) YXH_DWW(float);
    else if (dt == YXH_BF16) YXH_DWW(bf16);
    else YXH_DWW(f16);
#undef YXH_DWW
    YXH_CHECK_LAUNCH("dw_wgrad");
    const int n = C * k * k;
    hipLaunchKernelGGL(dw_wgrad_reduce, dim3((unsigned)((n + kDwThreads - 1) / kDwThreads)), dim3(kDwThreads), 0, st,
                       part, (int)nsplit, n, dw);
    YXH_CHECK_LAUNCH("dw_wgrad_reduce");
    return YXH_OK;
}

int dw_dgrad_launch(int dt, int B, const yxh_src* dy, const void* w, int C, int k, int stride, int pad, int in_h,
                    int in_w, float* dx, int dxcs, long long dxbs, int accumulate, hipStream_t st) {
    YXH_CHECK_ARG(dy && dy->ptr && w && dx, "dw_dgrad: null pointer");
    YXH_CHECK_ARG(k == 3 && (stride == 1 || stride == 2) && pad == 1, "dw_dgrad: 3x3, stride 1/2, pad 1 only");
    YXH_CHECK_ARG(dt == YXH_F32 || dt == YXH_BF16 || dt == YXH_F16, "dw_dgrad dtype %d", dt);
    const int es = elem_bytes(dt);
    YXH_CHECK_ARG(B > 0 && C > 0 && dy->channels >= C && !dy->upsample && dy->h == (in_h + 2 * pad - k) / stride + 1 &&
                      dy->w == (in_w + 2 * pad - k) / stride + 1 && ((uintptr_t)dy->ptr % 16) == 0 &&
                      (dy->cstride * es) % 16 == 0 && (dy->bstride * es) % 16 == 0 && dxcs >= C,
                  "dw_dgrad: dy view (16-byte rows) does not match the input size");
    const int epc = 16 / es;
    const long long total = (long long)B * in_h * in_w * ((C + epc - 1) / epc);
    dim3 grid((unsigned)((total + kDwThreads - 1) / kDwThreads));
#define YXH_DWD(T)                                                                                                     \
    hipLaunchKernelGGL((dw_dgrad<T, 3>), grid, dim3(kDwThreads), 0, st, (const T*)dy->ptr, dy->cstride, dy->bstride, \
                       dy->h, dy->w, (const T*)w, C, stride, pad, in_h, in_w, B, dx, dxcs, dxbs, accumulate)
    if (dt == YXH_F32) YXH_DWD(float);
    else if (dt == YXH_BF16) YXH_DWD(bf16);
    else YXH_DWD(f16);
#undef YXH_DWD
    YXH_CHECK_LAUNCH("dw_dgrad");
    return YXH_OK;
}

}  // namespace yxh
