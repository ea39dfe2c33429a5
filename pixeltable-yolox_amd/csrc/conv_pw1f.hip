// conv_pw1f: fp32 1x1 stride-1 conv as a GEMM for the training path (BASELINE configs[2] trains in
// fp32: the 1x1 BaseConvs' forward, network_blocks.py:48-49 with ksize 1 -- CSP conv1/2/3, SPP convs,
// PAFPN laterals, head stems, head preds -- and their data gradients, which are 1x1 convs with the
// transposed weights of yxh_pack_dgrad_weight accumulated into the fp32 input gradient).
//
// Y[p][n] (+)= sum_k X[p][k] W[n][k]: D = W . X^T on v_mfma_f32_16x16x4_f32 with both operands read
// k-minor from LDS (lane l: A = W[n0 + l % 16][k + l / 16], B = X[p0 + l % 16][k + l / 16]), so the
// pixel-major activations need no transpose.  A block computes TN channels x TM pixels; each K stage
// (32 channels) of both operands arrives by 16-byte register loads into a double-buffered LDS image
// (rows padded by 4 floats: a ds_read_b32 of 16 rows x 4 k-columns is at most 2-way conflicted, and
// reads are 1/16 of the MFMA issue), the next stage's loads flying under this stage's MFMAs.  The
// 16x16 result fragments hold 4 consecutive channels of one pixel per lane: one 16-byte store (or
// read-add-store under YXH_CONV_ACCUMULATE) per lane and fragment.
#include "conv_common.hpp"

namespace yxh {

template <int TN, int TM, int WN, int WM>
__global__ __launch_bounds__(256) void conv_pw1f(ConvParams p, int ntn) {
    static_assert(WN * WM == 4, "4 waves");
    constexpr int KC = 32, KP = KC + 4;  // K stage, LDS row pitch (floats)
    constexpr int WTN = TN / WN, WTM = TM / WM, FR = WTN / 16, FC = WTM / 16;
    constexpr int ACH = TN * KC / 4, BCH = TM * KC / 4, AL = (ACH + 255) / 256, BL = (BCH + 255) / 256;
    constexpr int ASZ = TN * KP, BSZ = TM * KP;
    __shared__ __attribute__((aligned(16))) float lds[2][ASZ + BSZ];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wn = wave % WN, wm = wave / WN;
    const int n0 = (blockIdx.x % ntn) * TN, m0 = (blockIdx.x / ntn) * TM;
    const int M = p.M, cout = p.cout, cin = p.cin;
    const int nk = (cin + KC - 1) / KC;
    const float* W = (const float*)p.w;
    const int c0 = p.src0_ch;

    // per-thread pixel source offsets (fixed for the block): row r of the X tile -> pixel m0 + r
    long long xoff0[BL], xoff1[BL];
#pragma unroll
    for (int i = 0; i < BL; ++i) {
        const int q = tid + 256 * i;
        const int r = q / (KC / 4);
        const int m = min(m0 + r, M - 1);
        const int b = m / p.ohw, pix = m - b * p.ohw;
        int spix = pix;
        if (p.sup[0]) {
            const int y = pix / p.out_w, x = pix - y * p.out_w;
            spix = (y >> 1) * p.sw[0] + (x >> 1);
        }
        xoff0[i] = (long long)b * p.sbs[0] + (long long)spix * p.scs[0];
        xoff1[i] = p.nsrc > 1 ? (long long)b * p.sbs[1] + (long long)pix * p.scs[1] : 0;
    }

    float4 ra[AL], rb[BL];
    auto gload = [&](int kb) {
        const int k0 = kb * KC;
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            const int r = q / (KC / 4), c = k0 + (q % (KC / 4)) * 4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < ACH && n0 + r < cout && c < cin) v = *(const float4*)(W + (long long)(n0 + r) * cin + c);
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            const int c = k0 + (q % (KC / 4)) * 4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < BCH && c < cin) {
                if (p.nsrc > 1 && c >= c0) v = *(const float4*)((const float*)p.sptr[1] + xoff1[i] + (c - c0));
                else v = *(const float4*)((const float*)p.sptr[0] + xoff0[i] + c);
            }
            rb[i] = v;
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            if (q < ACH) *(float4*)(lds[buf] + (q / (KC / 4)) * KP + (q % (KC / 4)) * 4) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            if (q < BCH) *(float4*)(lds[buf] + ASZ + (q / (KC / 4)) * KP + (q % (KC / 4)) * 4) = rb[i];
        }
    };

    f32x4 acc[FR][FC];
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fk = lane >> 4;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int kb = 0; kb < nk; ++kb) {
        const int buf = kb & 1;
        const bool more = kb + 1 < nk;
        if (more) gload(kb + 1);
        const float* A = lds[buf] + (wn * WTN + fr) * KP + fk;
        const float* B = lds[buf] + ASZ + (wm * WTM + fr) * KP + fk;
#pragma unroll
        for (int kk = 0; kk < KC / 4; ++kk) {
            float a[FR], b[FC];
#pragma unroll
            for (int i = 0; i < FR; ++i) a[i] = A[i * 16 * KP + 4 * kk];
#pragma unroll
            for (int j = 0; j < FC; ++j) b[j] = B[j * 16 * KP + 4 * kk];
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (more) lstore(buf ^ 1);
        __syncthreads();
    }

    // D[n][p] of fragment (i, j): this lane holds channels 4 (lane / 16) + r of pixel lane % 16
    float* dst = (float*)p.dst;
#pragma unroll
    for (int j = 0; j < FC; ++j) {
        const int m = m0 + wm * WTM + 16 * j + fr;
        if (m >= M) continue;
        long long off;
        if (p.dst_dense) {
            off = (long long)m * p.dst_cs;
        } else {
            const int b = m / p.ohw;
            off = (long long)b * p.dst_bs + (long long)(m - b * p.ohw) * p.dst_cs;
        }
#pragma unroll
        for (int i = 0; i < FR; ++i) {
            const int n = n0 + wn * WTN + 16 * i + 4 * fk;
            if (n >= cout) continue;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
                v[r] = apply_act<true>(acc[i][j][r] + (p.bias && n + r < cout ? p.bias[n + r] : 0.0f), p.act);
            float* dp = dst + off + n;
            if (n + 3 < cout) {
                if (p.accum) {
                    const float4 o = *(const float4*)dp;
                    v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
                }
                *(float4*)dp = make_float4(v[0], v[1], v[2], v[3]);
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (n + r < cout) dp[r] = p.accum ? dp[r] + v[r] : v[r];
            }
        }
    }
}

template <int TN, int TM, int WN, int WM>
static int launch_pw1f(const ConvParams& p, hipStream_t st) {
    const int ntn = (p.cout + TN - 1) / TN;
    const long long blocks = (long long)ntn * ((p.M + TM - 1) / TM);
    if (blocks >= (1LL << 31)) {
        set_error("conv_pw1f: grid too large");
        return YXH_EINVAL;
    }
    hipLaunchKernelGGL((conv_pw1f<TN, TM, WN, WM>), dim3((unsigned)blocks), dim3(256), 0, st, p, ntn);
    YXH_CHECK_LAUNCH("conv_pw1f launch");
    return YXH_OK;
}

int conv_pw1f_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st) {
    bool ok = dtype == YXH_F32 && p.taps == 1 && p.stride == 1 && p.pad == 0 && p.act < YXH_ACT_DECODE &&
              p.cin % 4 == 0 && (p.nsrc == 1 || p.src0_ch % 4 == 0) && p.dst_cs % 4 == 0 &&
              (p.dst_dense || p.dst_bs % 4 == 0) && ((uintptr_t)p.dst % 16) == 0 && ((uintptr_t)p.w % 16) == 0;
    for (int s = 0; s < p.nsrc; ++s)
        ok &= (s == 0 || !p.sup[s]) && p.scs[s] % 4 == 0 && p.sbs[s] % 4 == 0 && ((uintptr_t)p.sptr[s] % 16) == 0 &&
              (p.sup[s] ? p.sw[s] * 2 == p.out_w : p.sw[s] == p.out_w);
    if (!ok) {
        set_error("conv_pw1f: fp32 1x1 s1 conv over 16-byte aligned sources (the first may be x2 upsampled)");
        return YXH_EUNSUPPORTED;
    }
    switch (id) {
        case 1: return launch_pw1f<64, 128, 2, 2>(p, st);
        case 2: return launch_pw1f<128, 128, 2, 2>(p, st);
        case 3: return launch_pw1f<64, 64, 2, 2>(p, st);
        case 4: return launch_pw1f<32, 128, 1, 4>(p, st);
        default: set_error("conv_pw1f tile id %d", id); return YXH_EINVAL;
    }
}

}  // namespace yxh

namespace yxh {

// Data gradient of a 3x3 stride-2 pad-1 conv (darknet.py:148-156 stage downsampling, yolo_pafpn.py
// bu_conv1/2) in fp32 without the zero-dilated source: the dilated form runs all nine taps over an
// input three quarters zeros.  Output pixel (2i + py, 2j + px) only meets taps ty = 1 (py = 0) or
// ty in {0, 2} (py = 1) -- likewise tx -- at dy pixel (i + (py + ty - 1) / 2, j + (px + tx - 1) / 2),
// so each of the four parity classes is a GEMM over its 1, 2, 2 or 4 taps: D[c][pixel] = sum over
// (tap, n) of Wd[c][tap][n] dy[src pixel][n] with the flipped yxh_pack_dgrad_weight layout
// Wd[c][ty][tx][n].  Same k-minor MFMA operands, LDS staging and epilogue as conv_pw1f;
// blockIdx.y = parity class.
template <int TN, int TM, int WN, int WM>
__global__ __launch_bounds__(256) void dgrad_s2f(ConvParams p, int ntn, int oh, int ow) {
    static_assert(WN * WM == 4, "4 waves");
    constexpr int KC = 32, KP = KC + 4;
    constexpr int WTN = TN / WN, WTM = TM / WM, FR = WTN / 16, FC = WTM / 16;
    constexpr int ACH = TN * KC / 4, BCH = TM * KC / 4, AL = (ACH + 255) / 256, BL = (BCH + 255) / 256;
    constexpr int ASZ = TN * KP, BSZ = TM * KP;
    __shared__ __attribute__((aligned(16))) float lds[2][ASZ + BSZ];
    const int py = blockIdx.y >> 1, px = blockIdx.y & 1;
    const int H = p.out_h, W = p.out_w;
    const int ch = (H - py + 1) >> 1, cw = (W - px + 1) >> 1;  // class size
    const int nb = p.M / (H * W);
    const int Mc = nb * ch * cw;
    const int n0 = (blockIdx.x % ntn) * TN, m0 = (blockIdx.x / ntn) * TM;
    if (m0 >= Mc) return;  // block-uniform (the grid covers the largest class)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wn = wave % WN, wm = wave / WN;
    const int K = p.cin, cout = p.cout;  // K = dy channels (the forward's cout, padded)
    const int nkc = (K + KC - 1) / KC;
    const int nty = py ? 2 : 1, ntx = px ? 2 : 1, ntap = nty * ntx;
    const float* Wd = (const float*)p.w;
    const float* dy = (const float*)p.sptr[0];

    int rb_[BL], ri_[BL], rj_[BL];  // class pixel of each B row this thread loads
#pragma unroll
    for (int i = 0; i < BL; ++i) {
        const int q = tid + 256 * i;
        const int m = min(m0 + q / (KC / 4), Mc - 1);
        const int b = m / (ch * cw), r = m - b * (ch * cw);
        rb_[i] = b;
        ri_[i] = r / cw;
        rj_[i] = r - ri_[i] * cw;
    }
    float4 ra[AL], rb[BL];
    auto gload = [&](int st) {
        const int t = st / nkc, k0 = (st - t * nkc) * KC;
        const int a = t / ntx, c = t - a * ntx;
        const int ty = py ? 2 * a : 1, tx = px ? 2 * c : 1;
        const int dyo = (py + ty - 1) >> 1, dxo = (px + tx - 1) >> 1;
        const int tap = ty * 3 + tx;
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            const int r = q / (KC / 4), k = k0 + (q % (KC / 4)) * 4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < ACH && n0 + r < cout && k < K) v = *(const float4*)(Wd + ((long long)(n0 + r) * 9 + tap) * K + k);
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            const int k = k0 + (q % (KC / 4)) * 4;
            const int sy = ri_[i] + dyo, sx = rj_[i] + dxo;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < BCH && k < K && sy < oh && sx < ow)
                v = *(const float4*)(dy + (long long)rb_[i] * p.sbs[0] + (long long)(sy * ow + sx) * p.scs[0] + k);
            rb[i] = v;
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            if (q < ACH) *(float4*)(lds[buf] + (q / (KC / 4)) * KP + (q % (KC / 4)) * 4) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            if (q < BCH) *(float4*)(lds[buf] + ASZ + (q / (KC / 4)) * KP + (q % (KC / 4)) * 4) = rb[i];
        }
    };

    f32x4 acc[FR][FC];
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fk = lane >> 4;
    const int nst = ntap * nkc;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        const bool more = st + 1 < nst;
        if (more) gload(st + 1);
        const float* A = lds[buf] + (wn * WTN + fr) * KP + fk;
        const float* B = lds[buf] + ASZ + (wm * WTM + fr) * KP + fk;
#pragma unroll
        for (int kk = 0; kk < KC / 4; ++kk) {
            float a[FR], b[FC];
#pragma unroll
            for (int i = 0; i < FR; ++i) a[i] = A[i * 16 * KP + 4 * kk];
#pragma unroll
            for (int j = 0; j < FC; ++j) b[j] = B[j * 16 * KP + 4 * kk];
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (more) lstore(buf ^ 1);
        __syncthreads();
    }

    float* dst = (float*)p.dst;
#pragma unroll
    for (int j = 0; j < FC; ++j) {
        const int m = m0 + wm * WTM + 16 * j + fr;
        if (m >= Mc) continue;
        const int b = m / (ch * cw), r = m - b * (ch * cw);
        const int ci = r / cw, cj = r - ci * cw;
        const long long off = (long long)b * p.dst_bs + (long long)((2 * ci + py) * W + 2 * cj + px) * p.dst_cs;
#pragma unroll
        for (int i = 0; i < FR; ++i) {
            const int n = n0 + wn * WTN + 16 * i + 4 * fk;
            if (n >= cout) continue;
            float v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = acc[i][j][q] + (p.bias && n + q < cout ? p.bias[n + q] : 0.0f);
            float* dp = dst + off + n;
            if (n + 3 < cout) {
                if (p.accum) {
                    const float4 o = *(const float4*)dp;
                    v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
                }
                *(float4*)dp = make_float4(v[0], v[1], v[2], v[3]);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (n + q < cout) dp[q] = p.accum ? dp[q] + v[q] : v[q];
            }
        }
    }
}

template <int TN, int TM, int WN, int WM>
static int launch_dgrad_s2f(const ConvParams& p, hipStream_t st) {
    const int oh = (p.out_h + 1) / 2, ow = (p.out_w + 1) / 2;  // the dilated source's stored size
    const int ntn = (p.cout + TN - 1) / TN;
    const long long mc = (long long)(p.M / (p.out_h * p.out_w)) * oh * ow;  // the largest class
    const long long blocks = (long long)ntn * ((mc + TM - 1) / TM);
    if (blocks >= (1LL << 31)) {
        set_error("dgrad_s2f: grid too large");
        return YXH_EINVAL;
    }
    hipLaunchKernelGGL((dgrad_s2f<TN, TM, WN, WM>), dim3((unsigned)blocks, 4), dim3(256), 0, st, p, ntn, oh, ow);
    YXH_CHECK_LAUNCH("dgrad_s2f launch");
    return YXH_OK;
}

// The same parity classes for the 16-bit training step (--fp16 / bf16: dy and the flipped weights in
// T, the input gradient fp32, YXH_CONV_ACCUMULATE as above) on v_mfma_f32_16x16x32.  Both operands
// are already k-contiguous rows (Wd[c][tap][n], dy pixels [n]) = the MFMA operand form: a lane's 8 k
// of one row are one 16-byte global load, one ds_write_b128 and one ds_read_b128 (rows of 5 16-byte
// slots in LDS: the 8 lanes of a read phase hit distinct banks).  The zero-dilated form this replaces
// ran 9 taps over every output pixel: 4x the MFMA work and the dominant main-stream conv time of the
// configs[4] step (darknet.py:148-156 stage convs, yolo_pafpn.py bu_conv1/2).
template <typename T, int TN, int TM, int WN, int WM>
__global__ __launch_bounds__(256) void dgrad_s2h(ConvParams p, int ntn, int oh, int ow) {
    static_assert(WN * WM == 4, "4 waves");
    constexpr int KC = 32, RP = KC * 2 + 16;  // K stage (elements), LDS row pitch (bytes)
    constexpr int WTN = TN / WN, WTM = TM / WM, FR = WTN / 16, FC = WTM / 16;
    constexpr int ACH = TN * 4, BCH = TM * 4, AL = (ACH + 255) / 256, BL = (BCH + 255) / 256;
    constexpr int ASZ = TN * RP, BSZ = TM * RP;
    __shared__ __attribute__((aligned(16))) char lds[2][ASZ + BSZ];
    const int py = blockIdx.y >> 1, px = blockIdx.y & 1;
    const int H = p.out_h, W = p.out_w;
    const int ch = (H - py + 1) >> 1, cw = (W - px + 1) >> 1;  // class size
    const int nb = p.M / (H * W);
    const int Mc = nb * ch * cw;
    const int n0 = (blockIdx.x % ntn) * TN, m0 = (blockIdx.x / ntn) * TM;
    if (m0 >= Mc) return;  // block-uniform (the grid covers the largest class)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wn = wave % WN, wm = wave / WN;
    const int K = p.cin, cout = p.cout;  // K = dy channels (the forward's cout, padded)
    const int nkc = (K + KC - 1) / KC;
    const int ntx = px ? 2 : 1, ntap = (py ? 2 : 1) * ntx;
    const T* Wd = (const T*)p.w;
    const T* dy = (const T*)p.sptr[0];

    int rb_[BL], ri_[BL], rj_[BL];  // class pixel of each B row this thread loads
#pragma unroll
    for (int i = 0; i < BL; ++i) {
        const int q = tid + 256 * i;
        const int m = min(m0 + q / 4, Mc - 1);
        const int b = m / (ch * cw), r = m - b * (ch * cw);
        rb_[i] = b;
        ri_[i] = r / cw;
        rj_[i] = r - ri_[i] * cw;
    }
    uint4 ra[AL], rb[BL];
    auto gload = [&](int st) {
        const int t = st / nkc, k0 = (st - t * nkc) * KC;
        const int a = t / ntx, c = t - a * ntx;
        const int ty = py ? 2 * a : 1, tx = px ? 2 * c : 1;
        const int dyo = (py + ty - 1) >> 1, dxo = (px + tx - 1) >> 1;
        const int tap = ty * 3 + tx;
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            const int r = q >> 2, k = k0 + (q & 3) * 8;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (q < ACH && n0 + r < cout && k < K) v = *(const uint4*)(Wd + ((long long)(n0 + r) * 9 + tap) * K + k);
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            const int k = k0 + (q & 3) * 8;
            const int sy = ri_[i] + dyo, sx = rj_[i] + dxo;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (q < BCH && k < K && sy < oh && sx < ow)
                v = *(const uint4*)(dy + (long long)rb_[i] * p.sbs[0] + (long long)(sy * ow + sx) * p.scs[0] + k);
            rb[i] = v;
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            if (q < ACH) *(uint4*)(lds[buf] + (q >> 2) * RP + (q & 3) * 16) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            if (q < BCH) *(uint4*)(lds[buf] + ASZ + (q >> 2) * RP + (q & 3) * 16) = rb[i];
        }
    };

    f32x4 acc[FR][FC];
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fk = lane >> 4;
    const int nst = ntap * nkc;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        const bool more = st + 1 < nst;
        if (more) gload(st + 1);
        const char* A = lds[buf] + (wn * WTN + fr) * RP + fk * 16;
        const char* B = lds[buf] + ASZ + (wm * WTM + fr) * RP + fk * 16;
        uint4 a[FR], b[FC];
#pragma unroll
        for (int i = 0; i < FR; ++i) a[i] = *(const uint4*)(A + i * 16 * RP);
#pragma unroll
        for (int j = 0; j < FC; ++j) b[j] = *(const uint4*)(B + j * 16 * RP);
#pragma unroll
        for (int i = 0; i < FR; ++i)
#pragma unroll
            for (int j = 0; j < FC; ++j) Mma<T>::run(acc[i][j], a[i], b[j]);
        if (more) lstore(buf ^ 1);
        __syncthreads();
    }

    float* dst = (float*)p.dst;
#pragma unroll
    for (int j = 0; j < FC; ++j) {
        const int m = m0 + wm * WTM + 16 * j + fr;
        if (m >= Mc) continue;
        const int b = m / (ch * cw), r = m - b * (ch * cw);
        const int ci = r / cw, cj = r - ci * cw;
        const long long off = (long long)b * p.dst_bs + (long long)((2 * ci + py) * W + 2 * cj + px) * p.dst_cs;
#pragma unroll
        for (int i = 0; i < FR; ++i) {
            const int n = n0 + wn * WTN + 16 * i + 4 * fk;
            if (n >= cout) continue;
            float v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = acc[i][j][q] + (p.bias && n + q < cout ? p.bias[n + q] : 0.0f);
            float* dp = dst + off + n;
            if (n + 3 < cout) {
                if (p.accum) {
                    const float4 o = *(const float4*)dp;
                    v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
                }
                *(float4*)dp = make_float4(v[0], v[1], v[2], v[3]);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (n + q < cout) dp[q] = p.accum ? dp[q] + v[q] : v[q];
            }
        }
    }
}

template <typename T, int TN, int TM, int WN, int WM>
static int launch_dgrad_s2h(const ConvParams& p, hipStream_t st) {
    const int oh = (p.out_h + 1) / 2, ow = (p.out_w + 1) / 2;  // the dilated source's stored size
    const int ntn = (p.cout + TN - 1) / TN;
    const long long mc = (long long)(p.M / (p.out_h * p.out_w)) * oh * ow;  // the largest class
    const long long blocks = (long long)ntn * ((mc + TM - 1) / TM);
    if (blocks >= (1LL << 31)) {
        set_error("dgrad_s2h: grid too large");
        return YXH_EINVAL;
    }
    hipLaunchKernelGGL((dgrad_s2h<T, TN, TM, WN, WM>), dim3((unsigned)blocks, 4), dim3(256), 0, st, p, ntn, oh, ow);
    YXH_CHECK_LAUNCH("dgrad_s2h launch");
    return YXH_OK;
}

template <typename T>
static int dgrad_s2h_tile(int id, const ConvParams& p, hipStream_t st) {
    switch (id) {
        case 3: return launch_dgrad_s2h<T, 128, 128, 2, 2>(p, st);
        case 4: return launch_dgrad_s2h<T, 64, 128, 1, 4>(p, st);
        case 5: return launch_dgrad_s2h<T, 128, 64, 2, 2>(p, st);
        case 6: return launch_dgrad_s2h<T, 64, 64, 2, 2>(p, st);
        default: set_error("dgrad_s2h tile id %d", id); return YXH_EINVAL;
    }
}

int dgrad_s2f_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st) {
    const bool geo = p.nsrc == 1 && p.sup[0] == 2 && p.taps == 9 && p.kw == 3 && p.stride == 1 && p.pad == 1 &&
                     p.act == YXH_ACT_NONE && p.dst_cs % 4 == 0 && p.dst_bs % 4 == 0 && ((uintptr_t)p.dst % 16) == 0 &&
                     ((uintptr_t)p.sptr[0] % 16) == 0 && ((uintptr_t)p.w % 16) == 0 && p.sw[0] == (p.out_w + 1) / 2;
    if (id <= 2) {
        if (!(geo && dtype == YXH_F32 && p.cin % 4 == 0 && p.scs[0] % 4 == 0 && p.sbs[0] % 4 == 0)) {
            set_error("dgrad_s2f: fp32 data gradient of a 3x3 s2 p1 conv (a zero-dilated dy source, no activation)");
            return YXH_EUNSUPPORTED;
        }
        return id == 1 ? launch_dgrad_s2f<64, 128, 2, 2>(p, st) : launch_dgrad_s2f<128, 64, 2, 2>(p, st);
    }
    if (!(geo && dtype != YXH_F32 && p.dst_f32 && p.cin % 8 == 0 && p.scs[0] % 8 == 0 && p.sbs[0] % 8 == 0)) {
        set_error("dgrad_s2h: 16-bit data gradient of a 3x3 s2 p1 conv into fp32 (a zero-dilated dy source of "
                  "16-byte pixel rows, no activation)");
        return YXH_EUNSUPPORTED;
    }
    return dtype == YXH_BF16 ? dgrad_s2h_tile<bf16>(id, p, st) : dgrad_s2h_tile<f16>(id, p, st);
}

}  // namespace yxh
