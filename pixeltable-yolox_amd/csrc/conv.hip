// Convolution family of the YOLOX hot path on gfx950 (MI355X).
//
//  conv_igemm   : NHWC implicit-GEMM Conv2d (+folded BN, act, residual, head decode)
//                 on MFMA.  D[cout x pixels] = W[cout x K] * X[K x pixels], K ordered
//                 (ky, kx, cin) so every 16-byte chunk of K is 8 contiguous channels
//                 of one input pixel (bf16/f16; 4 for fp32).
//  dwconv       : depthwise 3x3 (DWConv.dconv, nano) -- HBM-bound, VALU.
//  focus_pack   : Focus space-to-depth of the network input into 16-ch NHWC.
//  spp_maxpool  : SPP 5/9/13 max pools, separable, LDS planes of 1-4 16-B chunks per pixel.
//  fold_bn_pack : BN folding + [cout][kh][kw][cin] repack of the weights.
//
// Reference call sites: network_blocks.py:27-208 (BaseConv, DWConv, Bottleneck,
// SPPBottleneck, CspLayer, Focus), yolo_pafpn.py:83-116 (cat/upsample),
// yolo_head.py:140-251 (stems, cls/reg convs, preds, decode).
#include <stdio.h>

#include "conv_common.hpp"

namespace yxh {

// conv_ws tiles for 80 / 160 / 320 / 512 input channels (yolox_x, yolox_l) and the fp32-gradient
// forms (tiles 281-288): tile ids 261..260+kNumWsWideTiles (conv_ws_dispatch ids 61..)
constexpr int kNumWsWideTiles = 29;

// ---------------------------------------------------------------- implicit GEMM
// Block: 256 threads = 4 waves on a WR x WC grid; tile TN output channels x TM
// output pixels; KS 64-byte K slabs per pipeline stage.  LDS holds two stages; a
// stage is [slab][chunk][row] of 16-byte chunks with the row index XOR-swizzled by
// (2*chunk + slab), which makes both the ds_write_b128 of the loaders (8 lanes =
// one row's chunks) and the ds_read_b128 fragment reads (16 rows x 1 chunk per lane
// group) bank-conflict free.
template <typename T, int TN, int TM, int WR, int WC, int KS>
__global__ __launch_bounds__(256) void conv_igemm(ConvParams p) {
    constexpr int EPC = Chunk<T>::N;
    constexpr int CPR = 4 * KS;        // chunks per row per stage
    constexpr int KSTAGE = CPR * EPC;  // K elements per stage
    constexpr int RPP = 256 / CPR;     // rows per loader pass
    constexpr int NA = (TN + RPP - 1) / RPP;
    constexpr int NB = (TM + RPP - 1) / RPP;
    constexpr int WTN = TN / WR, WTM = TM / WC;
    constexpr int FR = WTN / 16, FC = WTM / 16;
    constexpr int A_BYTES = TN * CPR * 16, B_BYTES = TM * CPR * 16;
    constexpr int BUF = A_BYTES + B_BYTES;
    static_assert(WR * WC == 4 && FR >= 1 && FC >= 1 && TN % 8 == 0 && TM % 16 == 0, "tile");
    __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WC, wc = wave % WC;
    const int n0 = blockIdx.y * TN, m0 = blockIdx.x * TM;
    const int cq = tid % CPR, rq = tid / CPR;
    const int ls = cq >> 2, lc = cq & 3;  // slab / chunk of this thread's loads
    const int coff = cq * EPC;

    int bb[NB], by[NB], bx[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        int r = rq + i * RPP;
        int m = m0 + r;
        bool ok = r < TM && m < p.M;
        if (p.src_dense) {  // 1x1 s1 over dense sources: pixel m is at m * scs, no split
            bb[i] = ok ? 0 : -1;
            by[i] = m;
            bx[i] = 0;
            continue;
        }
        int b = ok ? m / p.ohw : 0;
        int rem = m - b * p.ohw;
        int oy = rem / p.out_w, ox = rem - oy * p.out_w;
        bb[i] = ok ? b : -1;
        by[i] = oy * p.stride - p.pad;
        bx[i] = ox * p.stride - p.pad;
    }

    uint4 ra[NA], rb[NB];
    // K iterations (tap t = (ky, kx), channel block cb) are loaded strictly in order:
    // the indices advance incrementally instead of two divides per stage
    int g_t = 0, g_cb = 0, g_ky = 0, g_kx = 0;
    auto gload = [&](int) {
        const int t = g_t, cb = g_cb, ky = g_ky, kx = g_kx;
        if (++g_cb == p.ncb) {
            g_cb = 0;
            ++g_t;
            if (++g_kx == p.kw) {
                g_kx = 0;
                ++g_ky;
            }
        }
        const int c = cb * KSTAGE + coff;
        const bool cok = c < p.cin;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            int r = rq + i * RPP, n = n0 + r;
            ra[i] = make_uint4(0, 0, 0, 0);
            if (r < TN && n < p.cout && cok)
                ra[i] = *(const uint4*)((const T*)p.w + ((long long)n * p.taps + t) * p.cin + c);
        }
        int s = 0, cc = c;
        if (p.nsrc == 2 && c >= p.src0_ch) {
            s = 1;
            cc = c - p.src0_ch;
        }
        const T* sp = (const T*)p.sptr[s];
        const int scs = p.scs[s], sw = p.sw[s], up = p.sup[s] ? 1 : 0;
        const int odd = p.sup[s] == 2 ? 1 : 0;  // zero-inserting dilation: odd positions read 0
        const long long sbs = p.sbs[s];
        if (p.src_dense) {
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                rb[i] = make_uint4(0, 0, 0, 0);
                if (bb[i] >= 0 && cok) rb[i] = *(const uint4*)(sp + (long long)by[i] * scs + cc);
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            int iy = by[i] + ky, ix = bx[i] + kx;
            rb[i] = make_uint4(0, 0, 0, 0);
            if (bb[i] >= 0 && cok && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w && !((iy | ix) & odd))
                rb[i] = *(const uint4*)(sp + bb[i] * sbs +
                                        ((long long)(iy >> up) * sw + (ix >> up)) * scs + cc);
        }
    };
    auto lstore = [&](int buf) {
        char* A = smem + buf * BUF;
        char* B = A + A_BYTES;
        const int sw_ = 2 * lc + ls;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            int r = rq + i * RPP;
            if (r < TN) *(uint4*)(A + ((cq)*TN + (r ^ sw_)) * 16) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            int r = rq + i * RPP;
            if (r < TM) *(uint4*)(B + ((cq)*TM + (r ^ sw_)) * 16) = rb[i];
        }
    };

    f32x4 acc[FR][FC];
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int frow = lane & 15, fq = lane >> 4;
    auto compute = [&](int buf) {
        const char* A = smem + buf * BUF;
        const char* B = A + A_BYTES;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int chunk = s * 4 + fq, sw_ = 2 * fq + s;
            uint4 af[FR], bf[FC];
#pragma unroll
            for (int i = 0; i < FR; ++i) {
                int row = wr * WTN + i * 16 + frow;
                af[i] = *(const uint4*)(A + (chunk * TN + (row ^ sw_)) * 16);
            }
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                int row = wc * WTM + j * 16 + frow;
                bf[j] = *(const uint4*)(B + (chunk * TM + (row ^ sw_)) * 16);
            }
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) Mma<T>::run(acc[i][j], af[i], bf[j]);
        }
    };

    float lbias[FR][4];
    load_lane_bias<TN, WR, WC>(p, n0, lbias);
    const int nk = p.taps * p.ncb;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int k = 0; k < nk; ++k) {
        const int cur = k & 1;
        if (k + 1 < nk) gload(k + 1);
        compute(cur);
        if (k + 1 < nk) lstore(cur ^ 1);
        __syncthreads();
    }

    conv_epilogue<T, TN, TM, WR, WC, 2 * BUF>(p, acc, smem, m0, n0, lbias);
}

// ---------------------------------------------------------------- depthwise
template <typename T>
__global__ __launch_bounds__(256) void dwconv(ConvParams p) {
    constexpr int EPC = Chunk<T>::N;
    const int nch = (p.cin + EPC - 1) / EPC;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)p.M * nch) return;
    const int ch = (int)(idx % nch);
    const int m = (int)(idx / nch);
    const int b = m / p.ohw, pix = m - b * p.ohw;
    const int oy = pix / p.out_w, ox = pix - oy * p.out_w;
    const int c0 = ch * EPC;
    float acc[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) acc[e] = 0.0f;
    const T* sp = (const T*)p.sptr[0];
    const T* w = (const T*)p.w;
    for (int t = 0; t < p.taps; ++t) {
        const int ky = t / p.kw, kx = t - ky * p.kw;
        const int iy = oy * p.stride - p.pad + ky, ix = ox * p.stride - p.pad + kx;
        if (iy < 0 || iy >= p.in_h || ix < 0 || ix >= p.in_w) continue;
        uint4 u = *(const uint4*)(sp + b * p.sbs[0] +
                                  ((long long)(iy >> p.sup[0]) * p.sw[0] + (ix >> p.sup[0])) * p.scs[0] + c0);
        T xv[EPC];
        __builtin_memcpy(xv, &u, 16);
#pragma unroll
        for (int e = 0; e < EPC; ++e)
            if (c0 + e < p.cin) acc[e] += to_f32(xv[e]) * to_f32(w[(c0 + e) * p.taps + t]);
    }
    for (int q = 0; q < EPC; q += 4) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[q + r] + (c0 + q + r < p.cout ? p.bias[c0 + q + r] : 0.0f);
        if (c0 + q < p.cout) store4<T>(p, v, c0 + q, b, pix, ox, oy);
    }
}

// ---------------------------------------------------------------- focus pack
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void focus_pack(const TI* img, int layout, int B, int H, int W, TO* dst) {
    const int h2 = H / 2, w2 = W / 2;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)B * h2 * w2) return;
    const int j = (int)(idx % w2);
    const int i = (int)((idx / w2) % h2);
    const int b = (int)(idx / ((long long)w2 * h2));
    TO out[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int y = 2 * i + (q & 1), x = 2 * j + (q >> 1);  // TL, BL, TR, BR
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float v = layout == YXH_NCHW ? to_f32(img[(((long long)b * 3 + c) * H + y) * W + x])
                                         : to_f32(img[(((long long)b * H + y) * W + x) * 3 + c]);
            out[q * 3 + c] = from_f32<TO>(v);
        }
    }
#pragma unroll
    for (int k = 12; k < 16; ++k) out[k] = from_f32<TO>(0.0f);
    uint4* d = (uint4*)(dst + idx * 16);
#pragma unroll
    for (int k = 0; k < (int)(16 * sizeof(TO) / 16); ++k) {
        uint4 u;
        __builtin_memcpy(&u, (const char*)out + 16 * k, 16);
        d[k] = u;
    }
}

// ---------------------------------------------------------------- SPP
template <typename T>
__device__ __forceinline__ uint4 vmax(uint4 a, uint4 b) {
    if constexpr (__is_same(T, bf16)) {
        // bf16 maps to order-preserving int16 keys (spp_key) in LDS: 4 packed-int16 max per chunk
        // instead of 8 converts + compares + selects
        typedef short s2 __attribute__((ext_vector_type(2)));
        uint4 r;
        r.x = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2, a.x), __builtin_bit_cast(s2, b.x)));
        r.y = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2, a.y), __builtin_bit_cast(s2, b.y)));
        r.z = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2, a.z), __builtin_bit_cast(s2, b.z)));
        r.w = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2, a.w), __builtin_bit_cast(s2, b.w)));
        return r;
    }
    constexpr int EPC = Chunk<T>::N;
    T x[EPC], y[EPC];
    __builtin_memcpy(x, &a, 16);
    __builtin_memcpy(y, &b, 16);
#pragma unroll
    for (int e = 0; e < EPC; ++e) x[e] = to_f32(y[e]) > to_f32(x[e]) ? y[e] : x[e];
    uint4 r;
    __builtin_memcpy(&r, x, 16);
    return r;
}

// bf16 <-> order-preserving int16 key, both halves of a dword: a negative value (sign set) has its
// 15 magnitude bits flipped, so signed int16 order = float order (-0 sorts just below +0; NaN
// payloads sort outside every finite value); the map is its own inverse
template <typename T>
__device__ __forceinline__ uint4 spp_key(uint4 v) {
    if constexpr (__is_same(T, bf16)) {
        auto k = [](uint32_t d) { return d ^ (((d >> 15) & 0x00010001u) * 0x7fffu); };
        return make_uint4(k(v.x), k(v.y), k(v.z), k(v.w));
    }
    return v;
}

// One block per (CPB consecutive 16-byte channel chunks, image): horizontal 5/9/13 maxima
// into LDS, then vertical.  max_pool2d pads with -inf, i.e. out-of-range taps are skipped.
// Lanes run over (pixel, chunk) with the chunk fastest, so each pixel's CPB chunks are one
// contiguous 16*CPB-byte segment of the NHWC row (one 16-byte chunk per block read and
// wrote 400 scattered 16-byte pieces per plane: 36 us for a 6.5 MB tensor).
template <typename T, int CPB>
__global__ __launch_bounds__(256) void spp_maxpool(T* buf, int H, int W, int C, int cs, long long bs) {
    constexpr int EPC = Chunk<T>::N;
    extern __shared__ __attribute__((aligned(16))) uint4 sm[];
    const int HW = H * W, N = HW * CPB;
    uint4* P = sm;  // [pixel][chunk]
    uint4* H5 = sm + N;
    uint4* H9 = sm + 2 * N;
    uint4* H13 = sm + 3 * N;
    const int c0 = blockIdx.x * EPC * CPB;
    T* base = buf + blockIdx.y * bs;
    for (int q = threadIdx.x; q < N; q += blockDim.x) {
        const int px = q / CPB, ch = q - px * CPB;
        P[q] = spp_key<T>(*(const uint4*)(base + (long long)px * cs + c0 + ch * EPC));
    }
    __syncthreads();
    for (int q = threadIdx.x; q < N; q += blockDim.x) {
        const int px = q / CPB;
        const int y = px / W, x = px - y * W;
        uint4 m5 = P[q];
        for (int d = 1; d <= 2; ++d) {
            if (x - d >= 0) m5 = vmax<T>(m5, P[q - d * CPB]);
            if (x + d < W) m5 = vmax<T>(m5, P[q + d * CPB]);
        }
        uint4 m9 = m5;
        for (int d = 3; d <= 4; ++d) {
            if (x - d >= 0) m9 = vmax<T>(m9, P[q - d * CPB]);
            if (x + d < W) m9 = vmax<T>(m9, P[q + d * CPB]);
        }
        uint4 m13 = m9;
        for (int d = 5; d <= 6; ++d) {
            if (x - d >= 0) m13 = vmax<T>(m13, P[q - d * CPB]);
            if (x + d < W) m13 = vmax<T>(m13, P[q + d * CPB]);
        }
        (void)y;
        H5[q] = m5;
        H9[q] = m9;
        H13[q] = m13;
    }
    __syncthreads();
    const int row = W * CPB;
    for (int q = threadIdx.x; q < N; q += blockDim.x) {
        const int px = q / CPB, ch = q - px * CPB;
        const int y = px / W;
        uint4 o5 = H5[q], o9 = H9[q], o13 = H13[q];
        for (int d = 1; d <= 6; ++d) {
            const bool up = y - d >= 0, dn = y + d < H;
            if (d <= 2) {
                if (up) o5 = vmax<T>(o5, H5[q - d * row]);
                if (dn) o5 = vmax<T>(o5, H5[q + d * row]);
            }
            if (d <= 4) {
                if (up) o9 = vmax<T>(o9, H9[q - d * row]);
                if (dn) o9 = vmax<T>(o9, H9[q + d * row]);
            }
            if (up) o13 = vmax<T>(o13, H13[q - d * row]);
            if (dn) o13 = vmax<T>(o13, H13[q + d * row]);
        }
        T* pp = base + (long long)px * cs + c0 + ch * EPC;
        *(uint4*)(pp + C) = spp_key<T>(o5);
        *(uint4*)(pp + 2 * C) = spp_key<T>(o9);
        *(uint4*)(pp + 3 * C) = spp_key<T>(o13);
    }
}

// ---------------------------------------------------------------- BN fold + pack
template <typename T>
__global__ __launch_bounds__(256) void fold_bn_pack(const float* w, const float* cb, const float* g,
                                                    const float* beta, const float* mean, const float* var,
                                                    float eps, int cout, int cin_g, int kh, int kw,
                                                    int cin_pad, T* wo, float* bo) {
    const int taps = kh * kw;
    const long long total = (long long)cout * taps * cin_pad;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int c = (int)(idx % cin_pad);
    const int t = (int)((idx / cin_pad) % taps);
    const int n = (int)(idx / ((long long)cin_pad * taps));
    const float scale = g ? g[n] / sqrtf(var[n] + eps) : 1.0f;
    const int ky = t / kw, kx = t - ky * kw;
    float v = c < cin_g ? w[(((long long)n * cin_g + c) * kh + ky) * kw + kx] * scale : 0.0f;
    wo[idx] = from_f32<T>(v);
    if (t == 0 && c == 0) {
        float b = g ? beta[n] - mean[n] * scale : 0.0f;
        if (cb) b += cb[n] * scale;
        bo[n] = b;
    }
}

// ---------------------------------------------------------------- fragment-major weights
// [cout][taps][cin] -> 1 KiB blocks (nf, tap, kb): lane l = 16 q + r holds channel 16 nf + r,
// inputs 32 kb + 8 q .. + 8 (yxh_pack_frag); one thread per 16-byte piece
__global__ __launch_bounds__(256) void pack_frag(const uint4* w, int cout, int taps, int cin, uint4* out) {
    const int kbs = cin >> 5;
    const long long total = (long long)(cout >> 4) * taps * kbs * 64;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int l = (int)(idx & 63);
    const long long blk = idx >> 6;
    const int kb = (int)(blk % kbs), tap = (int)((blk / kbs) % taps), nf = (int)(blk / ((long long)kbs * taps));
    const int n = nf * 16 + (l & 15), k = kb * 32 + (l >> 4) * 8;
    out[idx] = w[(((long long)n * taps + tap) * cin + k) >> 3];
}

// ================================================================ host side
namespace {

int elem_size(int dt) { return dt == YXH_F32 ? 4 : dt == YXH_U8 ? 1 : 2; }

bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15u) == 0; }

template <typename T, int TN, int TM, int WR, int WC>
int launch_igemm(const ConvParams& p, int ks, hipStream_t st) {
    dim3 grid((p.M + TM - 1) / TM, (p.cout + TN - 1) / TN);
    if (ks == 2)
        hipLaunchKernelGGL((conv_igemm<T, TN, TM, WR, WC, 2>), grid, dim3(256), 0, st, p);
    else
        hipLaunchKernelGGL((conv_igemm<T, TN, TM, WR, WC, 1>), grid, dim3(256), 0, st, p);
    YXH_CHECK_LAUNCH("conv_igemm launch");
    return YXH_OK;
}

// Tile configurations (id -> TN x TM, wave grid).  yxh_conv_desc.tile = id * 2 + (KS - 1)
// selects one explicitly (the planner autotunes it per layer on the device); 0 picks
// by a block-count heuristic.
struct TileCfg { int tn, tm; };
constexpr TileCfg kTiles[] = {{0, 0},     {16, 256}, {32, 256}, {32, 128}, {64, 256},
                              {64, 128},  {64, 64},  {80, 128}, {128, 128}, {128, 64}};
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

template <typename T>
int launch_tile(int id, const ConvParams& p, int ks, hipStream_t st) {
    switch (id) {
        case 1: return launch_igemm<T, 16, 256, 1, 4>(p, ks, st);
        case 2: return launch_igemm<T, 32, 256, 1, 4>(p, ks, st);
        case 3: return launch_igemm<T, 32, 128, 1, 4>(p, ks, st);
        case 4: return launch_igemm<T, 64, 256, 1, 4>(p, ks, st);
        case 5: return launch_igemm<T, 64, 128, 1, 4>(p, ks, st);
        case 6: return launch_igemm<T, 64, 64, 2, 2>(p, ks, st);
        case 7: return launch_igemm<T, 80, 128, 1, 4>(p, ks, st);
        case 8: return launch_igemm<T, 128, 128, 2, 2>(p, ks, st);
        case 9: return launch_igemm<T, 128, 64, 2, 2>(p, ks, st);
        default: set_error("tile id %d", id); return YXH_EINVAL;
    }
}

int heuristic_tile(const ConvParams& p) {
    auto blocks = [&](int tn, int tm) { return (long long)((p.M + tm - 1) / tm) * ((p.cout + tn - 1) / tn); };
    const long long target = 512;
    if (p.cout <= 16) return 1;
    if (p.cout <= 32) return blocks(32, 256) >= target ? 2 : 3;
    if (p.cout <= 64) return blocks(64, 256) >= target ? 4 : blocks(64, 128) >= target ? 5 : 6;
    if (p.cout <= 80) return 7;
    return blocks(128, 128) >= target ? 8 : blocks(128, 64) >= target ? 9 : 6;
}

}  // namespace

int conv2d(const yxh_conv_desc* d, hipStream_t st) {
    YXH_CHECK_ARG(d, "null descriptor");
    const int dt = d->dtype;
    YXH_CHECK_ARG(dt == YXH_F32 || dt == YXH_BF16 || dt == YXH_F16, "conv dtype %d", dt);
    const int es = elem_size(dt), epc = 16 / es;
    YXH_CHECK_ARG(d->batch > 0 && d->out_h > 0 && d->out_w > 0 && d->in_h > 0 && d->in_w > 0, "empty conv");
    YXH_CHECK_ARG(d->cin > 0 && d->cout > 0 && d->kh > 0 && d->kw > 0 && d->stride > 0 && d->pad >= 0,
                  "bad conv geometry");
    YXH_CHECK_ARG(d->nsrc == 1 || d->nsrc == 2, "nsrc %d", d->nsrc);
    YXH_CHECK_ARG(d->weight && d->bias && (d->dst || d->post_weight), "null weight/bias/dst");
    YXH_CHECK_ARG(d->dst_dtype == dt || d->dst_dtype == YXH_F32, "dst dtype %d", d->dst_dtype);
    YXH_CHECK_ARG(d->act >= YXH_ACT_NONE && d->act <= YXH_ACT_DECODE_RAW, "act %d", d->act);
    YXH_CHECK_ARG(d->act < YXH_ACT_DECODE || d->dst_dtype == YXH_F32, "decode needs an f32 dst");
    const bool dw = d->groups != 1;
    YXH_CHECK_ARG(!dw || (d->groups == d->cin && d->cout == d->cin && d->nsrc == 1), "groups %d", d->groups);
    int chs = 0;
    bool dilated = false;
    for (int s = 0; s < d->nsrc; ++s) {
        const yxh_src& q = d->src[s];
        YXH_CHECK_ARG(q.ptr && aligned16(q.ptr), "src%d null or not 16-byte aligned", s);
        YXH_CHECK_ARG(q.channels > 0 && q.channels % epc == 0, "src%d channels %d not a multiple of %d", s,
                      q.channels, epc);
        YXH_CHECK_ARG(q.cstride % epc == 0 && q.bstride % epc == 0, "src%d strides not 16-byte multiples", s);
        YXH_CHECK_ARG(q.upsample >= 0 && q.upsample <= 2, "upsample %d", q.upsample);
        YXH_CHECK_ARG(q.upsample != 2 || !dw, "dilated source on a depthwise conv");
        const int ush = q.upsample ? 1 : 0;
        // a zero-dilated source (a stride-2 conv's data gradient) of an odd-sized input: the
        // dilated map's last row / column is odd, i.e. zero, so it may be cut off (logical size
        // 2h - 1): reads past in_h / in_w are the conv's zero padding either way
        const bool odd_ok = q.upsample == 2 && ((q.h << 1) - d->in_h) >= 0 && ((q.h << 1) - d->in_h) <= 1 &&
                            ((q.w << 1) - d->in_w) >= 0 && ((q.w << 1) - d->in_w) <= 1;
        YXH_CHECK_ARG(odd_ok || ((q.h << ush) == d->in_h && (q.w << ush) == d->in_w),
                      "src%d spatial %dx%d (up %d) vs input %dx%d", s, q.h, q.w, q.upsample, d->in_h, d->in_w);
        dilated |= q.upsample == 2;
        chs += q.channels;
    }
    const bool grp2 = (d->flags & YXH_CONV_GROUPS2) != 0;
    YXH_CHECK_ARG(chs == (grp2 ? 2 * d->cin : d->cin), "source channels %d != cin %d%s", chs, d->cin,
                  grp2 ? " x 2 groups" : "");
    YXH_CHECK_ARG(!grp2 || (d->nsrc == 1 && d->groups == 1 && d->cout % 2 == 0 && !d->pre_weight && !d->residual &&
                            dt != YXH_F32),
                  "YXH_CONV_GROUPS2: 16-bit, one source, even cout, no residual / fused conv1");
    YXH_CHECK_ARG((d->in_h + 2 * d->pad - d->kh) / d->stride + 1 == d->out_h &&
                      (d->in_w + 2 * d->pad - d->kw) / d->stride + 1 == d->out_w,
                  "output size mismatch");
    YXH_CHECK_ARG(aligned16(d->weight), "weight not 16-byte aligned");

    ConvParams p{};
    p.in_h = d->in_h; p.in_w = d->in_w; p.out_h = d->out_h; p.out_w = d->out_w;
    p.cin = d->cin; p.cout = d->cout; p.kw = d->kw; p.stride = d->stride; p.pad = d->pad;
    p.ohw = d->out_h * d->out_w;
    const long long M = (long long)d->batch * p.ohw;
    YXH_CHECK_ARG(M < (1LL << 31), "too many output pixels");
    p.M = (int)M;
    p.taps = d->kh * d->kw;
    p.nsrc = d->nsrc;
    p.src0_ch = d->src[0].channels;
    for (int s = 0; s < d->nsrc; ++s) {
        p.sptr[s] = d->src[s].ptr;
        p.scs[s] = d->src[s].cstride;
        p.sbs[s] = d->src[s].bstride;
        p.sw[s] = d->src[s].w;
        p.sup[s] = d->src[s].upsample;
    }
    p.w = d->weight;
    p.bias = d->bias;
    p.res = d->residual;
    p.res_cs = d->res_cstride;
    p.res_bs = d->res_bstride;
    p.dst = d->dst;
    p.dst_cs = d->dst_cstride;
    p.dst_bs = d->dst_bstride;
    p.dst_f32 = d->dst_dtype == YXH_F32 && dt != YXH_F32 ? 1 : (dt == YXH_F32 ? 1 : 0);
    YXH_CHECK_ARG(!(d->flags & YXH_CONV_ACCUMULATE) || d->dst_dtype == YXH_F32, "accumulate needs an f32 dst");
    YXH_CHECK_ARG(!(d->flags & YXH_CONV_POST_STORE) || d->post_weight, "YXH_CONV_POST_STORE needs a post conv");
    p.accum = (d->flags & YXH_CONV_ACCUMULATE) ? 1 : 0;
    p.act = d->act;
    p.dstride = d->decode_stride;
    p.dcoff = d->decode_coff;
    const int des = elem_size(d->dst_dtype);
    const int vbytes = des == 4 ? 16 : 8;
    p.vec_store = (((uintptr_t)d->dst % vbytes) == 0 && (d->dst_cstride * des) % vbytes == 0 &&
                   (d->dst_bstride * des) % vbytes == 0)
                      ? 1
                      : 0;
    p.vec_res = d->residual && ((uintptr_t)d->residual % 8) == 0 && (d->res_cstride * es) % 8 == 0 &&
                (d->res_bstride * es) % 8 == 0;
    p.src_dense = p.taps == 1 && p.stride == 1 && p.pad == 0;
    for (int s = 0; s < d->nsrc; ++s)
        p.src_dense &= !p.sup[s] && p.sw[s] == p.out_w && p.sbs[s] == (long long)p.ohw * p.scs[s];
    p.dst_dense = d->dst_bstride == (long long)p.ohw * d->dst_cstride;
    p.res_dense = d->residual && d->res_bstride == (long long)p.ohw * d->res_cstride;
    p.pw1 = d->pre_weight;
    p.pb1 = d->pre_bias;
    YXH_CHECK_ARG(!d->weight_frag || (dt != YXH_F32 && aligned16(d->weight_frag) && d->cout % 16 == 0 &&
                                      d->cin % 32 == 0 && d->groups == 1),
                  "weight_frag: 16-bit, cout %% 16 == 0, cin %% 32 == 0, groups 1");
    p.wf = d->weight_frag;
    YXH_CHECK_ARG(d->grid_cap >= 0, "grid_cap %d", d->grid_cap);
    const int cus = device_cus();
    p.cus = d->grid_cap > 0 && d->grid_cap < cus ? d->grid_cap : cus;
    p.grp2 = grp2 ? 1 : 0;
    if (d->post_weight) {
        // a 1x1 post conv (or the head form: two groups, each with its own preds) runs on the
        // conv_ws post tiles; dispatched here, after the grid / weight-copy fields are set
        const bool head = grp2;
        YXH_CHECK_ARG(dt != YXH_F32 && d->post_bias && d->post_dst && aligned16(d->post_weight) && d->post_cout > 0 &&
                          d->kh == 3 && d->groups == 1 && !d->pre_weight && d->post_src.channels >= 0 &&
                          d->post_src.channels % 32 == 0,
                      "post conv: 16-bit 3x3 conv (no pre_weight / groups), post_src channels %% 32");
        if (head) {
            YXH_CHECK_ARG(d->post_weight2 && d->post_bias2 && aligned16(d->post_weight2) && d->post_cout2 == 5 &&
                              d->post_cout >= 65 && d->post_cout <= 80 && d->post_src.channels == 0 &&
                              ((uintptr_t)d->post_dst % 4) == 0 && d->post_dst_cstride == 5 + d->post_cout,
                          "head post form: reg|obj (5) and 65-80 class preds, rows of 5 + classes fp32");
        } else {
            YXH_CHECK_ARG(d->post_cout % 16 == 0 && !d->post_weight2 &&
                              (d->post_src.channels == 0 ||
                               (d->post_src.ptr && aligned16(d->post_src.ptr) && d->post_src.cstride % 8 == 0 &&
                                d->post_src.bstride % 8 == 0 && !d->post_src.upsample &&
                                d->post_src.h == d->out_h && d->post_src.w == d->out_w)) &&
                              ((uintptr_t)d->post_dst % 8) == 0 && d->post_dst_cstride % 4 == 0 &&
                              d->post_dst_bstride % 4 == 0,
                          "post conv: post_cout %% 16, post_src at the output size (16-byte rows), 8-byte aligned "
                          "post_dst rows");
        }
        p.pgw = d->post_weight;
        p.pgb = d->post_bias;
        p.pgw2 = d->post_weight2;
        p.pgb2 = d->post_bias2;
        p.pg_cout2 = d->post_cout2;
        p.pg_stride = d->post_stride;
        p.pgd = d->post_dst;
        p.pgd_cs = d->post_dst_cstride;
        p.pgd_bs = d->post_dst_bstride;
        p.pgs = d->post_src.channels ? d->post_src.ptr : nullptr;
        p.pgs_cs = d->post_src.cstride;
        p.pgs_bs = d->post_src.bstride;
        p.pgs_ch = d->post_src.channels;
        p.pg_cout = d->post_cout;
        p.pg_store = (d->flags & YXH_CONV_POST_STORE) ? 1 : 0;
        YXH_CHECK_ARG(!p.pg_store || (!head && d->dst && p.vec_store && d->dst_dtype == dt),
                      "YXH_CONV_POST_STORE: a 1x1 post conv (not the head form) and a 16-bit dst of 8-byte rows");
        if (d->tile == 0) {  // default post tile per shape
            const bool chain = d->post_src.channels == 0 && d->stride == 1;
            return conv_ws_dispatch(
                dt, head ? 51 : d->stride == 2 ? 45 : chain ? (d->cin == 64 ? 54 : 55) : d->cin == 32 ? 41 : 43, p, st);
        }
        if (!((d->tile >> 1) > 220 && (d->tile >> 1) <= 220 + kNumWsPostTiles)) {
            set_error("a post conv runs on the conv_ws post tiles (ids 221-%d) only", 220 + kNumWsPostTiles);
            return YXH_EUNSUPPORTED;
        }
        return conv_ws_dispatch(dt, (d->tile >> 1) - 220 + 40, p, st);
    }
    if (grp2 && d->tile == 0) return conv_ws_dispatch(dt, d->cin == 256 ? 176 - 160 : 185 - 160, p, st);
    if (grp2 && !((d->tile >> 1) > 160 && (d->tile >> 1) <= 190)) {
        set_error("YXH_CONV_GROUPS2 runs on the plain conv_ws tiles (ids 161-190) only");
        return YXH_EUNSUPPORTED;
    }
    YXH_CHECK_ARG(!d->pre_weight || (d->pre_bias && aligned16(d->pre_weight) && d->kh == 3 && d->stride == 1 &&
                                     d->pad == 1 && d->groups == 1 && d->nsrc == 1 && dt != YXH_F32),
                  "fused Bottleneck: 16-bit 3x3 s1 conv over one source with a pre_bias");
    if (d->pre_weight && d->tile == 0)  // default fused tile per channel count
        return conv_ws_dispatch(dt, d->cin == 32 ? 191 - 160 : d->cin == 64 ? 194 - 160 : 195 - 160, p, st);
    if (d->pre_weight && (d->tile >> 1) <= 160 + 30) {
        set_error("fused Bottleneck runs on the conv_ws fused tiles (ids 191-196) only");
        return YXH_EUNSUPPORTED;
    }
    p.vec16 = d->dst_dtype == dt && ((uintptr_t)d->dst % 16) == 0 && (d->dst_cstride * des) % 16 == 0 &&
              (d->dst_bstride * des) % 16 == 0 && (d->cout * des) % 16 == 0;

    if (dw) {
        YXH_CHECK_ARG(d->dst_dtype == dt && d->act < YXH_ACT_DECODE, "depthwise output");
        const long long total = M * ((d->cin + epc - 1) / epc);
        dim3 grid((unsigned)((total + 255) / 256));
        if (dt == YXH_BF16) hipLaunchKernelGGL(dwconv<bf16>, grid, dim3(256), 0, st, p);
        else if (dt == YXH_F16) hipLaunchKernelGGL(dwconv<f16>, grid, dim3(256), 0, st, p);
        else hipLaunchKernelGGL(dwconv<float>, grid, dim3(256), 0, st, p);
        YXH_CHECK_LAUNCH("dwconv launch");
        return YXH_OK;
    }

    // K staging: two 64-byte slabs per stage when the channel structure allows it
    const int k2 = 8 * epc;
    // (every loader picks the source per 16-byte chunk, so a concat split only has to
    // fall on a chunk boundary -- checked above -- not on a stage boundary: yolox_x's
    // 80/160/320-channel CSP halves)
    int ks = d->cin >= k2 ? 2 : 1;
    int tile = heuristic_tile(p);
    if (d->tile > 0) {
        tile = d->tile >> 1;
        const int want_ks = (d->tile & 1) + 1;
        YXH_CHECK_ARG((tile > 0 && tile < kNumTiles) || (tile > 16 && tile < 16 + kNumTiles) ||
                          (tile > 32 && tile <= 32 + kNumRowTiles) || (tile > 64 && tile <= 64 + kNumPwTiles) ||
                          (tile > 80 && tile <= 80 + kNumPwrTiles) || (tile > 96 && tile <= 96 + kNumPwfTiles) ||
                          (tile > 112 && tile <= 112 + kNumR3Tiles) || (tile > 160 && tile <= 160 + kNumWsTiles) ||
                          (tile > 200 && tile <= 200 + kNumWs1Tiles) || (tile > 210 && tile <= 210 + kNumPw1fTiles) ||
                          (tile > 214 && tile <= 214 + kNumDgradS2Tiles) ||
                          (tile > 220 && tile <= 220 + kNumWsPostTiles) ||
                          (tile > 240 && tile <= 240 + kNumWs1DeepTiles) ||
                          (tile > 260 && tile <= 260 + kNumWsWideTiles),
                      "tile %d", d->tile);
        YXH_CHECK_ARG(want_ks == 1 || ks == 2, "2-slab staging not possible for this conv");
        ks = want_ks;
    }
    const int kstage = 4 * ks * epc;
    p.ncb = (d->cin + kstage - 1) / kstage;
    if (tile > 260) return conv_ws_dispatch(dt, tile - 260 + 60, p, st);
    // conv_ws1 (tiles 201-210, 241-258): the slab bit selects the 16-byte-store epilogue (conv_ws1.hip V16, where
    // the destination rows allow it; tiles without it refuse the odd code); the autotuner times both codes.  (The
    // same epilogue in conv_ws measured neutral on the bench and was dropped)
    if ((tile > 240 && tile <= 240 + kNumWs1DeepTiles) || (tile > 200 && tile <= 200 + kNumWs1Tiles))
        p.v16_req = ks == 2;
    if (tile > 240) return conv_ws1_dispatch(dt, tile - 240 + kNumWs1Tiles, p, st);
    if (tile > 220) return conv_ws_dispatch(dt, tile - 220 + 40, p, st);
    if (tile > 214) return dgrad_s2f_dispatch(dt, tile - 214, p, st);
    if (dilated && tile > 16) {
        set_error("dilated (upsample == 2) sources run on the register-staged kernel only (tile ids 1-9)");
        return YXH_EUNSUPPORTED;
    }
    if (tile > 210) return conv_pw1f_dispatch(dt, tile - 210, p, st);
    if (tile > 200) return conv_ws1_dispatch(dt, tile - 200, p, st);
    if (tile > 160) return conv_ws_dispatch(dt, tile - 160, p, st);
    if (tile > 112) return conv_r3_dispatch(dt, tile - 112, p, st);
    if (tile > 96) return conv_pwf_dispatch(dt, tile - 96, p, st);
    if (tile > 80) return conv_pwr_dispatch(dt, tile - 80, p, st);
    if (tile > 64) return conv_pw_dispatch(dt, tile - 64, p, ks, st);
    if (tile > 32) return conv_rows_dispatch(dt, tile - 32, p, ks, st);
    if (tile > 16) return conv_glds_dispatch(dt, tile - 16, p, ks, st);
    if (dt == YXH_BF16) return launch_tile<bf16>(tile, p, ks, st);
    if (dt == YXH_F16) return launch_tile<f16>(tile, p, ks, st);
    return launch_tile<float>(tile, p, ks, st);
}

int focus_pack_launch(const void* img, int layout, int idt, int B, int H, int W, void* dst, int odt,
                      hipStream_t st) {
    YXH_CHECK_ARG(img && dst, "null pointer");
    YXH_CHECK_ARG(B > 0 && H > 1 && W > 1 && H % 2 == 0 && W % 2 == 0, "image size %dx%d", H, W);
    YXH_CHECK_ARG(layout == YXH_NCHW || layout == YXH_NHWC, "layout %d", layout);
    YXH_CHECK_ARG(aligned16(dst), "dst not aligned");
    const long long total = (long long)B * (H / 2) * (W / 2);
    dim3 grid((unsigned)((total + 255) / 256));
#define YXH_FOCUS(TI, TO) \
    hipLaunchKernelGGL((focus_pack<TI, TO>), grid, dim3(256), 0, st, (const TI*)img, layout, B, H, W, (TO*)dst)
#define YXH_FOCUS_OUT(TI)                          \
    if (odt == YXH_BF16) YXH_FOCUS(TI, bf16);      \
    else if (odt == YXH_F16) YXH_FOCUS(TI, f16);   \
    else if (odt == YXH_F32) YXH_FOCUS(TI, float); \
    else { set_error("focus dst dtype %d", odt); return YXH_EINVAL; }
    if (idt == YXH_F32) { YXH_FOCUS_OUT(float) }
    else if (idt == YXH_U8) { YXH_FOCUS_OUT(uint8_t) }
    else if (idt == YXH_BF16) { YXH_FOCUS_OUT(bf16) }
    else if (idt == YXH_F16) { YXH_FOCUS_OUT(f16) }
    else { set_error("focus img dtype %d", idt); return YXH_EINVAL; }
#undef YXH_FOCUS_OUT
#undef YXH_FOCUS
    YXH_CHECK_LAUNCH("focus_pack launch");
    return YXH_OK;
}

int spp_launch(void* buf, int dt, int B, int H, int W, int C, int cs, long long bs, hipStream_t st) {
    YXH_CHECK_ARG(buf && aligned16(buf), "spp buffer");
    const int es = elem_size(dt), epc = 16 / es;
    YXH_CHECK_ARG(dt == YXH_F32 || dt == YXH_BF16 || dt == YXH_F16, "spp dtype");
    YXH_CHECK_ARG(C % epc == 0 && cs % epc == 0 && bs % epc == 0 && cs >= 4 * C, "spp channels/strides");
    const int nch = C / epc;
    const size_t plane = (size_t)4 * H * W * 16;
    YXH_CHECK_ARG(plane <= 160 * 1024, "spp plane %dx%d too large for LDS", H, W);
    // chunks per block: the widest of 4 / 2 that divides the channels, fits LDS and still
    // leaves >= 512 blocks (two per CU); else 1
    int cpb = 1;
    for (int c = 4; c >= 2; c /= 2)
        if (nch % c == 0 && c * plane <= 160 * 1024 && (long long)(nch / c) * B >= 512) {
            cpb = c;
            break;
        }
    const size_t lds = plane * cpb;
    dim3 grid(nch / cpb, B);
#define YXH_SPP(T, CPB)                                                                                  \
    do {                                                                                                 \
        (void)hipFuncSetAttribute((const void*)spp_maxpool<T, CPB>,                                    \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                    \
        hipLaunchKernelGGL((spp_maxpool<T, CPB>), grid, dim3(256), lds, st, (T*)buf, H, W, C, cs, bs);   \
    } while (0)
#define YXH_SPP_T(T)                 \
    do {                             \
        if (cpb == 4) YXH_SPP(T, 4);     \
        else if (cpb == 2) YXH_SPP(T, 2); \
        else YXH_SPP(T, 1);          \
    } while (0)
    if (dt == YXH_BF16) YXH_SPP_T(bf16);
    else if (dt == YXH_F16) YXH_SPP_T(f16);
    else YXH_SPP_T(float);
#undef YXH_SPP_T
#undef YXH_SPP
    YXH_CHECK_LAUNCH("spp launch");
    return YXH_OK;
}

int pack_frag_launch(const void* w, int cout, int taps, int cin, int dt, void* out, hipStream_t st) {
    YXH_CHECK_ARG(w && out && aligned16(w) && aligned16(out), "pack_frag: null / unaligned");
    YXH_CHECK_ARG(dt == YXH_BF16 || dt == YXH_F16, "pack_frag: 16-bit weights");
    YXH_CHECK_ARG(cout > 0 && cout % 16 == 0 && taps > 0 && cin > 0 && cin % 32 == 0, "pack_frag geometry");
    const long long total = (long long)(cout / 16) * taps * (cin / 32) * 64;
    hipLaunchKernelGGL(pack_frag, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, (const uint4*)w, cout,
                       taps, cin, (uint4*)out);
    YXH_CHECK_LAUNCH("pack_frag");
    return YXH_OK;
}

int fold_launch(const float* w, const float* cb, const float* g, const float* beta, const float* mean,
                const float* var, float eps, int cout, int cin_g, int kh, int kw, int cin_pad, int dt, void* wo,
                float* bo, hipStream_t st) {
    YXH_CHECK_ARG(w && wo && bo, "null pointer");
    YXH_CHECK_ARG(!g || (beta && mean && var), "partial BN parameters");
    YXH_CHECK_ARG(cout > 0 && cin_g > 0 && cin_pad >= cin_g && kh > 0 && kw > 0, "fold geometry");
    const long long total = (long long)cout * kh * kw * cin_pad;
    dim3 grid((unsigned)((total + 255) / 256));
    if (dt == YXH_BF16)
        hipLaunchKernelGGL(fold_bn_pack<bf16>, grid, dim3(256), 0, st, w, cb, g, beta, mean, var, eps, cout,
                           cin_g, kh, kw, cin_pad, (bf16*)wo, bo);
    else if (dt == YXH_F16)
        hipLaunchKernelGGL(fold_bn_pack<f16>, grid, dim3(256), 0, st, w, cb, g, beta, mean, var, eps, cout,
                           cin_g, kh, kw, cin_pad, (f16*)wo, bo);
    else if (dt == YXH_F32)
        hipLaunchKernelGGL(fold_bn_pack<float>, grid, dim3(256), 0, st, w, cb, g, beta, mean, var, eps, cout,
                           cin_g, kh, kw, cin_pad, (float*)wo, bo);
    else {
        set_error("fold dtype %d", dt);
        return YXH_EINVAL;
    }
    YXH_CHECK_LAUNCH("fold launch");
    return YXH_OK;
}

}  // namespace yxh
