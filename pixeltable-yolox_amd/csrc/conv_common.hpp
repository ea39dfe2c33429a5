// Pieces shared by the conv kernels (conv.hip, conv_glds.hip).
#pragma once

#include "yxh_common.hpp"

namespace yxh {

struct ConvParams {
    int in_h, in_w, out_h, out_w, cin, cout, kw, stride, pad;
    int M, ohw, taps, ncb, nsrc, src0_ch;
    const void* sptr[2];
    int scs[2], sw[2], sup[2];
    long long sbs[2];
    const void* w;
    const float* bias;
    const void* res;
    int res_cs;
    long long res_bs;
    void* dst;
    int dst_cs;
    long long dst_bs;
    int dst_f32, act, dcoff, vec_store, vec_res;
    int vec16;  // dst rows 16-byte aligned and cout a chunk multiple: LDS-staged epilogue
    int v16_req;  // conv_ws / conv_ws1: the 16-byte-store epilogue was asked for (odd tile code)
    int accum;  // f32 dst += result (YXH_CONV_ACCUMULATE: data-gradient accumulation)
    // image stride == pixels x pixel stride: pixel m lives at m * cs, no (b, pix) split
    // (the integer divides were most of a 1x1 conv's VALU work: tools/gpu_pmc.sh)
    int dst_dense, res_dense;
    int src_dense;  // 1x1 s1 p0 over sources without upsample whose pixel m is at m * scs
    float dstride;
    const void* pw1;  // fused Bottleneck conv1 (1x1, cin -> cin) ahead of the 3x3: conv_ws only
    const float* pb1;
    int grp2;  // YXH_CONV_GROUPS2: output half g reads source channels [g*cin, (g+1)*cin)
    const void* wf;  // weights in yxh_pack_frag's fragment-major layout, or null (conv_ws / conv_ws1)
    int cus;         // CUs the persistent grids may occupy (yxh_conv_desc.grid_cap; 256 = all)
    // 1x1 post conv (yxh_conv_desc.post_*): conv_ws post tiles only
    const void* pgw;
    const float* pgb;
    void* pgd;
    int pgd_cs;
    long long pgd_bs;
    const void* pgs;
    int pgs_cs, pgs_ch;
    long long pgs_bs;
    int pg_cout;
    // head form (groups2 + post_weight2): group 1's preds, the decode stride
    const void* pgw2;
    const float* pgb2;
    int pg_cout2;
    float pg_stride;
    int pg_store;  // YXH_CONV_POST_STORE: the conv output tile is stored to dst as well
};

// Stationary weight fragment (i: 16 output channels from n_first, tap, kb: 32-channel K block)
// of a weight-stationary tile: one 1 KiB wave read from the fragment-major copy when present
// (whole 128-byte lines), else 16 row pieces of 64 bytes from [cout][taps][cin].
template <typename T>
__device__ __forceinline__ uint4 ws_weight(const ConvParams& p, int n_first, int tap, int taps, int cin, int kb,
                                           int lane) {
    const int frow = lane & 15, fq = lane >> 4;
    if (p.wf) {
        const int nf = min(n_first, p.cout - 16) >> 4;
        return ((const uint4*)p.wf)[((long long)(nf * taps + tap) * (cin >> 5) + kb) * 64 + lane];
    }
    const int n = min(n_first + frow, p.cout - 1);
    return *(const uint4*)((const T*)p.w + ((long long)n * taps + tap) * cin + kb * 32 + fq * 8);
}

// ---------------------------------------------------------------- MFMA step
// One 64-byte K slab: lane l holds row (l & 15), 16-byte chunk (l >> 4) of both
// operands.  bf16/f16: a single 16x16x32 MFMA.  f32: four 16x16x4 MFMAs; step e
// takes element e of every chunk, i.e. K is permuted identically for A and B.
template <typename T> struct Mma;
template <> struct Mma<bf16> {
    static __device__ __forceinline__ void run(f32x4& acc, const uint4& a, const uint4& b) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                      __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
    }
};
template <> struct Mma<f16> {
    static __device__ __forceinline__ void run(f32x4& acc, const uint4& a, const uint4& b) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                     __builtin_bit_cast(f16x8, b), acc, 0, 0, 0);
    }
};
template <> struct Mma<float> {
    static __device__ __forceinline__ void run(f32x4& acc, const uint4& a, const uint4& b) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
    }
};

// ---------------------------------------------------------------- epilogue
template <typename T>
__device__ __forceinline__ void finish4(const ConvParams& p, float v[4], int n, int b, int pix, int ox,
                                        int oy) {
    if (p.act >= YXH_ACT_DECODE) {
        // yolo_head.py:233-251 (eval) / :213-231 (train): fp32 output rows
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            int ch = p.dcoff + n + r;
            if (ch < 4) {
                if (p.act != YXH_ACT_DECODE_RAW)
                    v[r] = ch < 2 ? (v[r] + (float)(ch == 0 ? ox : oy)) * p.dstride : expf(v[r]) * p.dstride;
            } else if (p.act != YXH_ACT_DECODE_TRAIN) {
                v[r] = 1.0f / (1.0f + expf(-v[r]));
            }
        }
    } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = apply_act<sizeof(T) == 4>(v[r], p.act);
    }
    const bool full = n + 3 < p.cout;
    if (p.res) {
        const T* rp = (const T*)p.res + (long long)b * p.res_bs + (long long)pix * p.res_cs + n;
        if (full && p.vec_res && sizeof(T) == 2) {
            uint2 u = *(const uint2*)rp;
            T t[4];
            __builtin_memcpy(t, &u, 8);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += to_f32(t[r]);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (n + r < p.cout) v[r] += to_f32(rp[r]);
        }
    }
}

template <typename T>
__device__ __forceinline__ void store4(const ConvParams& p, float v[4], int n, int b, int pix, int ox,
                                       int oy) {
    finish4<T>(p, v, n, b, pix, ox, oy);
    const bool full = n + 3 < p.cout;
    long long off = (long long)b * p.dst_bs + (long long)pix * p.dst_cs + n;
    if (p.dst_f32) {
        float* dp = (float*)p.dst + off;
        if (p.accum) {
            if (full && p.vec_store) {
                const float4 o = *(const float4*)dp;
                v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (n + r < p.cout) v[r] += dp[r];
            }
        }
        if (full && p.vec_store) {
            *(float4*)dp = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (n + r < p.cout) dp[r] = v[r];
        }
    } else {
        T* dp = (T*)p.dst + off;
        if (full && p.vec_store && sizeof(T) == 2) {
            T t[4] = {from_f32<T>(v[0]), from_f32<T>(v[1]), from_f32<T>(v[2]), from_f32<T>(v[3])};
            uint2 u;
            __builtin_memcpy(&u, t, 8);
            *(uint2*)dp = u;
        } else if (full && p.vec_store) {
            *(float4*)dp = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (n + r < p.cout) dp[r] = from_f32<T>(v[r]);
        }
    }
}

// Epilogue shared by the conv kernels: lane holds channels n..n+3 (rows 4*fq..) of
// pixel column frow for every (i, j) fragment.  `map(pl)` turns a tile-local pixel
// index into the global output pixel m = b*ohw + pix (or -1 outside the output).
// Staged form: bias/act/residual in registers, the [TM pixels][TN channels] tile of
// the output dtype goes through LDS, then whole pixel rows leave as 16-byte chunks
// (coalesced) instead of 8-byte lane-scattered stores.  Caller guarantees all LDS
// reads of the K loop are done.
// The bias of this lane's output channels, loaded before the K loop so the epilogue
// does not start with a dependent global round trip (caller: load_lane_bias at entry).
template <int TN, int WR, int WC>
__device__ __forceinline__ void load_lane_bias(const ConvParams& p, int n0, float (&bias)[TN / WR / 16][4]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, fq = lane >> 4;
    const int wr = wave / WC;
#pragma unroll
    for (int i = 0; i < TN / WR / 16; ++i) {
        const int n = n0 + wr * (TN / WR) + i * 16 + fq * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[i][r] = n + r < p.cout ? p.bias[n + r] : 0.0f;
    }
}

template <typename T, int TN, int TM, int WR, int WC, int SMEM_BYTES, typename Map>
__device__ __forceinline__ void conv_epilogue_map(const ConvParams& p, f32x4 (&acc)[TN / WR / 16][TM / WC / 16],
                                                  char* smem, const Map& map, int n0,
                                                  const float (&bias)[TN / WR / 16][4]) {
    constexpr int WTN = TN / WR, WTM = TM / WC;
    constexpr int FR = WTN / 16, FC = WTM / 16;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WC, wc = wave % WC;
    const int frow = lane & 15, fq = lane >> 4;
    constexpr int OES = sizeof(T);
    constexpr int OROW = TN * OES + 16;  // +16 B: 16-byte aligned rows, <= 2-way write conflicts
    constexpr bool CAN_STAGE = TM * OROW <= SMEM_BYTES && (TN * OES) % 16 == 0;
    if (CAN_STAGE && p.vec16 && !p.dst_f32) {
#pragma unroll
        for (int j = 0; j < FC; ++j) {
            const int pl = wc * WTM + j * 16 + frow;
            const int m = map(pl);
            const int mm = m >= 0 ? m : 0;
            // residual offset b*res_bs + pix*res_cs; no decode on this path (bf16/f16 dst)
            int b = 0, pix = mm;
            if (p.res && !p.res_dense) {
                b = mm / p.ohw;
                pix = mm - b * p.ohw;
            }
            const int oy = 0, ox = 0;
#pragma unroll
            for (int i = 0; i < FR; ++i) {
                const int nl = wr * WTN + i * 16 + fq * 4;
                const int n = n0 + nl;
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[i][r];
                if (m >= 0 && n < p.cout) finish4<T>(p, v, n, b, pix, ox, oy);
                T t[4] = {from_f32<T>(v[0]), from_f32<T>(v[1]), from_f32<T>(v[2]), from_f32<T>(v[3])};
                char* dstl = smem + pl * OROW + nl * OES;
                if constexpr (OES == 2) {
                    uint2 u;
                    __builtin_memcpy(&u, t, 8);
                    *(uint2*)dstl = u;
                } else {
                    uint4 u;
                    __builtin_memcpy(&u, t, 16);
                    *(uint4*)dstl = u;
                }
            }
        }
        __syncthreads();
        constexpr int CPO = TN * OES / 16;  // 16-byte chunks per output row
        const int ncols = min(TN, p.cout - n0) * OES / 16;
        for (int q = tid; q < TM * CPO; q += 64 * WR * WC) {
            const int r = q / CPO, c = q - r * CPO;
            const int m = map(r);
            if (m < 0 || c >= ncols) continue;
            long long off;
            if (p.dst_dense) {
                off = (long long)m * p.dst_cs;
            } else {
                const int b = m / p.ohw, pix = m - b * p.ohw;
                off = (long long)b * p.dst_bs + (long long)pix * p.dst_cs;
            }
            const uint4 u = *(const uint4*)(smem + r * OROW + c * 16);
            *(uint4*)((char*)p.dst + (off + n0) * OES + c * 16) = u;
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < FC; ++j) {
        const int m = map(wc * WTM + j * 16 + frow);
        if (m < 0) continue;
        const int b = m / p.ohw, pix = m - b * p.ohw;
        const int oy = pix / p.out_w, ox = pix - oy * p.out_w;
#pragma unroll
        for (int i = 0; i < FR; ++i) {
            const int n = n0 + wr * WTN + i * 16 + fq * 4;
            if (n >= p.cout) continue;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[i][r];
            store4<T>(p, v, n, b, pix, ox, oy);
        }
    }
}

// Linear pixel tiles: tile-local pixel pl is output pixel m0 + pl.
template <typename T, int TN, int TM, int WR, int WC, int SMEM_BYTES>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, f32x4 (&acc)[TN / WR / 16][TM / WC / 16],
                                              char* smem, int m0, int n0, const float (&bias)[TN / WR / 16][4]) {
    const int M = p.M;
    conv_epilogue_map<T, TN, TM, WR, WC, SMEM_BYTES>(
        p, acc, smem, [m0, M](int pl) { return m0 + pl < M ? m0 + pl : -1; }, n0, bias);
}

// LDS-DMA variant (conv_glds.hip); id as in conv.hip's tile table
int conv_glds_dispatch(int dtype, int id, const ConvParams& p, int ks, hipStream_t st);
// Row-tiled 3x3 conv (conv_rows.hip): 2D output tiles, kx taps share one LDS row image
int conv_rows_dispatch(int dtype, int id, const ConvParams& p, int ks, hipStream_t st);
constexpr int kNumRowTiles = 19;
// Persistent streaming 1x1 conv (conv_pw.hip): tile ids 65..64+kNumPwTiles
int conv_pw_dispatch(int dtype, int id, const ConvParams& p, int ks, hipStream_t st);
constexpr int kNumPwTiles = 6;
// Register-operand 1x1 conv (conv_pwr.hip): tile ids 81..80+kNumPwrTiles
int conv_pwr_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st);
constexpr int kNumPwrTiles = 2;
// VALU-free-loop dense 1x1 conv (conv_pwf.hip): tile ids 97..96+kNumPwfTiles
int conv_pwf_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st);
constexpr int kNumPwfTiles = 8;
// 3x3 conv with the branch-free buffer-LDS loader (conv_r3.hip): tile ids 113..112+kNumR3Tiles
int conv_r3_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st);
constexpr int kNumR3Tiles = 48;  // ids beyond the built ones report EINVAL
// Weight-stationary persistent 3x3 conv (conv_ws.hip): tile ids 161..160+kNumWsTiles
int conv_ws_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st);
constexpr int kNumWsTiles = 36;  // 31..36: fused Bottleneck (pre_weight)
// conv_ws tiles with a 1x1 post conv (yxh_conv_desc.post_weight): tile ids 221..220+kNumWsPostTiles
// (conv_ws_dispatch ids 41..40+kNumWsPostTiles)
constexpr int kNumWsPostTiles = 16;
// Weight-stationary persistent 1x1 conv over dense sources (conv_ws1.hip): tile ids 201..200+kNumWs1Tiles
int conv_ws1_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st);
constexpr int kNumWs1Tiles = 10;
// ... and its deep row pipelines (conv_ws1 ids 11..10+kNumWs1DeepTiles): tile ids 241..240+kNumWs1DeepTiles
constexpr int kNumWs1DeepTiles = 18;  // 249-252, 256: upsampled source 0; 253-258: full-width (round 5)
// fp32 1x1 GEMM for the training path, k-minor MFMA operands (conv_pw1f.hip): tile ids 211..210+kNumPw1fTiles
int conv_pw1f_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st);
constexpr int kNumPw1fTiles = 4;
// fp32 data gradient of a 3x3 s2 conv by output parity class (conv_pw1f.hip): tile ids 215..216
int dgrad_s2f_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st);
constexpr int kNumDgradS2Tiles = 6;  // 215-216 fp32 (dgrad_s2f), 217-220 16-bit (dgrad_s2h)

}  // namespace yxh
