// head_pred: the three 1x1 pred convs of one YOLOX head level + cat + sigmoid + decode
// in ONE kernel (reference yolo_head.py:149-160 reg_preds / obj_preds / cls_preds,
// :185-187 cat([reg, obj.sigmoid(), cls.sigmoid()]), :205-207 flatten/permute,
// :233-251 decode_outputs), writing the level's rows of the [B, A, 5+C] fp32 output.
//
// Persistent blocks (weights loaded into LDS once) walk tiles of TM = 64 consecutive
// pixels m (image-major) of the level:
//  * the reg_feat and cls_feat tiles [64][cin] and both weight matrices ([5][cin] reg+obj,
//    [C][cin] cls, zero rows up to whole 16-row fragments) are staged in LDS (XOR-swizzled);
//  * wave w computes pixel fragment w (16 pixels) x every output-channel fragment
//    (1 reg/obj + ceil(C/16) cls) on MFMA 16x16x32 -- no block-diagonal zero work;
//  * bias + decode in registers: ch 0-1 (v + grid) * stride, ch 2-3 exp(v) * stride,
//    ch 4.. sigmoid -- hardware exp2 + reciprocal (hd_exp / hd_sigmoid, ~1 ulp each), NOT
//    the IEEE expf / divide of conv_common.hpp's fp32 decode path (test_gpu_ops.py
//    test_head_pred_fused_level: vs torch fp32 exp / sigmoid within 1e-4 abs + rel);
//  * the decoded [64][5+C] tile is staged in LDS and leaves as 16-byte stores over the
//    contiguous output rows (a level's rows of one image are consecutive; a tile
//    straddles at most one image boundary) -- instead of 4-byte scattered stores of
//    340-byte rows.
#include <stdlib.h>

#include <algorithm>

#include "conv_common.hpp"

namespace yxh {

namespace {

// The fused head runs on the 16-bit inference path only (the fp32 parity path keeps the
// decode convs and their IEEE exp / divide): hardware exp2 + reciprocal (~1 ulp each), as
// the bf16 SiLU -- the per-element exp / divide sequences were most of this kernel's VALU.
__device__ __forceinline__ float hd_exp(float v) { return __builtin_amdgcn_exp2f(v * 1.4426950408889634f); }
__device__ __forceinline__ float hd_sigmoid(float v) { return __builtin_amdgcn_rcpf(1.0f + hd_exp(-v)); }

}  // namespace

// CIN: feature channels (a multiple of 32); NCF: cls output fragments (16 rows each)
template <typename T, int CIN, int NCF>
__global__ __launch_bounds__(256) void head_pred(yxh_head_desc d) {
    constexpr int TM = 64;
    constexpr int EPC = Chunk<T>::N;
    constexpr int CPR = CIN / EPC;        // 16-byte chunks per row
    constexpr int ROWB = CIN * sizeof(T);
    constexpr int NF = 1 + NCF;           // output-channel fragments
    constexpr int WROWS = NF * 16;        // weight rows in LDS
    constexpr int XB = TM * ROWB;         // one feature tile
    constexpr int WB = WROWS * ROWB;
    constexpr int STG = TM * (5 + NCF * 16) * 4;  // staged rows, stride 5 + C (<= 5 + NCF * 16)
    __shared__ __attribute__((aligned(16))) char smem[2 * XB + WB + STG];
    char* xr = smem;            // reg_feat tile [TM][CIN] (chunks XOR-swizzled by row)
    char* xc = smem + XB;       // cls_feat tile
    char* wl = smem + 2 * XB;   // weights [WROWS][CIN]: row 0-4 reg+obj, 16.. cls
    float* stg = (float*)(smem + 2 * XB + WB);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int C = d.num_classes, hw = d.h * d.w;
    const int M = d.batch * hw;
    const int ntiles = (M + TM - 1) / TM;
    auto swz = [](int r, int c) { return c ^ (r & (CPR - 1)); };

    // weights once per block (the grid is persistent over pixel tiles)
    for (int q = tid; q < WROWS * CPR; q += 256) {
        const int r = q / CPR, c = q - r * CPR;
        const int cs = swz(r, c);
        uint4 v = make_uint4(0, 0, 0, 0);
        if (r < 5)
            v = *(const uint4*)((const T*)d.w_reg + (long long)r * CIN + cs * EPC);
        else if (r >= 16 && r - 16 < C)
            v = *(const uint4*)((const T*)d.w_cls + (long long)(r - 16) * CIN + cs * EPC);
        *(uint4*)(wl + q * 16) = v;
    }
    const int frow = lane & 15, fq = lane >> 4;
    const int rowf = 5 + C;

    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int m0 = tile * TM;
        const int b0 = m0 / hw, p0 = m0 - b0 * hw;
        // ---- feature tiles -> LDS (chunk c of row r stored at c ^ (r & (CPR - 1))): all
        // loads of the tile issued before any LDS store
        constexpr int NQ = TM * CPR / 256;  // 16-byte chunks per thread per tensor
        uint4 vr[NQ], vc[NQ];
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const int q = tid + 256 * k;
            const int r = q / CPR, c = q - r * CPR;
            int pix = p0 + min(r, M - 1 - m0), b = b0;
            while (pix >= hw) {  // levels smaller than a tile: several images per tile
                pix -= hw;
                ++b;
            }
            const int cs = swz(r, c);
            vr[k] = *(const uint4*)((const T*)d.reg.ptr + (long long)b * d.reg.bstride + (long long)pix * d.reg.cstride +
                                    cs * EPC);
            vc[k] = *(const uint4*)((const T*)d.cls.ptr + (long long)b * d.cls.bstride + (long long)pix * d.cls.cstride +
                                    cs * EPC);
        }
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const int q = tid + 256 * k;
            *(uint4*)(xr + q * 16) = vr[k];
            *(uint4*)(xc + q * 16) = vc[k];
        }
        __syncthreads();

        // ---- MFMA: out[ch][pix], wave = pixel fragment
        f32x4 acc[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int pr = wave * 16 + frow;  // tile pixel of this lane's B fragment
#pragma unroll
        for (int s = 0; s < CIN / 32; ++s) {
            const int ch = s * 4 + fq;
            const uint4 br = *(const uint4*)(xr + (pr * CPR + swz(pr, ch)) * 16);
            const uint4 bc = *(const uint4*)(xc + (pr * CPR + swz(pr, ch)) * 16);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int wr = f * 16 + frow;
                const uint4 a = *(const uint4*)(wl + (wr * CPR + swz(wr, ch)) * 16);
                Mma<T>::run(acc[f], a, f == 0 ? br : bc);
            }
        }

        // ---- bias + decode -> staged fp32 rows
        {
            int pix = p0 + min(pr, M - 1 - m0);
            while (pix >= hw) pix -= hw;
            const int gy = pix / d.w, gx = pix - gy * d.w;
            const float st = d.stride;
            float* row = stg + pr * rowf;
#pragma unroll
            for (int f = 0; f < NF; ++f) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int ch = f * 16 + fq * 4 + r;  // fragment row
                    float v = acc[f][r];
                    if (f == 0) {
                        if (ch < 5) {
                            v += d.b_reg[ch];
                            if (ch < 4) {
                                if (d.train != 2) v = ch < 2 ? (v + (float)(ch == 0 ? gx : gy)) * st : hd_exp(v) * st;
                            } else {
                                v = d.train == 1 ? v : hd_sigmoid(v);
                            }
                            row[ch] = v;
                        }
                    } else {
                        const int c = ch - 16;
                        if (c < C) {
                            v += d.b_cls[c];
                            row[5 + c] = d.train == 1 ? v : hd_sigmoid(v);
                        }
                    }
                }
            }
        }
        __syncthreads();

        // ---- the staged rows have the output's row stride, so each piece of the tile (it
        // splits at an image boundary) is one contiguous, 16-byte aligned run in both LDS and
        // the output: a plain float4 copy
        const int n = min(TM, M - m0);
        int t0 = 0, b = b0, pix = p0;
        while (t0 < n) {
            const int cnt = min(n - t0, hw - pix);
            float* dst = d.out + (long long)b * d.out_bstride + (long long)(d.a_off + pix) * rowf;
            const float* src = stg + t0 * rowf;
            const int total = cnt * rowf;  // floats, a multiple of 4 (cnt % 4 == 0)
            for (int q = tid * 4; q < total; q += 1024) *(float4*)(dst + q) = *(const float4*)(src + q);
            t0 += cnt;
            ++b;
            pix = 0;
        }
        __syncthreads();  // staging and feature tiles are reused by the next tile
    }
}

// head_pred2 (CIN 64 / 128): every wave an independent worker over 16-pixel groups.  head_pred
// above spent 68 % of its wave cycles waiting (profiles/r04/mfma_util_r4z.txt): each tile's
// feature loads were issued and waited for before any MFMA, and two barriers per tile
// serialised the block.  Here
//  * a wave's B operands come straight from global memory into registers (lane (r, q) of
//    step s: pixel r's channels 32 s + 8 q .. + 8 -- 64-byte segments of the pixel rows), the
//    NEXT group's loads issued before this group's MFMAs, so HBM latency hides behind a whole
//    group of work;
//  * the weights of all 6 output fragments live in VGPRs for the wave's life (one LDS copy per
//    block feeds them), the biases in LDS;
//  * the decoded [16][5 + C] rows go through a per-wave LDS slot and leave as 16-byte stores of
//    the contiguous output rows -- no block barrier after the prologue.
// Same MFMA order and decode arithmetic as head_pred: bit-identical output
// (tests/test_gpu_ops.py test_head_pred_fused_level runs both).
// MODE = yxh_head_desc.train, fixed per instantiation (0: eval decode, 1: training rows -- decoded boxes, raw
// obj / cls logits, 2: eval raw rows -- raw boxes, sigmoid obj / cls): the decode is branch-free (every lane
// evaluates its fragment-0 candidates and selects; 32-bit pixel / image arithmetic), where the runtime mode
// tests and per-lane branches had split it into exec-masked blocks with SGPR spills (round 6)
// 8 waves per block (two per SIMD) for 64 / 128 channels; 4 for 256 (yolox_l: its 6 x 8 weight fragments and the
// two groups of 16 feature operands need ~350 registers, one wave per SIMD)
constexpr int head2_waves(int cin) { return cin >= 256 ? 4 : 8; }

template <typename T, int CIN, int NCF, int MODE>
__global__ __launch_bounds__(64 * head2_waves(CIN)) void head_pred2(yxh_head_desc d) {
    constexpr int NW = head2_waves(CIN);
    constexpr int KS = CIN / 32;                 // K steps
    constexpr int NF = 1 + NCF;                  // output fragments: reg|obj, then cls
    constexpr int WROWS = NF * 16;
    constexpr int WRB = CIN * 2 + 16;            // LDS weight row: +16 B (odd 16-B slots: conflict-free)
    constexpr int STGF = 16 * (5 + NCF * 16);    // per-wave staging floats (>= 16 rows of 5 + C)
    // ~70 KB of LDS for CIN 128: one block per CU on gfx950 (160 KiB), built for that target only
    static_assert(WROWS * WRB + WROWS * 4 + NW * STGF * 4 <= 160 * 1024, "head_pred2 LDS exceeds gfx950's 160 KiB");
    __shared__ __attribute__((aligned(16))) char wl[WROWS * WRB];
    __shared__ float bl[WROWS];
    __shared__ __attribute__((aligned(16))) float stg_all[NW][STGF];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int frow = lane & 15, fq = lane >> 4;
    const int C = d.num_classes, hw = d.h * d.w, rowf = 5 + C, W = d.w;
    const int M = d.batch * hw;  // < 2^31 (head_pred_launch)
    const int G = (M + 15) / 16;
    const int gstride = (int)gridDim.x * NW;
    int g = (int)blockIdx.x * NW + wave;
    // ---- weights / biases -> LDS (rows past 5 reg|obj and C cls rows are zero), then VGPRs
    for (int q = tid; q < WROWS * (CIN / 8); q += 64 * NW) {
        const int r = q / (CIN / 8), c = q - (CIN / 8) * (q / (CIN / 8));
        uint4 v = make_uint4(0, 0, 0, 0);
        if (r < 5) v = *(const uint4*)((const T*)d.w_reg + (long long)r * CIN + c * 8);
        else if (r >= 16 && r - 16 < C) v = *(const uint4*)((const T*)d.w_cls + (long long)(r - 16) * CIN + c * 8);
        *(uint4*)(wl + r * WRB + c * 16) = v;
    }
    for (int q = tid; q < WROWS; q += 64 * NW)
        bl[q] = q < 5 ? d.b_reg[q] : (q >= 16 && q - 16 < C) ? d.b_cls[q - 16] : 0.0f;
    __syncthreads();
    uint4 wr[NF][KS];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int s = 0; s < KS; ++s) wr[f][s] = *(const uint4*)(wl + (f * 16 + frow) * WRB + (s * 4 + fq) * 16);
    if (g >= G) return;  // wave-uniform; no block barrier follows

    // B operands of group g: [0..KS) reg features, [KS..2KS) cls features of pixel 16 g + frow
    auto load_b = [&](int gg, uint4 (&b)[2 * KS]) {
        int m = gg * 16 + frow;
        m = m < M ? m : M - 1;
        const int bi = m / hw, pix = m - bi * hw;
        const T* pr = (const T*)d.reg.ptr + (long long)bi * d.reg.bstride + (long long)pix * d.reg.cstride + fq * 8;
        const T* pc = (const T*)d.cls.ptr + (long long)bi * d.cls.bstride + (long long)pix * d.cls.cstride + fq * 8;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            b[s] = *(const uint4*)(pr + s * 32);
            b[KS + s] = *(const uint4*)(pc + s * 32);
        }
    };
    float* stg = stg_all[wave];
    uint4 bc[2 * KS], bn[2 * KS];
    load_b(g, bc);
    const float st = d.stride;
    for (; g < G; g += gstride) {
        const bool more = g + gstride < G;
        if (more) load_b(g + gstride, bn);
        f32x4 acc[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int f = 0; f < NF; ++f) Mma<T>::run(acc[f], wr[f][s], f == 0 ? bc[s] : bc[KS + s]);
        // ---- bias + decode -> this wave's staging rows (row = frow, the group's pixel)
        const int m0 = g * 16;
        int m = m0 + frow;
        m = m < M ? m : M - 1;
        const int img = m / hw, pix = m - img * hw;
        const int gy = pix / W, gx = pix - gy * W;
        float* row = stg + frow * rowf;
        // serving score records (ABI 18): this lane's classes (f - 1) * 16 + fq * 4 + r, in increasing
        // order, scanned as postprocess.hip's filter scans a row (class 0 -- lane fq 0 -- starts the
        // scan even when NaN, every later class replaces only on a strict '>'), from the very values
        // the row gets
        float cbest = -INFINITY, objv = 0.0f;
        float boxv[4];  // ch 0-3 (lane fq 0): the decoded box, copied into the record
        int cbi = C;
        // fragment 0: lane row fq 0 holds ch 0-3 (the box), fq 1 ch 4 (obj); every lane evaluates both
        // candidates of its values and selects (the same arithmetic as the branchy form: bit-identical)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int ch = fq * 4 + r;
            const float v = acc[0][r] + bl[ch];
            float bx = v;
            if constexpr (MODE != 2) bx = r < 2 ? (v + (float)(r == 0 ? gx : gy)) * st : hd_exp(v) * st;
            const float ob = MODE == 1 ? v : hd_sigmoid(v);
            boxv[r] = bx;
            if (r == 0) objv = ob;  // lane row fq 1: ch 4
            if (ch < 5) row[ch] = ch < 4 ? bx : ob;
        }
#pragma unroll
        for (int f = 1; f < NF; ++f) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ch = f * 16 + fq * 4 + r;
                const float v = acc[f][r] + bl[ch];
                const float sv = MODE == 1 ? v : hd_sigmoid(v);
                if (ch - 16 < C) {
                    row[5 + ch - 16] = sv;
                    if (ch == 16 || sv > cbest) {
                        cbest = sv;
                        cbi = ch - 16;
                    }
                }
            }
        }
        if (d.scores != nullptr) {
            // the four lanes of a pixel (fq = 0..3: lanes frow + 16 fq) merged with the filter's rules
#pragma unroll
            for (int off = 16; off < 64; off <<= 1) {
                const float ob = __shfl_xor(cbest, off);
                const int oi = __shfl_xor(cbi, off);
                bool take;
                if (oi >= C) take = false;
                else if (cbi >= C) take = true;
                else if (cbest != cbest) take = false;  // class 0 is NaN: the serial answer
                else if (ob != ob) take = true;
                else take = ob > cbest || (ob == cbest && oi < cbi);
                if (take) { cbest = ob; cbi = oi; }
            }
            const float obj = __shfl(objv, frow + 16);  // ch 4 (obj) lives in lane fq = 1
            const int mr = m0 + frow;
            if (fq == 0 && mr < M) {
                float4* rec = (float4*)(d.scores + 8 * ((long long)img * (d.out_bstride / rowf) + d.a_off + pix));
                rec[0] = make_float4(obj * cbest, cbest, (float)cbi, obj);
                rec[1] = make_float4(boxv[0], boxv[1], boxv[2], boxv[3]);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): every lane's rows are in LDS
        __builtin_amdgcn_wave_barrier();
        const int n = M - m0 < 16 ? M - m0 : 16;
        // ---- the group's rows are contiguous in the output (split once at an image boundary)
        int t0 = 0, bi = m0 / hw, p0 = m0 - bi * hw;
        while (t0 < n) {
            const int cnt = min(n - t0, hw - p0);
            float* dst = d.out + (long long)bi * d.out_bstride + (long long)(d.a_off + p0) * rowf;
            const float* src = stg + t0 * rowf;
            const int total4 = cnt * rowf / 4;  // cnt % 4 == 0: 16-byte runs
            for (int q = lane; q < total4; q += 64) *(float4*)(dst + 4 * q) = *(const float4*)(src + 4 * q);
            t0 += cnt;
            ++bi;
            p0 = 0;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // the staging reads are done before the next group's writes
        __builtin_amdgcn_wave_barrier();
        if (more) {
#pragma unroll
            for (int q = 0; q < 2 * KS; ++q) bc[q] = bn[q];
        }
    }
}

int head_pred_launch(const yxh_head_desc* d, hipStream_t st) {
    YXH_CHECK_ARG(d && d->out && d->cls.ptr && d->reg.ptr && d->w_reg && d->w_cls && d->b_reg && d->b_cls,
                  "head_pred: null pointer");
    YXH_CHECK_ARG(d->batch > 0 && d->h > 0 && d->w > 0, "head_pred: empty level");
    YXH_CHECK_ARG(d->train >= 0 && d->train <= 2, "head_pred: mode %d", d->train);
    YXH_CHECK_ARG(((long long)d->h * d->w) % 4 == 0 && d->a_off % 4 == 0 && d->out_bstride % 4 == 0 &&
                      ((uintptr_t)d->out & 15) == 0,
                  "head_pred: level rows must be 16-byte aligned (h*w, a_off multiples of 4)");
    YXH_CHECK_ARG(d->reg.channels == d->cin && d->cls.channels == d->cin, "head_pred: feature channels");
    const long long M = (long long)d->batch * d->h * d->w;
    YXH_CHECK_ARG(M < (1LL << 31), "head_pred: too many pixels");
    const long long tiles = (M + 63) / 64;
    const unsigned grid = (unsigned)(tiles < 512 ? tiles : 512);  // persistent: weights loaded once per block
#define YXH_HEAD(T, CIN, NCF) \
    hipLaunchKernelGGL((head_pred<T, CIN, NCF>), dim3(grid), dim3(256), 0, st, *d)
    const int ncf = (d->num_classes + 15) / 16;
    if (ncf != 5) {
        set_error("head_pred built for 65-80 classes (got %d)", d->num_classes);
        return YXH_EUNSUPPORTED;
    }
    // head_pred2 for 64 / 128 feature channels (YXH_HEAD_V1=1: the tile kernel, for A/B and the
    // bit-identity test); 16-byte aligned feature rows
    const char* v1e = getenv("YXH_HEAD_V1");
    const bool v1 = v1e != nullptr && v1e[0] == '1';
    const bool rows16 = ((uintptr_t)d->reg.ptr % 16) == 0 && ((uintptr_t)d->cls.ptr % 16) == 0 &&
                        d->reg.cstride % 8 == 0 && d->cls.cstride % 8 == 0 && d->reg.bstride % 8 == 0 &&
                        d->cls.bstride % 8 == 0;
    YXH_CHECK_ARG(!d->scores || (!v1 && rows16 && (d->cin == 64 || d->cin == 128 || d->cin == 256) && d->train == 0 &&
                                 ((uintptr_t)d->scores % 16) == 0 && d->out_bstride % (5 + d->num_classes) == 0),
                  "head_pred: score records need the head_pred2 path (eval decode rows, 64 / 128 / 256 16-bit channels, "
                  "16-byte rows) and a 16-byte aligned buffer");
    if (!v1 && rows16 && (d->cin == 64 || d->cin == 128 || d->cin == 256)) {
        const long long groups = (M + 15) / 16;
#define YXH_HEAD2(T, CIN)                                                                                        \
    do {                                                                                                         \
        constexpr int nw = head2_waves(CIN);                                                                     \
        const unsigned grid2 = (unsigned)std::min<long long>((groups + nw - 1) / nw, device_cus()); /* a block per CU */ \
        if (d->train == 1) hipLaunchKernelGGL((head_pred2<T, CIN, 5, 1>), dim3(grid2), dim3(64 * nw), 0, st, *d);     \
        else if (d->train == 2) hipLaunchKernelGGL((head_pred2<T, CIN, 5, 2>), dim3(grid2), dim3(64 * nw), 0, st, *d); \
        else hipLaunchKernelGGL((head_pred2<T, CIN, 5, 0>), dim3(grid2), dim3(64 * nw), 0, st, *d);                \
    } while (0)
        if (d->dtype == YXH_BF16 && d->cin == 128) YXH_HEAD2(bf16, 128);
        else if (d->dtype == YXH_BF16 && d->cin == 256) YXH_HEAD2(bf16, 256);
        else if (d->dtype == YXH_BF16) YXH_HEAD2(bf16, 64);
        else if (d->dtype == YXH_F16 && d->cin == 128) YXH_HEAD2(f16, 128);
        else if (d->dtype == YXH_F16 && d->cin == 256) YXH_HEAD2(f16, 256);
        else if (d->dtype == YXH_F16) YXH_HEAD2(f16, 64);
        else {
            set_error("head_pred: dtype %d not built", d->dtype);
            return YXH_EUNSUPPORTED;
        }
#undef YXH_HEAD2
        YXH_CHECK_LAUNCH("head_pred2 launch");
        return YXH_OK;
    }
    if (d->dtype == YXH_BF16 && d->cin == 128) YXH_HEAD(bf16, 128, 5);
    else if (d->dtype == YXH_BF16 && d->cin == 64) YXH_HEAD(bf16, 64, 5);
    else if (d->dtype == YXH_BF16 && d->cin == 256) YXH_HEAD(bf16, 256, 5);
    else if (d->dtype == YXH_F16 && d->cin == 128) YXH_HEAD(f16, 128, 5);
    else if (d->dtype == YXH_F16 && d->cin == 64) YXH_HEAD(f16, 64, 5);
    else if (d->dtype == YXH_F16 && d->cin == 256) YXH_HEAD(f16, 256, 5);
    else {
        set_error("head_pred: dtype %d / %d channels not built", d->dtype, d->cin);
        return YXH_EUNSUPPORTED;
    }
#undef YXH_HEAD
    YXH_CHECK_LAUNCH("head_pred launch");
    return YXH_OK;
}

}  // namespace yxh
