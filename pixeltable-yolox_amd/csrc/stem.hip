// Fused Focus + stem conv on gfx950 (reference network_blocks.py:186-208 Focus,
// darknet.py:112 stem = Focus(3, 64*width, ksize=3) -> BaseConv 3x3 s1 on 12 ch).
//
// Focus channel (q, c) with q = TL, BL, TR, BR = (dy + 2*dx) of pixel (2i+dy, 2j+dx),
// followed by a 3x3 pad-1 conv, is exactly a 6x6 stride-2 pad-2 conv on the raw
// 3-channel image: kernel row ky6 = 2*ky3 + dy, column kx6 = 2*kx3 + dx.  In NHWC
// the 18 values (kx6, c) of one kernel row are contiguous, so each kernel row is one
// 32-wide K slab (weights zero past 18) and the MFMA B fragment of an output pixel is
// 8 (bf16) / 4 (f32) contiguous values of an LDS copy of the input rows -- no
// space-to-depth pass, no 12-channel intermediate in HBM.
//
// Two kernels share that formulation:
//  * stem_rows (16-bit compute, NHWC rows of whole 16-byte chunks): block = 4 output
//    rows x the whole image width; the 12 input rows are staged once with 16-byte
//    loads, the weights live in registers.
//  * stem_conv (everything else): block = 256 threads = 4 waves = a 4 x 64 tile of
//    output pixels of one image (wave w = output row), all output channels (<= 80).
//    The input rows the tile needs (12 x 132 pixels) are staged once in LDS (zero
//    outside the image), the output tile goes back through LDS and leaves as 16-byte
//    chunks of whole pixel rows.
#include "conv_common.hpp"

namespace yxh {

constexpr int kStemTY = 4, kStemTX = 64;
constexpr int kStemRows = 2 * kStemTY + 4;   // 12 input rows
constexpr int kStemRowElems = 416;          // >= (2*64+4)*3 = 396 and the last 32-wide read
constexpr int kStemK = 32;                  // per kernel row: 18 used

struct StemParams {
    const void* img;
    int layout, idt, B, H, W, OH, OW, cout, act;
    const void* w;  // [cout_pad][6][32]
    const float* bias;
    void* dst;
    int dst_cs;
    long long dst_bs;
    int force_tiles;  // tests: force the 4x64-tile kernel
};

template <typename TI>
__device__ __forceinline__ float load_px(const StemParams& p, int b, int y, int x, int c) {
    const TI* img = (const TI*)p.img;
    if (p.layout == YXH_NCHW) return to_f32(img[(((long long)b * 3 + c) * p.H + y) * p.W + x]);
    return to_f32(img[(((long long)b * p.H + y) * p.W + x) * 3 + c]);
}

template <typename T, typename TI, int FR>
__global__ __launch_bounds__(256) void stem_conv(StemParams p) {
    constexpr int EPC = Chunk<T>::N;
    constexpr int SLABS = kStemK / (4 * EPC);  // 64-byte slabs per kernel row: 1 (bf16/f16), 2 (f32)
    constexpr int IN_BYTES = kStemRows * kStemRowElems * sizeof(T);
    constexpr int OUT_ROW = FR * 16 * sizeof(T) + 16;
    constexpr int OUT_BYTES = kStemTY * kStemTX * OUT_ROW;
    constexpr int SMEM = IN_BYTES > OUT_BYTES ? IN_BYTES : OUT_BYTES;
    __shared__ __attribute__((aligned(16))) char smem[SMEM];
    T* in = (T*)smem;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.z;
    const int oy0 = blockIdx.y * kStemTY, ox0 = blockIdx.x * kStemTX;
    const int y0 = 2 * oy0 - 2, x0 = 2 * ox0 - 2;
    // stage the input rows (zero padded) as T
    for (int q = tid; q < kStemRows * kStemRowElems; q += 256) {
        const int r = q / kStemRowElems, e = q - r * kStemRowElems;
        const int y = y0 + r, x = x0 + e / 3, c = e - (e / 3) * 3;
        float v = 0.0f;
        if (e < (2 * kStemTX + 4) * 3 && y >= 0 && y < p.H && x >= 0 && x < p.W) v = load_px<TI>(p, b, y, x, c);
        in[q] = from_f32<T>(v);
    }
    __syncthreads();

    f32x4 acc[FR][4];
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int frow = lane & 15, fq = lane >> 4;
    const T* wt = (const T*)p.w;
#pragma unroll
    for (int ky = 0; ky < 6; ++ky) {
        const T* inrow = in + (2 * wave + ky) * kStemRowElems;
#pragma unroll
        for (int s = 0; s < SLABS; ++s) {
            const int koff = s * 4 * EPC + fq * EPC;  // this lane's K chunk within the row
            uint4 af[FR], bf[4];
#pragma unroll
            for (int i = 0; i < FR; ++i) {
                const int n = i * 16 + frow;
                af[i] = *(const uint4*)(wt + ((long long)n * 6 + ky) * kStemK + koff);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int oxl = j * 16 + frow;
                const unsigned* src = (const unsigned*)(inrow + 6 * oxl + koff);  // 4-byte aligned
                bf[j] = make_uint4(src[0], src[1], src[2], src[3]);
            }
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) Mma<T>::run(acc[i][j], af[i], bf[j]);
        }
    }
    __syncthreads();  // input tile dead; reuse LDS for the output tile
    // epilogue: bias + act in registers, tile [4*64 px][FR*16 ch] through LDS
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int pl = wave * kStemTX + j * 16 + frow;
#pragma unroll
        for (int i = 0; i < FR; ++i) {
            const int n = i * 16 + fq * 4;
            T t[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = acc[i][j][r] + (n + r < p.cout ? p.bias[n + r] : 0.0f);
                t[r] = from_f32<T>(apply_act<sizeof(T) == 4>(v, p.act));
            }
            char* d = smem + pl * OUT_ROW + n * sizeof(T);
            if constexpr (sizeof(T) == 2) {
                uint2 u;
                __builtin_memcpy(&u, t, 8);
                *(uint2*)d = u;
            } else {
                uint4 u;
                __builtin_memcpy(&u, t, 16);
                *(uint4*)d = u;
            }
        }
    }
    __syncthreads();
    const int cpo = p.cout * (int)sizeof(T) / 16;  // chunks per output pixel (cout*es % 16 == 0)
    for (int q = tid; q < kStemTY * kStemTX * cpo; q += 256) {
        const int px = q / cpo, c = q - px * cpo;
        const int oy = oy0 + px / kStemTX, ox = ox0 + (px % kStemTX);
        if (oy >= p.OH || ox >= p.OW) continue;
        const uint4 u = *(const uint4*)(smem + px * OUT_ROW + c * 16);
        *(uint4*)((char*)p.dst + (b * p.dst_bs + ((long long)oy * p.OW + ox) * p.dst_cs) * sizeof(T) + c * 16) = u;
    }
}

// ---------------------------------------------------------------- full-row strips
// Block = 4 output rows x the whole output width of one image.  The 12 input rows are
// staged once with 16-byte loads of whole NHWC image rows (pixel x at element 8 + 3x,
// zeros around it), the weights stay in registers, and each wave (= one output row)
// walks its row in 64-pixel chunks, staging each chunk's outputs in its own LDS area
// and writing them back as 16-byte chunks of whole pixel rows.
constexpr int kStripPx = 64;

__host__ __device__ constexpr int strip_row_elems(int W) { return (8 + 3 * W + 32 + 7) / 8 * 8; }

static size_t strip_lds(int W, int fr, int es) {
    return (size_t)kStemRows * strip_row_elems(W) * es + (size_t)4 * kStripPx * (fr * 16 * es + 16);
}

template <typename T, typename TI, int FR>
__global__ __launch_bounds__(256) void stem_rows(StemParams p) {
    constexpr int EPC = Chunk<T>::N;
    constexpr int SLABS = kStemK / (4 * EPC);
    constexpr int OUT_ROW = FR * 16 * sizeof(T) + 16;
    constexpr int TIN = 16 / sizeof(TI);  // image elements per 16-byte load
    constexpr int BATCH = 8;               // loads in flight per thread
    extern __shared__ __attribute__((aligned(16))) char smem_dyn[];
    const int RE = strip_row_elems(p.W);
    T* in = (T*)smem_dyn;
    char* stage = smem_dyn + (size_t)kStemRows * RE * sizeof(T);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.y, oy0 = blockIdx.x * kStemTY, y0 = 2 * oy0 - 2;
    const int frow = lane & 15, fq = lane >> 4;

    // weights and bias into registers first: their latency overlaps the row staging
    const T* wt = (const T*)p.w;
    uint4 wreg[6][SLABS][FR];
#pragma unroll
    for (int ky = 0; ky < 6; ++ky)
#pragma unroll
        for (int s = 0; s < SLABS; ++s)
#pragma unroll
            for (int i = 0; i < FR; ++i)
                wreg[ky][s][i] =
                    *(const uint4*)(wt + ((long long)(i * 16 + frow) * 6 + ky) * kStemK + s * 4 * EPC + fq * EPC);
    float bias[FR][4];
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = i * 16 + fq * 4 + r;
            bias[i][r] = n < p.cout ? p.bias[n] : 0.0f;
        }

    // zero borders ([0, 8) and [8 + 3W, RE) of every row) and the rows outside the image
    const T z = from_f32<T>(0.0f);
    const int tail0 = 8 + 3 * p.W;
    for (int r = wave; r < kStemRows; r += 4) {
        T* row = in + r * RE;
        const int y = y0 + r;
        if (y < 0 || y >= p.H) {
            for (int e = lane; e < RE; e += 64) row[e] = z;
        } else {
            if (lane < 8) row[lane] = z;
            for (int e = tail0 + lane; e < RE; e += 64) row[e] = z;
        }
    }
    // interiors: the block's rows inside the image are contiguous in memory
    const int cpr = 3 * p.W / TIN;  // 16-byte chunks per image row
    const int rlo = max(0, -y0), rhi = min(kStemRows, p.H - y0);
    const int total = (rhi - rlo) * cpr;
    const TI* img = (const TI*)p.img + ((long long)b * p.H + y0 + rlo) * p.W * 3;
    for (int q0 = 0; q0 < total; q0 += 256 * BATCH) {
        uint4 v[BATCH];
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
            const int q = q0 + k * 256 + tid;
            v[k] = q < total ? *(const uint4*)(img + (long long)q * TIN) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < BATCH; ++k) {
            const int q = q0 + k * 256 + tid;
            if (q >= total) continue;
            const int rr = q / cpr, c = q - rr * cpr;
            TI s[TIN];
            __builtin_memcpy(s, &v[k], 16);
            T t[TIN];
#pragma unroll
            for (int e = 0; e < TIN; ++e) t[e] = from_f32<T>(to_f32(s[e]));
            char* d = (char*)(in + (rlo + rr) * RE + 8 + c * TIN);
            if constexpr (TIN * sizeof(T) >= 16) {
#pragma unroll
                for (int u = 0; u < (int)(TIN * sizeof(T) / 16); ++u) {
                    uint4 w4;
                    __builtin_memcpy(&w4, (const char*)t + 16 * u, 16);
                    ((uint4*)d)[u] = w4;
                }
            } else {
                uint2 w2;
                __builtin_memcpy(&w2, t, 8);
                *(uint2*)d = w2;
            }
        }
    }
    __syncthreads();

    const int cpo = p.cout * (int)sizeof(T) / 16;
    const int oy = oy0 + wave;
    const T* rows0 = in + 2 * wave * RE + 2;  // kernel row 0 of this wave's output row; pixel ox at +6*ox
    char* wst = stage + wave * kStripPx * OUT_ROW;
    for (int ox0 = 0; ox0 < p.OW; ox0 += kStripPx) {
        f32x4 acc[FR][4];
#pragma unroll
        for (int i = 0; i < FR; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ky = 0; ky < 6; ++ky) {
            const T* inrow = rows0 + ky * RE;
#pragma unroll
            for (int s = 0; s < SLABS; ++s) {
                const int koff = s * 4 * EPC + fq * EPC;
                uint4 bf[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int ox = min(ox0 + j * 16 + frow, p.OW - 1);
                    const unsigned* src = (const unsigned*)(inrow + 6 * ox + koff);  // 4-byte aligned
                    bf[j] = make_uint4(src[0], src[1], src[2], src[3]);
                }
#pragma unroll
                for (int i = 0; i < FR; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) Mma<T>::run(acc[i][j], wreg[ky][s][i], bf[j]);
            }
        }
        // bias + act -> this wave's staging tile [64 px][FR*16 ch]
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int pl = j * 16 + frow;
#pragma unroll
            for (int i = 0; i < FR; ++i) {
                const int n = i * 16 + fq * 4;
                T t[4];
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    t[r] = from_f32<T>(apply_act<sizeof(T) == 4>(acc[i][j][r] + bias[i][r], p.act));
                uint2 u;
                __builtin_memcpy(&u, t, 8);
                *(uint2*)(wst + pl * OUT_ROW + n * sizeof(T)) = u;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (oy < p.OH) {
            for (int q = lane; q < kStripPx * cpo; q += 64) {
                const int px = q / cpo, c = q - px * cpo;
                const int ox = ox0 + px;
                if (ox >= p.OW) continue;
                const uint4 u = *(const uint4*)(wst + px * OUT_ROW + c * 16);
                *(uint4*)((char*)p.dst + (b * p.dst_bs + ((long long)oy * p.OW + ox) * p.dst_cs) * sizeof(T) +
                          c * 16) = u;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
}

// Pack the Focus-stem BaseConv (weight [cout][12][3][3] with BN) to [cout_pad][6][32].
template <typename T>
__global__ void stem_pack(const float* w, const float* g, const float* beta, const float* mean, const float* var,
                          float eps, int cout, int cout_pad, T* wo, float* bo) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= cout_pad * 6 * kStemK) return;
    const int e = idx % kStemK, ky6 = (idx / kStemK) % 6, n = idx / (6 * kStemK);
    float v = 0.0f;
    if (n < cout && e < 18) {
        const int kx6 = e / 3, c = e - kx6 * 3;
        const int ky3 = ky6 >> 1, dy = ky6 & 1, kx3 = kx6 >> 1, dx = kx6 & 1;
        const int q = dy + 2 * dx;  // Focus order TL, BL, TR, BR
        const float scale = g ? g[n] / sqrtf(var[n] + eps) : 1.0f;
        v = w[((n * 12 + q * 3 + c) * 3 + ky3) * 3 + kx3] * scale;
    }
    wo[idx] = from_f32<T>(v);
    if (idx < cout_pad) {
        const float scale = g && idx < cout ? g[idx] / sqrtf(var[idx] + eps) : 1.0f;
        bo[idx] = idx < cout && g ? beta[idx] - mean[idx] * scale : 0.0f;
    }
}

template <typename T, typename TI, int FR>
static int launch_strip(const StemParams& p, hipStream_t st) {
    const size_t lds = strip_lds(p.W, FR, sizeof(T));
    (void)hipFuncSetAttribute((const void*)stem_rows<T, TI, FR>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    hipLaunchKernelGGL((stem_rows<T, TI, FR>), dim3((p.OH + kStemTY - 1) / kStemTY, p.B), dim3(256), lds, st, p);
    YXH_CHECK_LAUNCH("stem_rows launch");
    return YXH_OK;
}

template <typename T, typename TI>
static int launch_ti(const StemParams& p, hipStream_t st) {
    const int fr = (p.cout + 15) / 16;
    if constexpr (sizeof(T) == 2) {
        if (p.layout == YXH_NHWC && !p.force_tiles && (3 * p.W * (int)sizeof(TI)) % 16 == 0 &&
            ((uintptr_t)p.img % 16) == 0 && fr <= 5 && strip_lds(p.W, fr, sizeof(T)) <= 160 * 1024) {
            switch (fr) {
                case 1: return launch_strip<T, TI, 1>(p, st);
                case 2: return launch_strip<T, TI, 2>(p, st);
                case 3: return launch_strip<T, TI, 3>(p, st);
                case 4: return launch_strip<T, TI, 4>(p, st);
                default: return launch_strip<T, TI, 5>(p, st);
            }
        }
    }
    dim3 grid((p.OW + kStemTX - 1) / kStemTX, (p.OH + kStemTY - 1) / kStemTY, p.B);
    switch (fr) {
        case 1: hipLaunchKernelGGL((stem_conv<T, TI, 1>), grid, dim3(256), 0, st, p); break;
        case 2: hipLaunchKernelGGL((stem_conv<T, TI, 2>), grid, dim3(256), 0, st, p); break;
        case 3: hipLaunchKernelGGL((stem_conv<T, TI, 3>), grid, dim3(256), 0, st, p); break;
        case 4: hipLaunchKernelGGL((stem_conv<T, TI, 4>), grid, dim3(256), 0, st, p); break;
        case 5: hipLaunchKernelGGL((stem_conv<T, TI, 5>), grid, dim3(256), 0, st, p); break;
        default: set_error("stem cout %d > 80", p.cout); return YXH_EUNSUPPORTED;
    }
    YXH_CHECK_LAUNCH("stem_conv launch");
    return YXH_OK;
}

template <typename T>
static int launch_t(const StemParams& p, hipStream_t st) {
    switch (p.idt) {
        case YXH_F32: return launch_ti<T, float>(p, st);
        case YXH_U8: return launch_ti<T, uint8_t>(p, st);
        case YXH_BF16: return launch_ti<T, bf16>(p, st);
        case YXH_F16: return launch_ti<T, f16>(p, st);
        default: set_error("stem image dtype %d", p.idt); return YXH_EINVAL;
    }
}

int stem_launch(const yxh_stem_desc* d, hipStream_t st) {
    YXH_CHECK_ARG(d && d->img && d->weight && d->bias && d->dst, "null pointer");
    YXH_CHECK_ARG(d->batch > 0 && d->h >= 2 && d->w >= 2 && d->h % 2 == 0 && d->w % 2 == 0, "image %dx%d", d->h,
                  d->w);
    YXH_CHECK_ARG(d->layout == YXH_NCHW || d->layout == YXH_NHWC, "layout");
    const int es = d->dtype == YXH_F32 ? 4 : 2;
    YXH_CHECK_ARG(d->dtype == YXH_F32 || d->dtype == YXH_BF16 || d->dtype == YXH_F16, "dtype");
    YXH_CHECK_ARG(d->cout > 0 && d->cout <= 80 && (d->cout * es) % 16 == 0, "stem cout %d", d->cout);
    YXH_CHECK_ARG(((uintptr_t)d->dst % 16) == 0 && (d->dst_cstride * es) % 16 == 0 && (d->dst_bstride * es) % 16 == 0,
                  "stem dst alignment");
    StemParams p;
    p.img = d->img;
    p.layout = d->layout;
    p.idt = d->img_dtype;
    p.B = d->batch;
    p.H = d->h;
    p.W = d->w;
    p.OH = d->h / 2;
    p.OW = d->w / 2;
    p.cout = d->cout;
    p.act = d->act;
    p.w = d->weight;
    p.bias = d->bias;
    p.dst = d->dst;
    p.dst_cs = d->dst_cstride;
    p.dst_bs = d->dst_bstride;
    p.force_tiles = d->reserved == 1;
    if (d->dtype == YXH_BF16) return launch_t<bf16>(p, st);
    if (d->dtype == YXH_F16) return launch_t<f16>(p, st);
    return launch_t<float>(p, st);
}

int stem_pack_launch(const float* w, const float* g, const float* beta, const float* mean, const float* var,
                     float eps, int cout, int dt, void* wo, float* bo, hipStream_t st) {
    YXH_CHECK_ARG(w && wo && bo && cout > 0 && cout <= 80, "stem pack");
    YXH_CHECK_ARG(!g || (beta && mean && var), "partial BN parameters");
    const int cout_pad = (cout + 15) / 16 * 16;
    const int total = cout_pad * 6 * kStemK;
    dim3 grid((total + 255) / 256);
    if (dt == YXH_BF16)
        hipLaunchKernelGGL(stem_pack<bf16>, grid, dim3(256), 0, st, w, g, beta, mean, var, eps, cout, cout_pad,
                           (bf16*)wo, bo);
    else if (dt == YXH_F16)
        hipLaunchKernelGGL(stem_pack<f16>, grid, dim3(256), 0, st, w, g, beta, mean, var, eps, cout, cout_pad,
                           (f16*)wo, bo);
    else if (dt == YXH_F32)
        hipLaunchKernelGGL(stem_pack<float>, grid, dim3(256), 0, st, w, g, beta, mean, var, eps, cout, cout_pad,
                           (float*)wo, bo);
    else {
        set_error("stem pack dtype %d", dt);
        return YXH_EINVAL;
    }
    YXH_CHECK_LAUNCH("stem pack");
    return YXH_OK;
}

}  // namespace yxh
