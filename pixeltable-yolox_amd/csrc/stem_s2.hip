// Fused Focus stem + first stride-2 3x3 conv on gfx950 (reference darknet.py:112-123:
// stem = Focus(3, C1, ksize=3) = space-to-depth + BaseConv(4*3 -> C1, 3x3 s1), then
// dark2[0] = BaseConv(C1 -> 2*C1, 3x3 s2); network_blocks.py:27-52, 186-208).
//
// The unfused forms write the C1-channel stem map at H/2 x W/2 (yolox_s @640 bs32: 210 MB)
// and read it back for the stride-2 conv.  Here one persistent block computes a 16 x 8 tile
// of the stride-2 conv's output directly from the image:
//   1. the image patch the tile needs (38 rows x 70 pixels x 3 channels, zero outside the
//      image) arrives by buffer loads issued one tile ahead into registers (groups of 4
//      pixels) and is written to LDS as RGB0 pixels of 8 bytes;
//   2. the stem conv over the 17 x 33 stem pixels the stride-2 conv reads.  Focus + 3x3 is
//      a 6x6 stride-2 conv on the image (stem.hip); one kernel row of it is 6 RGB0 pixels =
//      24 contiguous LDS values = three 16-byte K chunks, so K = 6 x 24 = 144 (108 real,
//      5 MFMA slabs) and every B fragment is one aligned ds_read_b128 -- bias + SiLU, zeros
//      outside the stem map (the stride-2 conv's zero padding), into a second LDS image laid
//      out as conv_ws's stride-2 halo (5 16-byte slots per pixel: conflict-free reads);
//   3. the stride-2 conv (K = 9 taps x C1) from that image with weights stationary in VGPRs,
//      bias + SiLU, 8-byte stores of 4 channels;
//   4. (CSP form, round 4) instead of storing the stride-2 map: dark2's CspLayer conv1 | conv2
//      (network_blocks.py:176-178, a 1x1 64 -> 64) over it from LDS, stored as whole pixel
//      rows, and its first Bottleneck's conv1 (network_blocks.py:95-96, 1x1 32 -> 32) over the
//      x_1 half -- the 64-channel map at H/4 x W/4 never reaches HBM (yolox_s @640 bs32: 105 MB
//      written + read, and two launches).
// Two blocks per CU: one block's image loads / barriers overlap the other's MFMAs.
#include <algorithm>

#include "conv_common.hpp"
#include "lds_dma.hpp"

namespace yxh {

struct Stem2Params {
    const void* img;
    int B, H, W, OH1, OW1, OH, OW;
    const void* w1;  // yxh_stem_pack layout [round16(C1)][6][32]: ky6, kx6 * 3 + c
    const float* b1;
    const void* w2;  // [C2][9][C1]
    const float* b2;
    void* dst;
    int dst_cs;
    long long dst_bs;
    int act1, act2;
    // CSP form (yxh_stem2_desc.w3 set): the stride-2 output Y stays in LDS; Z3 = SiLU(W3 . Y + b3)
    // (dark2's CspLayer conv1 | conv2, c2 -> c2) leaves to dst3 and, with w4, T = SiLU(W4 .
    // Z3[:, :c2/2] + b4) (its first Bottleneck's conv1, c2/2 -> c2/2) to dst4
    const void* w3;
    const float* b3;
    void* dst3;
    int dst3_cs;
    long long dst3_bs;
    const void* w4;
    const float* b4;
    void* dst4;
    int dst4_cs;
    long long dst4_bs;
};

namespace {

constexpr int kS2TX = 16, kS2TY = 8;                       // output tile of the stride-2 conv
constexpr int kS2SX = 2 * kS2TX + 1, kS2SY = 2 * kS2TY + 1;  // stem pixels the tile needs
constexpr int kS2IY = 4 * kS2TY + 6, kS2IX = 4 * kS2TX + 6;  // image rows / pixels of the patch
constexpr int kS2G = (kS2IX + 3) / 4;                       // 4-pixel groups per patch row (18)
constexpr int kS2IXP = 4 * kS2G;                            // LDS pixels per patch row (72)
constexpr int kS2NSP = kS2SX * kS2SY;                       // 561 stem pixels
constexpr int kS2NF1 = (kS2NSP + 15) / 16;                  // 36 stem pixel fragments
constexpr int kS2FBYTES = kS2IY * kS2IXP * 8;               // RGB0 image patch (21.9 KB)

// element q of a group of 4 RGB pixels (12 image values) held in 12 / (4 / sizeof(TI)) dwords
template <typename T, typename TI>
__device__ __forceinline__ T group_elem(const uint32_t* w, int q) {
    if constexpr (sizeof(TI) == 1) {
        return from_f32<T>((float)((w[q >> 2] >> (8 * (q & 3))) & 0xffu));
    } else {
        const uint32_t v = w[q >> 1] >> (16 * (q & 1));
        const uint16_t h = (uint16_t)v;
        TI x;
        __builtin_memcpy(&x, &h, 2);
        return from_f32<T>(to_f32(x));
    }
}

}  // namespace

template <typename T, typename TI, int C1, bool CSP>
__global__ __launch_bounds__(256, 2) void stem_s2(Stem2Params p, int tiles_x, int tiles_y, int ntiles) {
    static_assert(sizeof(T) == 2, "16-bit compute");
    static_assert(C1 == 32, "stem width");
    constexpr int C2 = 2 * C1;
    constexpr int GDW = 3 * (int)sizeof(TI);       // dwords per 4-pixel group (12 values)
    constexpr int NGR = kS2IY * kS2G;              // groups per patch (684)
    constexpr int NPT = (NGR + 255) / 256;         // groups per thread
    constexpr int HXP = kS2SX, PS = 5, PSB = PS * 16;  // stem image: conv_ws stride-2 halo layout
    constexpr int SBYTES = kS2SY * HXP * PSB;
    constexpr int FR2 = 2, FC2 = 4;                // stride-2 conv: 2 waves x 32 channels, 2 waves x 64 pixels
    static_assert(C2 == 2 * 16 * FR2 && kS2TX * kS2TY == 2 * 16 * FC2, "wave tiling");
    // CSP form: Y [128 px][C2] in the image patch's place (free once the stem stage has read
    // it), Z3 [128 px][C2] in the stem image's place (free once the stride-2 conv has read it);
    // rows of C2 / 8 + 1 16-byte slots (odd: the 16 rows of a fragment read hit distinct banks).
    // The 1x1 weights and biases live in LDS (the VGPRs hold the two stationary conv weights):
    // W3 [C2][C2] and W4 [C2/2][C2/2] with the same odd-slot rows, then b3, b4.
    constexpr int ZRS = (C2 / 8 + 1) * 16, W4RS = (C2 / 16 + 1) * 16;
    constexpr int WBYTES = CSP ? C2 * ZRS + (C2 / 2) * W4RS + (C2 + C2 / 2) * 4 : 0;
    static_assert(kS2TX * kS2TY * ZRS <= kS2FBYTES && kS2TX * kS2TY * ZRS <= SBYTES, "CSP staging");
    __shared__ __attribute__((aligned(16))) char smem[kS2FBYTES + SBYTES + WBYTES];
    char* fimg = smem;
    char* simg = smem + kS2FBYTES;
    char* ybuf = fimg;
    char* zbuf = simg;
    char* w3l = smem + kS2FBYTES + SBYTES;
    char* w4l = w3l + C2 * ZRS;
    float* b3l = (float*)(w4l + (C2 / 2) * W4RS);
    float* b4l = b3l + C2;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int frow = lane & 15, fq = lane >> 4;
    const int wn = wave & 1, wm = wave >> 1;

    // ---- stationary weights
    // stem A fragments, K = ky * 24 + kx * 4 + c (c = 3 and k >= 144 are zero), from the
    // yxh_stem_pack rows [6][32] (ky, kx * 3 + c)
    const T* w1 = (const T*)p.w1;
    uint4 a1[2][5];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int s = 0; s < 5; ++s) {
            T t[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = 32 * s + 8 * fq + e;
                const int ky = k / 24, kx = (k % 24) >> 2, c = k & 3;
                t[e] = (k < 144 && c < 3) ? w1[((i * 16 + frow) * 6 + ky) * 32 + kx * 3 + c] : from_f32<T>(0.0f);
            }
            __builtin_memcpy(&a1[i][s], t, 16);
        }
    const T* w2 = (const T*)p.w2;
    uint4 a2[FR2][9];
#pragma unroll
    for (int i = 0; i < FR2; ++i)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
            a2[i][tap] = *(const uint4*)(w2 + ((wn * 32 + i * 16 + frow) * 9 + tap) * C1 + fq * 8);
    float bias1[2][4], bias2[FR2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) bias1[i][r] = p.b1[i * 16 + fq * 4 + r];
#pragma unroll
    for (int i = 0; i < FR2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) bias2[i][r] = p.b2[wn * 32 + i * 16 + fq * 4 + r];
    // CSP form: the 1x1 weights / biases -> LDS once (wave w later owns Z3 channels 16 w .. +16,
    // K = C2 in two 32-deep blocks, and T channels 16 (w & 1) .. +16 of pixel fragments
    // 4 (w >> 1) .. +4, K = C2 / 2 in one block); made visible by the first tile's barriers
    const bool has4 = CSP && p.w4 != nullptr;
    if constexpr (CSP) {
        static_assert(C2 == 64, "CSP form: 64 -> 64 (+ 32 -> 32)");
        for (int q = tid; q < C2 * C2 / 8; q += 256) {
            const int r = q / (C2 / 8), c = q - (C2 / 8) * (q / (C2 / 8));
            *(uint4*)(w3l + r * ZRS + c * 16) = *(const uint4*)((const T*)p.w3 + r * C2 + c * 8);
        }
        if (tid < C2) b3l[tid] = p.b3[tid];
        if (has4) {
            for (int q = tid; q < (C2 / 2) * (C2 / 2) / 8; q += 256) {
                const int r = q / (C2 / 16), c = q - (C2 / 16) * (q / (C2 / 16));
                *(uint4*)(w4l + r * W4RS + c * 16) = *(const uint4*)((const T*)p.w4 + r * (C2 / 2) + c * 8);
            }
            if (tid < C2 / 2) b4l[tid] = p.b4[tid];
        }
    }

    // ---- per-lane stem K-chunk offsets (bytes from a stem pixel's base in the RGB0 patch):
    // chunk k0 = 32 s + 8 fq = kernel row k0 / 24, pixels (k0 % 24) / 4 .. +1; k0 >= 144 is
    // weight padding and re-reads a real chunk (finite values)
    uint32_t off1[5];
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        int k = 32 * s + 8 * fq;
        if (k >= 144) k = 136;
        off1[s] = (uint32_t)(((k / 24) * kS2IXP + (k % 24) / 4) * 8);
    }

    const int W3 = p.W * 3;
    const uint32_t ibytes = (uint32_t)((long long)p.H * W3 * sizeof(TI));
    const unsigned txy = (unsigned)(tiles_x * tiles_y);
    struct TileC { int b, oy0, ox0; };
    auto coords = [&](int t) -> TileC {
        const unsigned b = (unsigned)t / txy, r = (unsigned)t - b * txy;
        const unsigned ty = r / (unsigned)tiles_x, tx = r - ty * (unsigned)tiles_x;
        return TileC{(int)b, (int)ty * kS2TY, (int)tx * kS2TX};
    };
    uint32_t img[NPT][GDW];
    auto load_image = [&](const TileC& c) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)((const TI*)p.img + (long long)c.b * p.H * W3), (short)0, (int)ibytes, 0x00020000);
        const int iy0 = 4 * c.oy0 - 4, ix0 = 4 * c.ox0 - 4;
#pragma unroll
        for (int t = 0; t < NPT; ++t) {
            const int g = tid + 256 * t;
            const int row = g / kS2G, gc = g - kS2G * (g / kS2G);
            const int iy = iy0 + row, ix = ix0 + 4 * gc;
            // a group (4 pixels, W % 4 == 0, ix % 4 == 0) is wholly inside the image or outside
            const bool ok = g < NGR && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
            const int voff = ok ? (iy * W3 + ix * 3) * (int)sizeof(TI) : (int)dma::kOob;
#pragma unroll
            for (int d = 0; d < GDW; ++d) img[t][d] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff + 4 * d, 0, 0);
        }
    };
    auto store_image = [&]() {
#pragma unroll
        for (int t = 0; t < NPT; ++t) {
            const int g = tid + 256 * t;
            if (g >= NGR) continue;
            const int row = g / kS2G, gc = g - kS2G * (g / kS2G);
            char* d = fimg + (row * kS2IXP + 4 * gc) * 8;
#pragma unroll
            for (int px = 0; px < 4; ++px) {
                uint2 u;
                if constexpr (sizeof(TI) == 1 && __is_same(T, bf16)) {
                    // integers 0..255 are exact in bf16: the f32's upper half IS the bf16 value
                    const float r = (float)((img[t][(3 * px) >> 2] >> (8 * ((3 * px) & 3))) & 0xffu);
                    const float g = (float)((img[t][(3 * px + 1) >> 2] >> (8 * ((3 * px + 1) & 3))) & 0xffu);
                    const float b = (float)((img[t][(3 * px + 2) >> 2] >> (8 * ((3 * px + 2) & 3))) & 0xffu);
                    u.x = __builtin_amdgcn_perm(__float_as_uint(g), __float_as_uint(r), 0x07060302u);
                    u.y = __float_as_uint(b) >> 16;
                } else {
                    T t4[4] = {group_elem<T, TI>(img[t], 3 * px), group_elem<T, TI>(img[t], 3 * px + 1),
                               group_elem<T, TI>(img[t], 3 * px + 2), from_f32<T>(0.0f)};
                    __builtin_memcpy(&u, t4, 8);
                }
                *(uint2*)(d + px * 8) = u;
            }
        }
    };

    const int bid = dma::xcd_remap(blockIdx.x, gridDim.x);
    int tile = bid;
    if (tile >= ntiles) return;  // block-uniform
    TileC cur = coords(tile);
    load_image(cur);
    for (; tile < ntiles; tile += gridDim.x) {
        store_image();
        // image patch complete; every wave is past the last tile's conv stage (LDS only: the
        // image loads for the next tile stay in flight across the barrier)
        dma::barrier();
        const int next = tile + gridDim.x;
        TileC nc = cur;
        if (next < ntiles) {
            nc = coords(next);
            load_image(nc);  // lands during this tile's two GEMMs
        }

        // per-lane geometry below derives from an opaque copy of the lane ids, so it is
        // recomputed per tile instead of being hoisted out of the loop into (spilled) VGPRs
        int frow_o = frow;
        asm volatile("" : "+v"(frow_o));
        // a tile whose stem halo lies inside the stem map needs no zero-padding selects
        const bool interior = 2 * cur.oy0 - 1 >= 0 && 2 * cur.ox0 - 1 >= 0 && 2 * cur.oy0 + 2 * kS2TY - 1 < p.OH1 &&
                              2 * cur.ox0 + 2 * kS2TX - 1 < p.OW1;
        // ---- stem: 36 fragments of 16 stem pixels, wave w takes w, w + 4, ... (3 at a time)
#pragma unroll
        for (int g0 = 0; g0 < kS2NF1 / 4; g0 += 3) {
            f32x4 acc[2][3];
            uint32_t pb[3];
#pragma unroll
            for (int jj = 0; jj < 3; ++jj) {
                const int pix = min((wave + 4 * (g0 + jj)) * 16 + frow_o, kS2NSP - 1);
                const int sy = pix / kS2SX, sx = pix - kS2SX * (pix / kS2SX);
                pb[jj] = (uint32_t)((2 * sy * kS2IXP + 2 * sx) * 8);
#pragma unroll
                for (int i = 0; i < 2; ++i) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int s = 0; s < 5; ++s) {
                uint4 b[3];
#pragma unroll
                for (int jj = 0; jj < 3; ++jj) b[jj] = *(const uint4*)(fimg + pb[jj] + off1[s]);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int jj = 0; jj < 3; ++jj) Mma<T>::run(acc[i][jj], a1[i][s], b[jj]);
            }
            // bias + SiLU; zeros outside the stem map (the stride-2 conv's padding)
#pragma unroll
            for (int jj = 0; jj < 3; ++jj) {
                const int pix = (wave + 4 * (g0 + jj)) * 16 + frow_o;
                const int sy = pix / kS2SX, sx = pix - kS2SX * (pix / kS2SX);
                const int gy = 2 * cur.oy0 - 1 + sy, gx = 2 * cur.ox0 - 1 + sx;
                const bool valid = interior || ((unsigned)gy < (unsigned)p.OH1 && (unsigned)gx < (unsigned)p.OW1);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const f32x4 y =
                        yxh::silu4(acc[i][jj] + f32x4{bias1[i][0], bias1[i][1], bias1[i][2], bias1[i][3]});
                    // two paired conversions, then the zero padding selected on the packed pairs (a 16-bit +0
                    // is all-zero bits, as from_f32(0.0f)): selecting before converting made the compiler
                    // convert each value alone and re-pack the halves (10 VALU per 4 values instead of 4)
                    uint2 u = pack4<T>(y);
                    u.x = valid ? u.x : 0u;
                    u.y = valid ? u.y : 0u;
                    if (pix < kS2NSP) *(uint2*)(simg + (sy * HXP + sx) * PSB + (i * 16 + fq * 4) * 2) = u;
                }
            }
        }
        dma::barrier();  // stem image complete

        // ---- stride-2 conv: wave (wn, wm) = 32 channels x 64 pixels of the 16 x 8 tile
        f32x4 acc2[FR2][FC2];
        uint32_t boff[FC2];
#pragma unroll
        for (int j = 0; j < FC2; ++j) {
            const int pl = (wm * FC2 + j) * 16 + frow_o;
            const int ty = pl / kS2TX, tx = pl - kS2TX * (pl / kS2TX);
            boff[j] = (uint32_t)(((2 * ty) * HXP + 2 * tx) * PSB + fq * 16);
#pragma unroll
            for (int i = 0; i < FR2; ++i) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int ky = tap / 3, kx = tap - 3 * (tap / 3);
            const uint32_t so = (uint32_t)((ky * HXP + kx) * PSB);
            uint4 b[FC2];
#pragma unroll
            for (int j = 0; j < FC2; ++j) b[j] = *(const uint4*)(simg + boff[j] + so);
#pragma unroll
            for (int i = 0; i < FR2; ++i)
#pragma unroll
                for (int j = 0; j < FC2; ++j) Mma<T>::run(acc2[i][j], a2[i][tap], b[j]);
        }
        if constexpr (!CSP) {
            T* dst = (T*)p.dst + (long long)cur.b * p.dst_bs;
#pragma unroll
            for (int j = 0; j < FC2; ++j) {
                const int pl = (wm * FC2 + j) * 16 + frow;
                const int ty = pl / kS2TX, tx = pl - kS2TX * (pl / kS2TX);
                const int oy = cur.oy0 + ty, ox = cur.ox0 + tx;
                if (oy >= p.OH || ox >= p.OW) continue;
#pragma unroll
                for (int i = 0; i < FR2; ++i) {
                    const int n = wn * 32 + i * 16 + fq * 4;
                    const f32x4 y =
                        yxh::silu4(acc2[i][j] + f32x4{bias2[i][0], bias2[i][1], bias2[i][2], bias2[i][3]});
                    T t[4] = {from_f32<T>(y[0]), from_f32<T>(y[1]), from_f32<T>(y[2]), from_f32<T>(y[3])};
                    uint2 u;
                    __builtin_memcpy(&u, t, 8);
                    *(uint2*)(dst + (long long)(oy * p.OW + ox) * p.dst_cs + n) = u;
                }
            }
        } else {
            // ---- Y = SiLU(conv + b2), rounded to T as the unfused path stores it, into LDS
#pragma unroll
            for (int j = 0; j < FC2; ++j) {
                const int pl = (wm * FC2 + j) * 16 + frow;
#pragma unroll
                for (int i = 0; i < FR2; ++i) {
                    const int n = wn * 32 + i * 16 + fq * 4;
                    const f32x4 y =
                        yxh::silu4(acc2[i][j] + f32x4{bias2[i][0], bias2[i][1], bias2[i][2], bias2[i][3]});
                    T t[4] = {from_f32<T>(y[0]), from_f32<T>(y[1]), from_f32<T>(y[2]), from_f32<T>(y[3])};
                    uint2 u;
                    __builtin_memcpy(&u, t, 8);
                    *(uint2*)(ybuf + pl * ZRS + n * 2) = u;
                }
            }
            dma::barrier();  // Y complete; every wave is done reading the stem image
            // ---- Z3 = SiLU(W3 . Y + b3): wave w = channels 16 w .. +16 of all 8 pixel fragments
            constexpr int NPF = kS2TX * kS2TY / 16;
            uint4 a3[2];
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) a3[kb] = *(const uint4*)(w3l + (wave * 16 + frow) * ZRS + (kb * 4 + fq) * 16);
            // two pixel fragments at a time (the stationary conv weights hold most VGPRs)
#pragma unroll 1
            for (int f0 = 0; f0 < NPF; f0 += 2) {
                f32x4 acc3[2];
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    acc3[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int kb = 0; kb < 2; ++kb)
                        Mma<T>::run(acc3[g], a3[kb],
                                    *(const uint4*)(ybuf + ((f0 + g) * 16 + frow) * ZRS + (kb * 4 + fq) * 16));
                }
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    const float* bb = b3l + wave * 16 + fq * 4;
                    const f32x4 y = yxh::silu4(acc3[g] + f32x4{bb[0], bb[1], bb[2], bb[3]});
                    T t[4] = {from_f32<T>(y[0]), from_f32<T>(y[1]), from_f32<T>(y[2]), from_f32<T>(y[3])};
                    uint2 u;
                    __builtin_memcpy(&u, t, 8);
                    *(uint2*)(zbuf + ((f0 + g) * 16 + frow) * ZRS + (wave * 16 + fq * 4) * 2) = u;
                }
            }
            dma::barrier();  // Z3 complete
            // whole 128-byte pixel rows of Z3 leave as 16-byte stores: thread t moves chunk t % 8
            // of tile pixels t / 8 + 32 i.  (The lane indices are recomputed here from an opaque
            // copy of the thread id: hoisted out of the tile loop they would be spilled, and the
            // scratch reloads' vmcnt waits would drain the next tile's image loads.)
            {
                static_assert(C2 / 8 == 8 && kS2TX == 16, "Z3 store mapping");
                int t = tid;
                asm volatile("" : "+v"(t));
                const int c = t & 7, pr = t >> 3;
                T* d3 = (T*)p.dst3 + (long long)cur.b * p.dst3_bs + c * 8;
#pragma unroll
                for (int i = 0; i < kS2TX * kS2TY / 32; ++i) {
                    const int pl = pr + 32 * i;
                    const int oy = cur.oy0 + (pl >> 4), ox = cur.ox0 + (pl & 15);
                    if (oy < p.OH && ox < p.OW)
                        *(uint4*)(d3 + (long long)(oy * p.OW + ox) * p.dst3_cs) = *(const uint4*)(zbuf + pl * ZRS + c * 16);
                }
            }
            // ---- T = SiLU(W4 . Z3[:, :32] + b4): wave w = channels 16 (w & 1) of fragments 4 (w >> 1) ..
            if (has4) {
                T* d4 = (T*)p.dst4 + (long long)cur.b * p.dst4_bs;
                const uint4 a4 = *(const uint4*)(w4l + ((wave & 1) * 16 + frow) * W4RS + fq * 16);
                int fr = frow;
                asm volatile("" : "+v"(fr));
#pragma unroll
                for (int g = 0; g < NPF / 2; ++g) {
                    const int f = (wave >> 1) * (NPF / 2) + g;  // = tile pixel row (kS2TX = 16)
                    const int pl = f * 16 + fr;
                    f32x4 acc4 = f32x4{0.f, 0.f, 0.f, 0.f};
                    Mma<T>::run(acc4, a4, *(const uint4*)(zbuf + pl * ZRS + fq * 16));
                    const int oy = cur.oy0 + f, ox = cur.ox0 + fr;
                    const float* bb = b4l + (wave & 1) * 16 + fq * 4;
                    const f32x4 y = yxh::silu4(acc4 + f32x4{bb[0], bb[1], bb[2], bb[3]});
                    T t[4] = {from_f32<T>(y[0]), from_f32<T>(y[1]), from_f32<T>(y[2]), from_f32<T>(y[3])};
                    uint2 u;
                    __builtin_memcpy(&u, t, 8);
                    if (oy < p.OH && ox < p.OW)
                        *(uint2*)(d4 + (long long)(oy * p.OW + ox) * p.dst4_cs + (wave & 1) * 16 + fq * 4) = u;
                }
            }
        }
        cur = nc;
    }
}

template <typename T, typename TI, bool CSP>
static int launch_s2(const Stem2Params& p, hipStream_t st) {
    const int tiles_x = (p.OW + kS2TX - 1) / kS2TX, tiles_y = (p.OH + kS2TY - 1) / kS2TY;
    const long long ntiles = (long long)tiles_x * tiles_y * p.B;
    if (ntiles >= (1LL << 30)) {
        set_error("stem_s2: too many tiles");
        return YXH_EINVAL;
    }
    const int grid = (int)std::min<long long>(ntiles, 256 * 2);
    hipLaunchKernelGGL((stem_s2<T, TI, 32, CSP>), dim3(grid), dim3(256), 0, st, p, tiles_x, tiles_y, (int)ntiles);
    YXH_CHECK_LAUNCH("stem_s2 launch");
    return YXH_OK;
}

template <typename T>
static int launch_s2_t(int idt, const Stem2Params& p, hipStream_t st) {
    const bool csp = p.w3 != nullptr;
    switch (idt) {
        case YXH_U8: return csp ? launch_s2<T, uint8_t, true>(p, st) : launch_s2<T, uint8_t, false>(p, st);
        case YXH_BF16: return csp ? launch_s2<T, bf16, true>(p, st) : launch_s2<T, bf16, false>(p, st);
        case YXH_F16: return csp ? launch_s2<T, f16, true>(p, st) : launch_s2<T, f16, false>(p, st);
        default: set_error("stem_s2 image dtype %d", idt); return YXH_EINVAL;
    }
}

int stem_s2_launch(const yxh_stem2_desc* d, hipStream_t st) {
    YXH_CHECK_ARG(d && d->img && d->w1 && d->b1 && d->w2 && d->b2 && (d->dst || d->w3), "null pointer");
    YXH_CHECK_ARG(d->layout == YXH_NHWC, "stem_s2 reads NHWC images");
    YXH_CHECK_ARG(d->dtype == YXH_BF16 || d->dtype == YXH_F16, "stem_s2 computes in bf16/f16");
    YXH_CHECK_ARG(d->act == YXH_ACT_SILU, "stem_s2 is built for SiLU (got act %d)", d->act);
    YXH_CHECK_ARG(d->c1 == 32 && d->c2 == 64, "stem_s2 is built for 32 stem / 64 conv channels (got %d/%d)", d->c1,
                  d->c2);
    YXH_CHECK_ARG(d->batch > 0 && d->h >= 4 && d->w >= 4 && d->h % 4 == 0 && d->w % 4 == 0, "image %dx%d", d->h,
                  d->w);
    YXH_CHECK_ARG(d->img_dtype == YXH_U8 || d->img_dtype == YXH_BF16 || d->img_dtype == YXH_F16,
                  "stem_s2 reads u8 / bf16 / f16 images");
    const int es = d->img_dtype == YXH_U8 ? 1 : 2;
    YXH_CHECK_ARG(((uintptr_t)d->img % 4) == 0 && (long long)d->h * d->w * 3 * es < (1LL << 31),
                  "stem_s2 image alignment / size");
    if (!d->w3)
        YXH_CHECK_ARG(((uintptr_t)d->dst % 8) == 0 && d->dst_cstride % 4 == 0 && d->dst_cstride >= 64 &&
                          d->dst_bstride % 4 == 0,
                      "stem_s2 dst alignment");
    if (d->w3) {
        YXH_CHECK_ARG(d->b3 && d->dst3 && ((uintptr_t)d->dst3 % 16) == 0 && d->dst3_cstride % 8 == 0 &&
                          d->dst3_cstride >= 64 && d->dst3_bstride % 8 == 0,
                      "stem_s2 CSP form: dst3 rows must be 16-byte aligned, >= 64 channels");
        YXH_CHECK_ARG(!d->w4 || (d->b4 && d->dst4 && ((uintptr_t)d->dst4 % 8) == 0 && d->dst4_cstride % 4 == 0 &&
                                 d->dst4_cstride >= 32 && d->dst4_bstride % 4 == 0),
                      "stem_s2 CSP form: dst4 alignment");
    }
    Stem2Params p;
    p.img = d->img;
    p.B = d->batch;
    p.H = d->h;
    p.W = d->w;
    p.OH1 = d->h / 2;
    p.OW1 = d->w / 2;
    p.OH = (p.OH1 - 1) / 2 + 1;
    p.OW = (p.OW1 - 1) / 2 + 1;
    p.w1 = d->w1;
    p.b1 = d->b1;
    p.w2 = d->w2;
    p.b2 = d->b2;
    p.dst = d->dst;
    p.dst_cs = d->dst_cstride;
    p.dst_bs = d->dst_bstride;
    p.act1 = d->act;
    p.act2 = d->act;
    p.w3 = d->w3;
    p.b3 = d->b3;
    p.dst3 = d->dst3;
    p.dst3_cs = d->dst3_cstride;
    p.dst3_bs = d->dst3_bstride;
    p.w4 = d->w3 ? d->w4 : nullptr;
    p.b4 = d->b4;
    p.dst4 = d->dst4;
    p.dst4_cs = d->dst4_cstride;
    p.dst4_bs = d->dst4_bstride;
    if (d->dtype == YXH_BF16) return launch_s2_t<bf16>(d->img_dtype, p, st);
    return launch_s2_t<f16>(d->img_dtype, p, st);
}

}  // namespace yxh
