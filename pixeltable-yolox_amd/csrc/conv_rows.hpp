// conv_rows: 3x3 conv (stride 1 or 2, pad 1) with 2D output tiles whose three kx
// taps share one LDS image of the input rows (reference network_blocks.py:48-49
// BaseConv, the 3x3 convs of darknet.py / yolo_pafpn.py / yolo_head.py).
//
// Block = 256 threads (4 waves) computing TN = 64 output channels x a TY x TX tile of
// output pixels of one image.  The K loop runs over (channel block cb, kernel row ky):
// one stage moves, by LDS-DMA (global_load_lds_dwordx4),
//   * A: the 3 taps (ky, 0..2) x TN rows x CH 16-byte chunks of packed weights, in the
//     XOR-swizzled [kx][chunk][row] image of conv_glds;
//   * B: the TY input rows iy = oy*S + ky - 1 that the tile's output rows read, each
//     HX = (TX-1)*S + 3 pixels wide (zero chunk outside the image), stored
//     [pixel][chunk ^ f(pixel)] so 16 consecutive pixels of one chunk hit 16 distinct
//     16-byte bank groups;
// and the three kx taps read the same B image shifted by kx pixels -- 3x fewer B
// bytes than the per-tap im2col of conv.hip, and 3 taps x (TN x TM) MFMA work per
// barrier instead of one.
// The pipeline is a 2- or 3-buffer ring (NBUF): stage k+1 (and k+2) is issued right
// after the barrier that retires stage k and lands while stage k computes.
// TN = 64 (4 waves along pixels) or 128 (2 x 2 waves).  Variants are instantiated per
// dtype in conv_rows_{bf16,f16,f32}.hip so the build parallelises.
#pragma once
#include "conv_common.hpp"

namespace yxh {

namespace {

__device__ __attribute__((aligned(16))) uint4 g_rows_zero[4];

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void raw_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// XCD-aware block order: blocks that the dispatcher places on one XCD (id % 8) get
// consecutive logical ids, so the N tiles and neighbouring pixel tiles that share
// input rows share an L2.  Bijective for any block count.
__device__ __forceinline__ int xcd_remap(int id, int nblk) {
    const int q = nblk / 8, r = nblk % 8, xcd = id % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
}

}  // namespace

template <typename T, int S, int TX, int TY, int CH, int TN, int NBUF>
__global__ __launch_bounds__(256) void conv_rows(ConvParams p, int tiles_x, int tiles_y, int ntn) {
    constexpr int WN = TN / 64, WM = 4 / WN;  // waves: WN along channels (64 each) x WM along pixels
    constexpr int EPC = Chunk<T>::N;
    constexpr int KS = CH / 4;  // 64-byte slabs per stage
    constexpr int KST = CH * EPC;
    constexpr int TM = TX * TY, WTM = TM / WM;
    constexpr int FR = 4, FC = WTM / 16;
    constexpr int HX = (TX - 1) * S + 3;
    constexpr int A_SLOTS = 3 * TN * CH, B_SLOTS = TY * HX * CH;
    constexpr int SLOTS = ((A_SLOTS + B_SLOTS + 255) / 256) * 256;
    constexpr int G = SLOTS / 256;
    constexpr int BUF = SLOTS * 16;
    constexpr int PXG = 16 / CH;  // consecutive pixels per bank row of 16-byte slots
    static_assert(TM % (16 * WM) == 0, "pixel tile must split into 16-pixel fragments per wave");
    static_assert(A_SLOTS % 64 == 0, "a wave's 64 slots must not straddle A and B");
    static_assert(G <= 40, "vmcnt range");
    __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nblk = tiles_x * tiles_y * (p.M / p.ohw) * ntn;
    const int bid = xcd_remap(blockIdx.x, nblk);
    const int nt = bid % ntn;
    int t = bid / ntn;
    const int tx_i = t % tiles_x;
    t /= tiles_x;
    const int ty_i = t % tiles_y;
    const int b = t / tiles_y;
    const int n0 = nt * TN, oy0 = ty_i * TY, ox0 = tx_i * TX;
    const int wr = wave / WM, wc = wave % WM;

    const T* src = (const T*)p.sptr[0] + (long long)b * p.sbs[0];
    const int scs = p.scs[0], sw = p.sw[0];

    auto issue = [&](int k, int buf) {
        const int cb = k / 3, ky = k - cb * 3;
        char* base = smem + buf * BUF;
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const int s = 64 * (wave + 4 * i) + lane;
            const void* g = (const void*)g_rows_zero;
            if (s < A_SLOTS) {
                const int kx = s / (CH * TN), rem = s - kx * (CH * TN);
                const int c = rem / TN, rp = rem - c * TN;
                const int n = n0 + (rp ^ (2 * (c & 3) + (c >> 2)));
                const int ch = cb * KST + c * EPC;
                if (n < p.cout && ch < p.cin) g = (const T*)p.w + ((long long)n * 9 + ky * 3 + kx) * p.cin + ch;
            } else if (s < A_SLOTS + B_SLOTS) {
                const int sb = s - A_SLOTS;
                const int hp = sb / CH, cp = sb - hp * CH;
                const int c = cp ^ ((hp / PXG) & (CH - 1));
                const int ty = hp / HX, hx = hp - ty * HX;
                const int iy = (oy0 + ty) * S + ky - 1, ix = ox0 * S - 1 + hx;
                const int ch = cb * KST + c * EPC;
                if (iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w && ch < p.cin)
                    g = src + ((long long)iy * sw + ix) * scs + ch;
            }
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                             (__attribute__((address_space(3))) void*)(base + 64 * 16 * (wave + 4 * i)),
                                             16, 0, 0);
        }
    };

    f32x4 acc[FR][FC];
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float lbias[FR][4];
    load_lane_bias<TN, WN, WM>(p, n0, lbias);

    const int frow = lane & 15, fq = lane >> 4;
    int hp0[FC];  // B-image pixel of this lane's fragment column at kx = 0
#pragma unroll
    for (int j = 0; j < FC; ++j) {
        const int pl = wc * WTM + j * 16 + frow;
        const int ty = pl / TX, tx = pl - ty * TX;
        hp0[j] = ty * HX + tx * S;
    }

    auto compute = [&](int buf) {
        const char* A = smem + buf * BUF;
        const char* B = A + A_SLOTS * 16;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
#pragma unroll
            for (int sl = 0; sl < KS; ++sl) {
                const int chunk = sl * 4 + fq, swa = 2 * fq + sl;
                uint4 af[FR], bf[FC];
#pragma unroll
                for (int i = 0; i < FR; ++i) {
                    const int r = wr * 64 + i * 16 + frow;
                    af[i] = *(const uint4*)(A + ((kx * CH + chunk) * TN + (r ^ swa)) * 16);
                }
#pragma unroll
                for (int j = 0; j < FC; ++j) {
                    const int hp = hp0[j] + kx;
                    bf[j] = *(const uint4*)(B + (hp * CH + (chunk ^ ((hp / PXG) & (CH - 1)))) * 16);
                }
#pragma unroll
                for (int i = 0; i < FR; ++i)
#pragma unroll
                    for (int j = 0; j < FC; ++j) Mma<T>::run(acc[i][j], af[i], bf[j]);
            }
        }
    };

    const int nk = p.ncb * 3;
    issue(0, 0);
    if constexpr (NBUF == 2) {
        for (int k = 0; k < nk; ++k) {
            wait_vm<0>();   // this wave's part of stage k landed
            raw_barrier();  // every wave's part landed; compute(k-1) finished -> its buffer is free
            if (k + 1 < nk) issue(k + 1, (k + 1) % NBUF);
            compute(k % NBUF);
        }
    } else {
        // one more stage in flight across each barrier (counted vmcnt, raw s_barrier)
        if (nk > 1) issue(1, 1);
        for (int k = 0; k < nk; ++k) {
            if (k + 1 < nk)
                wait_vm<G>();  // stage k landed; stage k+1 (G DMA instructions) may still fly
            else
                wait_vm<0>();
            raw_barrier();
            if (k + 2 < nk) issue(k + 2, (k + 2) % NBUF);
            compute(k % NBUF);
        }
    }
    wait_vm<0>();
    raw_barrier();
    const int OH = p.out_h, OW = p.out_w, mb = b * p.ohw;
    conv_epilogue_map<T, TN, TM, WN, WM, NBUF * BUF>(
        p, acc, smem,
        [=](int pl) {
            const int ty = pl / TX, tx = pl - ty * TX;
            const int oy = oy0 + ty, ox = ox0 + tx;
            return (oy < OH && ox < OW) ? mb + oy * OW + ox : -1;
        },
        n0, lbias);
}

template <typename T, int S, int TX, int TY, int CH, int TN, int NBUF>
constexpr int rows_lds_bytes() {
    constexpr int HX = (TX - 1) * S + 3;
    constexpr int slots = ((3 * TN * CH + TY * HX * CH + 255) / 256) * 256;
    return NBUF * slots * 16;
}

template <typename T, int S, int TX, int TY, int CH, int TN, int NBUF>
static int launch_rows(const ConvParams& p, hipStream_t st) {
    if constexpr (rows_lds_bytes<T, S, TX, TY, CH, TN, NBUF>() > 160 * 1024) {
        set_error("conv_rows variant needs more than 160 KiB of LDS for this stride / slab count");
        return YXH_EUNSUPPORTED;
    } else {
        const int tiles_x = (p.out_w + TX - 1) / TX, tiles_y = (p.out_h + TY - 1) / TY;
        const int ntn = (p.cout + TN - 1) / TN;
        const long long nblk = (long long)tiles_x * tiles_y * (p.M / p.ohw) * ntn;
        if (nblk >= (1LL << 31)) {
            set_error("conv_rows grid too large");
            return YXH_EINVAL;
        }
        hipLaunchKernelGGL((conv_rows<T, S, TX, TY, CH, TN, NBUF>), dim3((unsigned)nblk), dim3(256), 0, st, p,
                           tiles_x, tiles_y, ntn);
        YXH_CHECK_LAUNCH("conv_rows launch");
        return YXH_OK;
    }
}

// Variant table (yoloxhip.h tile ids 33..32+kNumRowTiles): output tile TX x TY, TN, NBUF.
// Ids 1-6 exist for every dtype, 7+ for bf16/f16 only.
template <typename T, int S, int CH>
static int dispatch_shape(int id, const ConvParams& p, hipStream_t st) {
    switch (id) {
        case 1: return launch_rows<T, S, 16, 16, CH, 64, 2>(p, st);
        case 2: return launch_rows<T, S, 20, 16, CH, 64, 2>(p, st);
        case 3: return launch_rows<T, S, 40, 8, CH, 64, 2>(p, st);
        case 4: return launch_rows<T, S, 80, 4, CH, 64, 2>(p, st);
        case 5: return launch_rows<T, S, 32, 8, CH, 64, 2>(p, st);
        case 6: return launch_rows<T, S, 64, 4, CH, 64, 2>(p, st);
        default: break;
    }
    if constexpr (sizeof(T) == 2) {
        switch (id) {
            case 7: return launch_rows<T, S, 40, 8, CH, 64, 3>(p, st);
            case 8: return launch_rows<T, S, 20, 16, CH, 64, 3>(p, st);
            case 9: return launch_rows<T, S, 32, 8, CH, 64, 3>(p, st);
            case 10: return launch_rows<T, S, 16, 8, CH, 64, 2>(p, st);
            case 11: return launch_rows<T, S, 32, 4, CH, 64, 2>(p, st);
            case 12: return launch_rows<T, S, 16, 16, CH, 128, 2>(p, st);
            case 13: return launch_rows<T, S, 32, 8, CH, 128, 2>(p, st);
            case 14: return launch_rows<T, S, 32, 4, CH, 128, 2>(p, st);
            case 15: return launch_rows<T, S, 16, 8, CH, 128, 2>(p, st);
            case 16: return launch_rows<T, S, 16, 8, CH, 64, 3>(p, st);
            case 17: return launch_rows<T, S, 32, 4, CH, 64, 3>(p, st);
            case 18: return launch_rows<T, S, 8, 16, CH, 64, 2>(p, st);
            case 19: return launch_rows<T, S, 64, 2, CH, 64, 2>(p, st);
            default: break;
        }
    } else if (id > 6 && id <= kNumRowTiles) {
        set_error("conv_rows variant %d is built for bf16/f16 only", id);
        return YXH_EUNSUPPORTED;
    }
    set_error("rows tile id %d", id);
    return YXH_EINVAL;
}

template <typename T>
int conv_rows_dispatch_t(int id, const ConvParams& p, int ks, hipStream_t st) {
    if (p.stride == 1) return ks == 2 ? dispatch_shape<T, 1, 8>(id, p, st) : dispatch_shape<T, 1, 4>(id, p, st);
    if (ks == 2) {
        set_error("conv_rows: 2-slab stages not built for stride 2");
        return YXH_EUNSUPPORTED;
    }
    return dispatch_shape<T, 2, 4>(id, p, st);
}

}  // namespace yxh
