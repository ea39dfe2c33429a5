// conv_pwr: pointwise (1x1, stride 1) conv whose pixel operand goes straight from
// global memory into MFMA fragment registers (reference network_blocks.py:48-49
// BaseConv with ksize 1: CSP conv1/2/3, PAFPN laterals, head stems, pred convs of
// yolo_head.py:149-160).
//
// The wide 1x1 layers of YOLOX at 160x160 / 80x80 move ~2 B per MAC column and are
// HBM-bound; the LDS round trip of the operand tiles is pure overhead there.  In the
// NHWC layout the 16-byte K chunk a 16x16x32 MFMA lane needs (8 channels of one pixel)
// is contiguous, so lane (frow, fq) of a fragment loads pixel frow's chunk fq directly:
// one wave instruction covers 16 whole pixel rows.
//  * Block = 4 independent waves; each wave owns pixel tiles of 16*FC pixels x TN =
//    16*FR output channels and grid-strides over the tiles with the next tile's
//    fragments prefetched into registers (no barrier in the loop).
//  * The TN x Cin weight slice is resident in LDS for the block's lifetime (the
//    [chunk][row ^ (2*chunk%4 + chunk/4)] image of conv.hip, conflict-free reads).
//  * Epilogue: bias + act in registers; a per-wave LDS staging tile turns the lane-
//    scattered 8-byte pieces into 16-byte chunks of whole pixel rows (coalesced);
//    fp32 / decode outputs (the head preds) take the scalar store path.
#include "conv_common.hpp"

namespace yxh {

namespace {

__device__ __attribute__((aligned(16))) uint4 g_pwr_zero[4];

__device__ __forceinline__ int pwr_xcd_remap(int id, int nblk) {
    const int q = nblk / 8, r = nblk % 8, xcd = id % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
}

}  // namespace

struct PwrArgs {
    int ntiles;          // pixel tiles of 16*FC
    int dense0, dense1;  // source image stride == pixels * pixel stride (no (b, y, x) split needed)
};

template <typename T, int FR, int KSL, int FC>
__global__ __launch_bounds__(256) void conv_pwr(ConvParams p, PwrArgs a) {
    constexpr int EPC = Chunk<T>::N;
    constexpr int NCH = 4 * KSL;  // 16-byte K chunks
    constexpr int TN = FR * 16;
    constexpr int WB = TN * NCH * 16;
    constexpr int OES = sizeof(T);
    constexpr int OROW = TN * OES + 16;
    constexpr int STG = 16 * FC * OROW;
    __shared__ __attribute__((aligned(16))) char smem[WB + 4 * STG + TN * 4];
    char* wl = smem;
    float* lbias = (float*)(smem + WB + 4 * STG);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int frow = lane & 15, fq = lane >> 4;
    const int n0 = blockIdx.y * TN;
    char* wst = smem + WB + wave * STG;

    const int nwav = gridDim.x * 4;
    const int first = pwr_xcd_remap(blockIdx.x, gridDim.x) * 4 + wave;
    const T* sp0 = (const T*)p.sptr[0];
    const T* sp1 = (const T*)p.sptr[1];
    const T* zero = (const T*)g_pwr_zero;

    auto load = [&](int tile, uint4 (&d)[FC][KSL]) {
#pragma unroll
        for (int j = 0; j < FC; ++j) {
            const int m = tile * 16 * FC + j * 16 + frow;
            const bool mok = tile < a.ntiles && m < p.M;
            const int mm = mok ? m : 0;
            long long off0, off1 = 0;
            if (a.dense0) {
                off0 = (long long)mm * p.scs[0];
            } else {
                const int b = mm / p.ohw, pix = mm - b * p.ohw;
                const int y = pix / p.out_w, x = pix - y * p.out_w;
                const int up = p.sup[0];
                off0 = b * p.sbs[0] + ((long long)(y >> up) * p.sw[0] + (x >> up)) * p.scs[0];
            }
            if (p.nsrc == 2) {
                if (a.dense1) {
                    off1 = (long long)mm * p.scs[1];
                } else {
                    const int b = mm / p.ohw, pix = mm - b * p.ohw;
                    const int y = pix / p.out_w, x = pix - y * p.out_w;
                    const int up = p.sup[1];
                    off1 = b * p.sbs[1] + ((long long)(y >> up) * p.sw[1] + (x >> up)) * p.scs[1];
                }
            }
#pragma unroll
            for (int s = 0; s < KSL; ++s) {
                const int ch = (s * 4 + fq) * EPC;
                const T* ptr = (p.nsrc == 2 && ch >= p.src0_ch) ? sp1 + off1 + (ch - p.src0_ch) : sp0 + off0 + ch;
                d[j][s] = *(const uint4*)((mok && ch < p.cin) ? ptr : zero);
            }
        }
    };

    const bool staged = p.vec16 && !p.dst_f32;
    uint4 bf[FC][KSL], nb[FC][KSL];
    // first pixel tile in flight before the weight image is staged: the two global
    // round trips overlap instead of chaining through the barrier
    load(first, bf);
    for (int s = tid; s < TN * NCH; s += 256) {
        const int c = s / TN, rp = s - c * TN;
        const int n = n0 + (rp ^ (2 * (c & 3) + (c >> 2)));
        const int ch = c * EPC;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (n < p.cout && ch < p.cin) v = *(const uint4*)((const T*)p.w + (long long)n * p.cin + ch);
        *(uint4*)(wl + s * 16) = v;
    }
    if (tid < TN) lbias[tid] = n0 + tid < p.cout ? p.bias[n0 + tid] : 0.0f;
    __syncthreads();
    for (int t = first; t < a.ntiles; t += nwav) {
        load(t + nwav, nb);
        f32x4 acc[FR][FC];
#pragma unroll
        for (int i = 0; i < FR; ++i)
#pragma unroll
            for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KSL; ++s) {
            const int chunk = s * 4 + fq, sw_ = 2 * fq + s;
            uint4 af[FR];
#pragma unroll
            for (int i = 0; i < FR; ++i) af[i] = *(const uint4*)(wl + (chunk * TN + ((i * 16 + frow) ^ sw_)) * 16);
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) Mma<T>::run(acc[i][j], af[i], bf[j][s]);
        }
        const int m0 = t * 16 * FC;
        if (staged) {
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                const int pl = j * 16 + frow;
#pragma unroll
                for (int i = 0; i < FR; ++i) {
                    const int nl = i * 16 + fq * 4;
                    T o[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        o[r] = from_f32<T>(apply_act<sizeof(T) == 4>(acc[i][j][r] + lbias[nl + r], p.act));
                    uint2 u;
                    __builtin_memcpy(&u, o, 8);
                    *(uint2*)(wst + pl * OROW + nl * OES) = u;
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            constexpr int CPO = TN * OES / 16;
            const int ncols = min(TN, p.cout - n0) * OES / 16;
            for (int q = lane; q < 16 * FC * CPO; q += 64) {
                const int r = q / CPO, c = q - r * CPO;
                const int m = m0 + r;
                if (m >= p.M || c >= ncols) continue;
                long long off;
                if (p.dst_dense) {
                    off = (long long)m * p.dst_cs;
                } else {
                    const int b = m / p.ohw, pix = m - b * p.ohw;
                    off = (long long)b * p.dst_bs + (long long)pix * p.dst_cs;
                }
                const uint4 u = *(const uint4*)(wst + r * OROW + c * 16);
                *(uint4*)((char*)p.dst + (off + n0) * OES + c * 16) = u;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
        } else {
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                const int m = m0 + j * 16 + frow;
                if (m >= p.M) continue;
                const int b = m / p.ohw, pix = m - b * p.ohw;
                const int oy = pix / p.out_w, ox = pix - oy * p.out_w;
#pragma unroll
                for (int i = 0; i < FR; ++i) {
                    const int nl = i * 16 + fq * 4, n = n0 + nl;
                    if (n >= p.cout) continue;
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + lbias[nl + r];
                    store4<T>(p, v, n, b, pix, ox, oy);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < FC; ++j)
#pragma unroll
            for (int s = 0; s < KSL; ++s) bf[j][s] = nb[j][s];
    }
}

namespace {

template <typename T, int FR, int KSL>
int launch_pwr(const ConvParams& p, const PwrArgs& a0, hipStream_t st) {
    constexpr int FC0 = 8 / FR < 8 / KSL ? 8 / FR : 8 / KSL;
    constexpr int FC = FC0 < 1 ? 1 : FC0;
    constexpr int TN = FR * 16;
    constexpr int LDS = TN * 4 * KSL * 16 + 4 * 16 * FC * (TN * (int)sizeof(T) + 16) + TN * 4;
    PwrArgs a = a0;
    a.ntiles = (p.M + 16 * FC - 1) / (16 * FC);
    const int ntn = (p.cout + TN - 1) / TN;
    const int occ = max(1, min(4, (160 * 1024) / LDS));
    long long blocks = (long long)256 * occ / ntn;
    const long long want = (a.ntiles + 3) / 4;
    if (blocks > want) blocks = want;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL((conv_pwr<T, FR, KSL, FC>), dim3((unsigned)blocks, ntn), dim3(256), 0, st, p, a);
    YXH_CHECK_LAUNCH("conv_pwr launch");
    return YXH_OK;
}

template <typename T, int FR>
int pwr_ksl(int ksl, const ConvParams& p, const PwrArgs& a, hipStream_t st) {
    switch (ksl) {
        case 1: return launch_pwr<T, FR, 1>(p, a, st);
        case 2: return launch_pwr<T, FR, 2>(p, a, st);
        case 4: return launch_pwr<T, FR, 4>(p, a, st);
        case 8: return launch_pwr<T, FR, 8>(p, a, st);
        default: set_error("conv_pwr K slabs %d", ksl); return YXH_EUNSUPPORTED;
    }
}

template <typename T>
int pwr_t(int fr, int ksl, const ConvParams& p, const PwrArgs& a, hipStream_t st) {
    switch (fr) {
        case 1: return pwr_ksl<T, 1>(ksl, p, a, st);
        case 2: return pwr_ksl<T, 2>(ksl, p, a, st);
        case 4: return pwr_ksl<T, 4>(ksl, p, a, st);
        case 5: return pwr_ksl<T, 5>(ksl, p, a, st);
        case 8: return pwr_ksl<T, 8>(ksl, p, a, st);
        default: set_error("conv_pwr row fragments %d", fr); return YXH_EUNSUPPORTED;
    }
}

}  // namespace

// Variant id 1: the smallest channel tile covering cout (<= 128, else 128-wide tiles);
// id 2: 64-wide channel tiles (32 for cout <= 32).
int conv_pwr_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st) {
    if (p.taps != 1 || p.stride != 1 || p.pad != 0 || p.res) {
        set_error("conv_pwr needs a 1x1 stride-1 conv without residual");
        return YXH_EUNSUPPORTED;
    }
    if (dtype != YXH_BF16 && dtype != YXH_F16) {
        set_error("conv_pwr is built for bf16/f16 only");
        return YXH_EUNSUPPORTED;
    }
    if (p.sup[0] > 1 || (p.nsrc == 2 && p.sup[1] > 1)) {
        set_error("conv_pwr: dilated sources unsupported");
        return YXH_EUNSUPPORTED;
    }
    const int nch = (p.cin + 7) / 8;  // 16-byte K chunks
    int ksl = (nch + 3) / 4;
    ksl = ksl <= 1 ? 1 : ksl <= 2 ? 2 : ksl <= 4 ? 4 : ksl <= 8 ? 8 : 0;
    if (!ksl || (p.nsrc == 2 && p.src0_ch % 8)) {
        set_error("conv_pwr: cin %d beyond 256 (or a source split inside a chunk)", p.cin);
        return YXH_EUNSUPPORTED;
    }
    int fr;
    if (id == 1) {
        const int need = (p.cout + 15) / 16;
        fr = need <= 1 ? 1 : need <= 2 ? 2 : need <= 4 ? 4 : need <= 5 ? 5 : 8;
    } else if (id == 2) {
        fr = p.cout <= 32 ? 2 : 4;
    } else {
        set_error("conv_pwr tile id %d", id);
        return YXH_EINVAL;
    }
    PwrArgs a{};
    a.dense0 = !p.sup[0] && p.sw[0] == p.out_w && p.sbs[0] == (long long)p.ohw * p.scs[0];
    a.dense1 = p.nsrc == 2 && !p.sup[1] && p.sw[1] == p.out_w && p.sbs[1] == (long long)p.ohw * p.scs[1];
    if (dtype == YXH_BF16) return pwr_t<bf16>(fr, ksl, p, a, st);
    return pwr_t<f16>(fr, ksl, p, a, st);
}

}  // namespace yxh
