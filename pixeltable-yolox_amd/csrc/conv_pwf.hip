// conv_pwf: 1x1 stride-1 conv over dense NHWC activations as a plain GEMM whose K loop
// costs (almost) no VALU (reference network_blocks.py:48-49 BaseConv with ksize 1: CSP
// conv1/2/3, SPP convs, PAFPN laterals, head stems).
//
// The 1x1 layers of YOLOX are HBM/issue bound (PMC: the register-staged kernels spent
// ~500 VALU instructions per wave on loader/epilogue index math for 16 MFMAs).  Here:
//  * every operand row is a contiguous run of K elements (pixel m at m * cstride, weight
//    row n at n * cin), so each lane's LDS-DMA source is fixed for the whole K loop: one
//    32-bit per-lane byte offset per DMA instruction, computed once, plus a wave-uniform
//    (SGPR) stage base -- the loop issues global_load_lds with no address arithmetic;
//  * a K stage is KCH 16-byte chunks per row (4: 32 elements, 8: 64); LDS-DMA writes
//    lane-linearly, so the row's chunks are XOR-swizzled through the SOURCE address
//    (phys chunk c holds logical chunk c ^ f(row)) and the fragment reads undo it:
//    ds_read_b128 of 16 rows x one chunk spans all 64 banks (conflict free);
//  * NBUF-deep ring, counted s_waitcnt vmcnt + raw s_barrier (no vmcnt(0) drain);
//  * out-of-range rows (M or cout tails) re-read the last valid row (their outputs are
//    never stored), so no lane branches around a load;
//  * epilogue straight from the accumulators: bias, activation, optional residual
//    (added after the activation, one rounding), 8-byte stores of 4 channels per lane.
// Wave grid: TN = 64 x 4 waves along pixels, or TN = 128 as 2 x 2; every wave owns
// 64 output channels x TM / WM pixels (4 x FC MFMA 16x16x32 tiles).
#include "conv_common.hpp"

namespace yxh {

namespace {

template <int N>
__device__ __forceinline__ void pwf_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void pwf_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// swizzle of a row's 16-byte chunks: rows of KCH chunks share a 256-byte bank row with
// 256 / (16 * KCH) - 1 others; XOR with the row's index among them spreads 16 rows
template <int KCH>
__device__ __forceinline__ int pwf_swz(int row) {
    return KCH == 8 ? (row >> 1) & 7 : (row >> 2) & 3;
}

__device__ __forceinline__ int pwf_xcd_remap(int id, int nblk) {
    const int q = nblk / 8, r = nblk % 8, xcd = id % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
}

}  // namespace

template <typename T, int FR, int FC, int WTM, int TN, int ACT>
__device__ __forceinline__ void pwf_epilogue(const ConvParams& p, const f32x4 (&acc)[FR][FC], const float* lbias,
                                             int m0, int n0, int wr, int wc);

// The LDS-DMA is issued from inline asm: hipcc tracks its own global_load_lds as a
// pending LDS write and puts s_waitcnt vmcnt(0) in front of every later ds_read (it
// cannot tell the ring buffers apart), which drains the ring each stage.  Our counted
// vmcnt waits + barriers order the reads instead (MI355X_MICROARCH.md: only the issuing
// wave's vmcnt orders a ds_read behind an LDS-DMA).  M0 = wave-uniform LDS address.
__device__ __forceinline__ void pwf_glds(const char* sbase, uint32_t voff, uint32_t lds) {
    uint32_t saved;  // M0 is reserved to the compiler: save and restore it around the DMA
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
        : "=&s"(saved)
        : "v"(voff), "s"(sbase), "s"(lds)
        : "memory");
}

__device__ __forceinline__ uint32_t pwf_lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Persistent over pixel tiles: block L owns channel tile L % ntn and pixel tiles
// L / ntn, + gridDim.x / ntn, ...; the stage sequence (tile, k) runs across tiles, so
// the next tile's loads fly while this tile's epilogue stores drain.
template <typename T, int TN, int TM, int KCH, int NBUF>
__global__ __launch_bounds__(256) void conv_pwf(ConvParams p, int ntn, int nk, int ntm) {
    constexpr int WN = TN / 64, WM = 4 / WN;
    constexpr int WTM = TM / WM;
    constexpr int FR = 4, FC = WTM / 16;
    constexpr int RPI = 64 / KCH;                        // rows per DMA instruction
    constexpr int GA = TN / RPI / 4, GB = TM / RPI / 4;  // DMA instructions per wave per stage
    constexpr int G = GA + GB;
    constexpr int ROWB = KCH * 16;                       // bytes per staged row
    constexpr int A_BYTES = TN * ROWB, BUF = (TN + TM) * ROWB;
    constexpr int KSTB = KCH * 16;                       // K bytes per stage (= ROWB)
    constexpr int ES = sizeof(T);
    static_assert(GA >= 1 && GB >= 1 && TN % (4 * RPI) == 0 && TM % (4 * RPI) == 0, "tile");
    __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF + TN * 4];
    float* lbias = (float*)(smem + NBUF * BUF);  // folded bias of the block's channels

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave / WM, wc = wave % WM;
    const int L = pwf_xcd_remap(blockIdx.x, gridDim.x);
    const int n0 = (L % ntn) * TN;
    // bias -> LDS before any DMA: a register load consumed in the epilogue would make
    // hipcc wait vmcnt(0) there, draining the next tile's loads
    if (tid < TN) lbias[tid] = n0 + tid < p.cout ? p.bias[n0 + tid] : 0.0f;
    __syncthreads();
    const int pstart = L / ntn, pstep = gridDim.x / ntn;
    const int mytiles = pstart < ntm ? (ntm - pstart + pstep - 1) / pstep : 0;
    const int nstages = mytiles * nk;
    const uint32_t lds0 = pwf_lds_addr(smem) + (uint32_t)wave * 1024;

    // per-lane DMA byte offsets (fixed for the block's life)
    const int prow = lane / KCH, pch = lane % KCH;
    uint32_t aoff[GA], boff0[GB], boff1[GB];
#pragma unroll
    for (int i = 0; i < GA; ++i) {
        const int r = (wave + 4 * i) * RPI + prow;
        const int n = min(n0 + r, p.cout - 1);
        aoff[i] = (uint32_t)n * (uint32_t)(p.cin * ES) + (uint32_t)((pch ^ pwf_swz<KCH>(r)) * 16);
    }
    const int nsrc = p.nsrc;
    const uint32_t rb0 = (uint32_t)(p.scs[0] * ES), rb1 = (uint32_t)(p.scs[nsrc == 2 ? 1 : 0] * ES);
#pragma unroll
    for (int i = 0; i < GB; ++i) {
        const int r = (wave + 4 * i) * RPI + prow;
        const uint32_t sw = (uint32_t)((pch ^ pwf_swz<KCH>(r)) * 16);
        boff0[i] = (uint32_t)r * rb0 + sw;
        boff1[i] = (uint32_t)r * rb1 + sw;
    }
    const int k_split = nsrc == 2 ? p.src0_ch / (KCH * Chunk<T>::N) : nk;
    const int M = p.M;
    // source 0 may be a nearest-x2 upsampled view (PAFPN cat(upsample(x), skip)): its rows
    // are not linear in m, so each lane's row offsets are recomputed once per pixel tile
    // (at the tile's first stage) instead of per stage
    const bool up0 = p.sup[0] != 0;
    uint32_t boffu[GB];
#pragma unroll
    for (int i = 0; i < GB; ++i) boffu[i] = 0;

    auto issue = [&](int st) {
        const int tl = st / nk, k = st - tl * nk;
        const int m0 = (pstart + tl * pstep) * TM;
        const uint32_t lbase = lds0 + (uint32_t)((st % NBUF) * BUF);
        const char* wa = (const char*)p.w + (long long)k * KSTB;
#pragma unroll
        for (int i = 0; i < GA; ++i) pwf_glds(wa, aoff[i], lbase + i * 4096);
        const bool s1 = k >= k_split;
        const uint32_t rb = s1 ? rb1 : rb0;
        const uint32_t lb = lbase + A_BYTES;
        if (up0 && !s1) {
            if (k == 0) {
#pragma unroll
                for (int i = 0; i < GB; ++i) {
                    const int r = (wave + 4 * i) * RPI + prow;
                    const int m = min(m0 + r, M - 1);
                    const int b = m / p.ohw, pix = m - b * p.ohw;
                    const int y = pix / p.out_w, x = pix - y * p.out_w;
                    boffu[i] = (uint32_t)(((long long)b * p.sbs[0] + (long long)((y >> 1) * p.sw[0] + (x >> 1)) * p.scs[0]) *
                                          ES) +
                               (uint32_t)((pch ^ pwf_swz<KCH>(r)) * 16);
                }
            }
            const char* xb = (const char*)p.sptr[0] + (long long)k * KSTB;
#pragma unroll
            for (int i = 0; i < GB; ++i) pwf_glds(xb, boffu[i], lb + i * 4096);
            return;
        }
        const char* xb = (const char*)p.sptr[s1 ? 1 : 0] + (long long)m0 * rb + (long long)(s1 ? k - k_split : k) * KSTB;
        if (m0 + TM <= M) {
#pragma unroll
            for (int i = 0; i < GB; ++i) pwf_glds(xb, s1 ? boff1[i] : boff0[i], lb + i * 4096);
        } else {  // pixel tail: rows past M re-read row M - 1 (never stored)
#pragma unroll
            for (int i = 0; i < GB; ++i) {
                const int r = (wave + 4 * i) * RPI + prow;
                const uint32_t o = s1 ? boff1[i] : boff0[i];
                const uint32_t clampd = o - (uint32_t)r * rb + (uint32_t)min(r, M - 1 - m0) * rb;
                pwf_glds(xb, clampd, lb + i * 4096);
            }
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
        for (int s = 0; s < KCH / 4; ++s) {
            const int ch = s * 4 + fq;
            uint4 af[FR], bf[FC];
#pragma unroll
            for (int i = 0; i < FR; ++i) {
                const int r = wr * 64 + i * 16 + frow;
                af[i] = *(const uint4*)(A + r * ROWB + ((ch ^ pwf_swz<KCH>(r)) * 16));
            }
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                const int r = wc * WTM + j * 16 + frow;
                bf[j] = *(const uint4*)(B + r * ROWB + ((ch ^ pwf_swz<KCH>(r)) * 16));
            }
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) Mma<T>::run(acc[i][j], af[i], bf[j]);
        }
    };

    constexpr int D = NBUF - 1;
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (d < nstages) issue(d);
    for (int st = 0; st < nstages; ++st) {
        const int younger = min(D - 1, nstages - 1 - st);  // stages issued after st still in flight
        if constexpr (D >= 3) {
            if (younger >= 2) pwf_wait_vm<2 * G>();
            else if (younger == 1) pwf_wait_vm<G>();
            else pwf_wait_vm<0>();
        } else if constexpr (D == 2) {
            if (younger >= 1) pwf_wait_vm<G>();
            else pwf_wait_vm<0>();
        } else {
            pwf_wait_vm<0>();
        }
        pwf_barrier();  // every wave's stage st landed; stage st-1's buffer is free
        if (st + D < nstages) issue(st + D);
        compute(st % NBUF);
        const int tl = st / nk;
        if (st - tl * nk == nk - 1) {
            // epilogue of this pixel tile (activation as a template argument: a runtime
            // switch inside the unrolled loops would branch per element)
            const int m0 = (pstart + tl * pstep) * TM;
            switch (p.act) {
                case YXH_ACT_SILU: pwf_epilogue<T, FR, FC, WTM, TN, YXH_ACT_SILU>(p, acc, lbias, m0, n0, wr, wc); break;
                case YXH_ACT_RELU: pwf_epilogue<T, FR, FC, WTM, TN, YXH_ACT_RELU>(p, acc, lbias, m0, n0, wr, wc); break;
                case YXH_ACT_LRELU: pwf_epilogue<T, FR, FC, WTM, TN, YXH_ACT_LRELU>(p, acc, lbias, m0, n0, wr, wc); break;
                default: pwf_epilogue<T, FR, FC, WTM, TN, YXH_ACT_NONE>(p, acc, lbias, m0, n0, wr, wc); break;
            }
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
}

template <typename T, int FR, int FC, int WTM, int TN, int ACT>
__device__ __forceinline__ void pwf_epilogue(const ConvParams& p, const f32x4 (&acc)[FR][FC], const float* lbias,
                                             int m0, int n0, int wr, int wc) {
    const int lane = threadIdx.x & 63, frow = lane & 15, fq = lane >> 4;
    if constexpr (ACT == YXH_ACT_NONE) {
        if (p.dst_f32) {  // the 16-bit training step's 1x1 data gradient: fp32 rows, YXH_CONV_ACCUMULATE
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                const int m = m0 + wc * WTM + j * 16 + frow;
                if (m >= p.M) continue;
                float* drow = (float*)p.dst + (long long)m * p.dst_cs;
#pragma unroll
                for (int i = 0; i < FR; ++i) {
                    const int n = n0 + wr * 64 + i * 16 + fq * 4;
                    if (n >= p.cout) continue;
                    const float* lb = lbias + wr * 64 + i * 16 + fq * 4;
                    f32x4 v = acc[i][j] + f32x4{lb[0], lb[1], lb[2], lb[3]};
                    float4* dp = (float4*)(drow + n);
                    if (p.accum) {
                        const float4 o = *dp;
                        v = v + f32x4{o.x, o.y, o.z, o.w};
                    }
                    *dp = make_float4(v[0], v[1], v[2], v[3]);
                }
            }
            return;
        }
    }
#pragma unroll
    for (int j = 0; j < FC; ++j) {
        const int m = m0 + wc * WTM + j * 16 + frow;
        if (m >= p.M) continue;
        T* drow = (T*)p.dst + (long long)m * p.dst_cs;
        const T* rrow = p.res ? (const T*)p.res + (long long)m * p.res_cs : nullptr;
#pragma unroll
        for (int i = 0; i < FR; ++i) {
            const int n = n0 + wr * 64 + i * 16 + fq * 4;
            if (n >= p.cout) continue;
            const float* lb = lbias + wr * 64 + i * 16 + fq * 4;
            f32x4 v = acc[i][j] + f32x4{lb[0], lb[1], lb[2], lb[3]};
            if constexpr (ACT == YXH_ACT_SILU) {
                v = silu4(v);  // packed pairs, bit-identical to apply_act's silu
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = apply_act<false>(v[r], ACT);
            }
            if (rrow) {
                const uint2 u = *(const uint2*)(rrow + n);
                T t[4];
                __builtin_memcpy(t, &u, 8);
                v = v + f32x4{to_f32(t[0]), to_f32(t[1]), to_f32(t[2]), to_f32(t[3])};
            }
            T t[4] = {from_f32<T>(v[0]), from_f32<T>(v[1]), from_f32<T>(v[2]), from_f32<T>(v[3])};
            uint2 u;
            __builtin_memcpy(&u, t, 8);
            *(uint2*)(drow + n) = u;
        }
    }
}

// PER_CU: resident blocks per CU for the persistent grid (0: one block per pixel tile)
template <typename T, int TN, int TM, int KCH, int NBUF, int PER_CU>
static int launch_pwf(const ConvParams& p, hipStream_t st) {
    constexpr int EPC = Chunk<T>::N;
    const int kst = KCH * EPC;
    if (p.cin % kst || (p.nsrc == 2 && p.src0_ch % kst)) {
        set_error("conv_pwf: cin %d (split %d) not a multiple of the %d-element K stage", p.cin, p.src0_ch, kst);
        return YXH_EUNSUPPORTED;
    }
    const int ntn = (p.cout + TN - 1) / TN, ntm = (p.M + TM - 1) / TM;
    long long blocks = (long long)ntn * ntm;
    if (PER_CU == 0 && p.cus < 256) {  // one block per tile: cap the grid as a persistent one would be
        const long long cap = std::max<long long>(ntn, (long long)p.cus * 2 / ntn * ntn);
        if (blocks > cap) blocks = cap;
    }
    if (PER_CU > 0) {
        long long cap = (long long)p.cus * PER_CU / ntn * ntn;  // whole channel-tile groups
        if (cap < ntn) cap = ntn;
        if (blocks > cap) blocks = cap;
    }
    hipLaunchKernelGGL((conv_pwf<T, TN, TM, KCH, NBUF>), dim3((unsigned)blocks), dim3(256), 0, st, p, ntn, p.cin / kst,
                       ntm);
    YXH_CHECK_LAUNCH("conv_pwf launch");
    return YXH_OK;
}

template <typename T>
static int pwf_dispatch_t(int id, const ConvParams& p, hipStream_t st) {
    // id -> (TN, TM, KCH, NBUF, resident blocks per CU of the persistent grid)
    switch (id) {
        case 1: return launch_pwf<T, 64, 128, 4, 3, 0>(p, st);
        case 2: return launch_pwf<T, 64, 128, 4, 3, 4>(p, st);
        case 3: return launch_pwf<T, 64, 128, 8, 3, 0>(p, st);
        case 4: return launch_pwf<T, 64, 128, 8, 3, 3>(p, st);
        case 5: return launch_pwf<T, 128, 128, 8, 3, 0>(p, st);
        case 6: return launch_pwf<T, 128, 128, 8, 3, 2>(p, st);
        case 7: return launch_pwf<T, 64, 256, 4, 3, 2>(p, st);
        case 8: return launch_pwf<T, 128, 64, 8, 4, 3>(p, st);
        default: set_error("conv_pwf tile id %d", id); return YXH_EINVAL;
    }
}

int conv_pwf_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st) {
    // an fp32 dst (16-bit operands): the training step's 1x1 data gradient -- no activation / residual,
    // 16-byte rows of whole 4-channel groups (vec_store is the 16-byte test for an fp32 dst)
    const bool f32ok = !p.dst_f32 || (p.act == YXH_ACT_NONE && !p.res && p.cout % 4 == 0);
    bool dense = p.taps == 1 && p.stride == 1 && p.pad == 0 && f32ok && p.act < YXH_ACT_DECODE && p.dst_dense &&
                 (!p.res || p.res_dense) && p.vec_store && (!p.res || p.vec_res);
    for (int s = 0; s < p.nsrc; ++s) {
        if (s == 0 && p.sup[0] == 1)  // nearest-x2 upsampled first source: any image stride
            dense &= p.sw[0] * 2 == p.out_w;
        else
            dense &= !p.sup[s] && p.sw[s] == p.out_w && p.sbs[s] == (long long)p.ohw * p.scs[s];
    }
    if (!dense) {
        set_error("conv_pwf needs a 1x1 s1 conv over dense sources (the first may be x2 upsampled) into a dense "
                  "16-bit dst (or an fp32 one without activation / residual)");
        return YXH_EUNSUPPORTED;
    }
    const long long img0 = p.sup[0] ? (p.M / p.ohw) * p.sbs[0] : (long long)p.M * p.scs[0];
    if (img0 * 2 >= (1LL << 32) || (p.nsrc == 2 && (long long)p.M * p.scs[1] * 2 >= (1LL << 32))) {
        set_error("conv_pwf: source exceeds 32-bit byte offsets");
        return YXH_EUNSUPPORTED;
    }
    if (dtype == YXH_BF16) return pwf_dispatch_t<bf16>(id, p, st);
    if (dtype == YXH_F16) return pwf_dispatch_t<f16>(id, p, st);
    set_error("conv_pwf is built for bf16/f16 only");
    return YXH_EUNSUPPORTED;
}

}  // namespace yxh
