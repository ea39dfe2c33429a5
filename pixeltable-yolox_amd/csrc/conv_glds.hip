// conv_glds: the implicit-GEMM conv of conv.hip with its operand tiles moved by
// LDS-DMA (global_load_lds_dwordx4) instead of global->VGPR->ds_write staging.
//
// * No staging registers and no ds_write instructions: the VGPR budget goes to
//   accumulators / occupancy, and each stage's loads stay in flight across barriers.
// * A 3-buffer LDS ring: at iteration k, stage k+1 is in flight while stage k+2 is
//   issued right after the barrier that retires stage k (counted s_waitcnt vmcnt,
//   raw s_barrier -- __syncthreads would drain every pending LDS-DMA).
// * LDS-DMA writes lane-linearly (wave-uniform base + 16 B x lane), so the XOR
//   swizzled [slab][chunk][row] image of conv.hip is produced by permuting the SOURCE
//   rows per lane (slot (c, r') <- row r' ^ (2*chunk + slab)); out-of-range rows,
//   padding pixels and masked channels read a 16-byte zero chunk.
// * Every wave issues the same number of LDS-DMA instructions per stage (the slot
//   count is padded to a multiple of 4 waves x 64 lanes with scratch slots) so one
//   compile-time vmcnt retires exactly one stage.
#include "conv_common.hpp"

namespace yxh {

__device__ __attribute__((aligned(16))) uint4 g_zero_chunk[4];

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void block_barrier() {
    // all of this wave's LDS reads are back (lgkmcnt), then the hardware barrier; the
    // asm memory clobbers keep the compiler from moving LDS accesses across it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <typename T, int TN, int TM, int WR, int WC, int KS>
__global__ __launch_bounds__(256) void conv_glds(ConvParams p) {
    constexpr int EPC = Chunk<T>::N;
    constexpr int CPR = 4 * KS;
    constexpr int KSTAGE = CPR * EPC;
    constexpr int WTN = TN / WR, WTM = TM / WC;
    constexpr int FR = WTN / 16, FC = WTM / 16;
    constexpr int A_SLOTS = TN * CPR, B_SLOTS = TM * CPR;
    constexpr int SLOTS = ((A_SLOTS + B_SLOTS + 255) / 256) * 256;  // padded to 4 waves x 64
    constexpr int G = SLOTS / 256;                                   // DMA instructions / wave / stage
    constexpr int BUF = SLOTS * 16;
    constexpr int NBUF = 3;
    static_assert(A_SLOTS % 64 == 0 && B_SLOTS % 64 == 0, "a wave's 64 slots must not straddle A and B");
    static_assert(G <= 20, "vmcnt range");
    __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave / WC, wc = wave % WC;
    const int n0 = blockIdx.y * TN, m0 = blockIdx.x * TM;

    // per DMA instruction i of this lane: which operand row / chunk it fetches
    int kind[G], row[G], cch[G], bb[G], by[G], bx[G];
#pragma unroll
    for (int i = 0; i < G; ++i) {
        const int s = 64 * (wave + 4 * i) + lane;
        kind[i] = 2;  // scratch
        row[i] = cch[i] = bb[i] = by[i] = bx[i] = 0;
        if (s < A_SLOTS) {
            const int c = s / TN, rp = s - c * TN;
            const int r = rp ^ (2 * (c & 3) + (c >> 2));
            kind[i] = 0;
            cch[i] = c;
            row[i] = n0 + r;
        } else if (s < A_SLOTS + B_SLOTS) {
            const int sb = s - A_SLOTS;
            const int c = sb / TM, rp = sb - c * TM;
            const int r = rp ^ (2 * (c & 3) + (c >> 2));
            const int m = m0 + r;
            kind[i] = 1;
            cch[i] = c;
            const bool ok = m < p.M;
            const int b = ok ? m / p.ohw : 0;
            const int rem = m - b * p.ohw;
            const int oy = rem / p.out_w, ox = rem - oy * p.out_w;
            bb[i] = ok ? b : -1;
            by[i] = oy * p.stride - p.pad;
            bx[i] = ox * p.stride - p.pad;
        }
    }

    // stages are issued strictly in order: (tap, channel block) advance incrementally
    int g_t = 0, g_cb = 0, g_ky = 0, g_kx = 0;
    auto issue = [&](int, int buf) {
        const int t = g_t, cb = g_cb, ky = g_ky, kx = g_kx;
        if (++g_cb == p.ncb) {
            g_cb = 0;
            ++g_t;
            if (++g_kx == p.kw) {
                g_kx = 0;
                ++g_ky;
            }
        }
        char* base = smem + buf * BUF;
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const void* src = (const void*)g_zero_chunk;
            const int c = cb * KSTAGE + cch[i] * EPC;
            if (kind[i] == 0) {
                if (row[i] < p.cout && c < p.cin)
                    src = (const T*)p.w + ((long long)row[i] * p.taps + t) * p.cin + c;
            } else if (kind[i] == 1) {
                const int iy = by[i] + ky, ix = bx[i] + kx;
                if (bb[i] >= 0 && c < p.cin && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w) {
                    int s = 0, cc = c;
                    if (p.nsrc == 2 && c >= p.src0_ch) {
                        s = 1;
                        cc = c - p.src0_ch;
                    }
                    const int up = p.sup[s];
                    src = (const T*)p.sptr[s] + bb[i] * p.sbs[s] +
                          ((long long)(iy >> up) * p.sw[s] + (ix >> up)) * p.scs[s] + cc;
                }
            }
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)(base + 64 * 16 * (wave + 4 * i)),
                                             16, 0, 0);
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
        const char* B = A + A_SLOTS * 16;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int chunk = s * 4 + fq, sw_ = 2 * fq + s;
            uint4 af[FR], bf[FC];
#pragma unroll
            for (int i = 0; i < FR; ++i) {
                int r = wr * WTN + i * 16 + frow;
                af[i] = *(const uint4*)(A + (chunk * TN + (r ^ sw_)) * 16);
            }
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                int r = wc * WTM + j * 16 + frow;
                bf[j] = *(const uint4*)(B + (chunk * TM + (r ^ sw_)) * 16);
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
    issue(0, 0);
    if (nk > 1) issue(1, 1);
    for (int k = 0; k < nk; ++k) {
        if (k + 1 < nk)
            wait_vmcnt<G>();  // stage k landed (this wave's part); stage k+1 may fly
        else
            wait_vmcnt<0>();
        block_barrier();      // every wave's part of stage k landed; compute(k-1) done
        if (k + 2 < nk) issue(k + 2, (k + 2) % NBUF);
        compute(k % NBUF);
    }
    block_barrier();
    conv_epilogue<T, TN, TM, WR, WC, NBUF * BUF>(p, acc, smem, m0, n0, lbias);
}

template <typename T, int TN, int TM, int WR, int WC>
static int launch(const ConvParams& p, int ks, hipStream_t st) {
    dim3 grid((p.M + TM - 1) / TM, (p.cout + TN - 1) / TN);
    // two-slab staging of the wide tiles spilled to scratch (tools/kernel_resources.py): not built
    constexpr bool K2 = !(TM == 256 || TN == 80 || (TN == 128 && TM == 128));
    if (ks == 2) {
        if constexpr (K2) {
            hipLaunchKernelGGL((conv_glds<T, TN, TM, WR, WC, 2>), grid, dim3(256), 0, st, p);
        } else {
            set_error("conv_glds %dx%d: two-slab staging is not built (it spilled)", TN, TM);
            return YXH_EUNSUPPORTED;
        }
    } else {
        hipLaunchKernelGGL((conv_glds<T, TN, TM, WR, WC, 1>), grid, dim3(256), 0, st, p);
    }
    YXH_CHECK_LAUNCH("conv_glds launch");
    return YXH_OK;
}

template <typename T>
static int dispatch(int id, const ConvParams& p, int ks, hipStream_t st) {
    switch (id) {
        case 1: return launch<T, 16, 256, 1, 4>(p, ks, st);
        case 2: return launch<T, 32, 256, 1, 4>(p, ks, st);
        case 3: return launch<T, 32, 128, 1, 4>(p, ks, st);
        case 4: return launch<T, 64, 256, 1, 4>(p, ks, st);
        case 5: return launch<T, 64, 128, 1, 4>(p, ks, st);
        case 6: return launch<T, 64, 64, 2, 2>(p, ks, st);
        case 7: return launch<T, 80, 128, 1, 4>(p, ks, st);
        case 8: return launch<T, 128, 128, 2, 2>(p, ks, st);
        case 9: return launch<T, 128, 64, 2, 2>(p, ks, st);
        default: set_error("glds tile id %d", id); return YXH_EINVAL;
    }
}

int conv_glds_dispatch(int dtype, int id, const ConvParams& p, int ks, hipStream_t st) {
    if (dtype == YXH_BF16) return dispatch<bf16>(id, p, ks, st);
    if (dtype == YXH_F16) return dispatch<f16>(id, p, ks, st);
    return dispatch<float>(id, p, ks, st);
}

}  // namespace yxh
