// conv_pw: pointwise (1x1, stride 1) conv as a persistent streaming GEMM
// (reference network_blocks.py:48-49 BaseConv with ksize 1: the CSP conv1/2/3, SPP
// convs, PAFPN laterals, head stems and the decoded pred convs of yolo_head.py).
//
// The 1x1 layers of YOLOX move ~2 B of activations per MAC-column and are HBM-bound,
// so the design goal is bytes in flight, not MFMA issue:
//  * a block keeps its TN x Cin weight slice resident in LDS for its whole life
//    (loaded once by LDS-DMA) and holds the folded bias in registers;
//  * it walks pixel tiles (TM consecutive output pixels) grid-strided, streaming the
//    activation tile through an NB-deep LDS-DMA ring in 64/128-byte K stages; the
//    stage sequence runs across tile boundaries, so the next tile's loads are in
//    flight while this tile's epilogue stores drain;
//  * waits are counted `s_waitcnt vmcnt(N)` on the loads only (stores issued later are
//    younger, which only makes the wait stricter) and barriers are raw `s_barrier`;
//    nothing in the loop reads global memory into registers, so hipcc never inserts a
//    vmcnt(0) that would drain the ring;
//  * dense sources (image stride = pixels x pixel stride) address the input tile as
//    m * cstride with no division; the PAFPN nearest-x2 upsampled / concatenated
//    sources take the general (b, y, x) path.
#include "conv_common.hpp"

namespace yxh {

namespace {

__device__ __attribute__((aligned(16))) uint4 g_pw_zero[4];

template <int N>
__device__ __forceinline__ void pw_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void pw_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void glds16(const void* g, void* l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

__device__ __forceinline__ int pw_xcd_remap(int id, int nblk) {
    const int q = nblk / 8, r = nblk % 8, xcd = id % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
}

}  // namespace

struct PwArgs {
    int ntiles;   // pixel tiles of TM
    int ntn;      // channel tiles of TN
    int nkc;      // K stages per tile
    int dense0, dense1;
};

template <typename T, int TN, int TM, int KS, int NB, int WBYTES>
__global__ __launch_bounds__(256) void conv_pw(ConvParams p, PwArgs a) {
    constexpr int EPC = Chunk<T>::N;
    constexpr int CPS = 4 * KS;          // 16-byte chunks per row per stage
    constexpr int KST = CPS * EPC;       // K elements per stage
    constexpr int WN = TN / 64, WM = 4 / WN;
    constexpr int WTM = TM / WM;
    constexpr int FR = 4, FC = WTM / 16;
    constexpr int B_SLOTS = TM * CPS;
    static_assert(B_SLOTS % 256 == 0, "stage = whole waves of 64 lanes x 4");
    constexpr int G = B_SLOTS / 256;     // LDS-DMA instructions per wave per stage
    constexpr int BUF = B_SLOTS * 16;
    constexpr int OES = sizeof(T);
    constexpr int OROW = TN * OES + 16;
    constexpr int STAGE_BYTES = TM * OROW;
    __shared__ __attribute__((aligned(16))) char smem[WBYTES + NB * BUF + STAGE_BYTES + TN * 4];
    char* wl = smem;
    char* ring = smem + WBYTES;
    char* stg = ring + NB * BUF;
    float* lbias = (float*)(stg + STAGE_BYTES);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave / WM, wc = wave % WM;
    const int frow = lane & 15, fq = lane >> 4;
    const int L = pw_xcd_remap(blockIdx.x, gridDim.x);
    const int nt = L % a.ntn;
    const int pstart = L / a.ntn, pstep = gridDim.x / a.ntn;
    const int n0 = nt * TN;
    const int mytiles = pstart < a.ntiles ? (a.ntiles - pstart + pstep - 1) / pstep : 0;
    const int nstages = mytiles * a.nkc;

    // folded bias -> LDS before any LDS-DMA is issued (a register load consumed inside
    // the loop would make hipcc drain the ring with vmcnt(0) at its use)
    if (tid < TN) lbias[tid] = n0 + tid < p.cout ? p.bias[n0 + tid] : 0.0f;

    // weights: [kc][chunk][row ^ swz] image of the whole Cin for rows n0..n0+TN
    {
        const int wslots = a.nkc * CPS * TN;
        for (int s0 = 64 * wave; s0 < wslots; s0 += 256) {
            const int s = s0 + lane;
            const void* g = (const void*)g_pw_zero;
            if (s < wslots) {
                const int kc = s / (CPS * TN), rem = s - kc * (CPS * TN);
                const int c = rem / TN, rp = rem - c * TN;
                const int n = n0 + (rp ^ (2 * (c & 3) + (c >> 2)));
                const int ch = kc * KST + c * EPC;
                if (n < p.cout && ch < p.cin) g = (const T*)p.w + (long long)n * p.cin + ch;
            }
            glds16(g, wl + s0 * 16);
        }
    }

    auto issue = [&](int st) {
        const int tl = st / a.nkc, kc = st - tl * a.nkc;
        const int m0 = (pstart + tl * pstep) * TM;
        char* base = ring + (st % NB) * BUF;
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const int s = 64 * (wave + 4 * i) + lane;
            const int c = s / TM, rp = s - c * TM;
            const int m = m0 + (rp ^ (2 * (c & 3) + (c >> 2)));
            int ch = kc * KST + c * EPC;
            const void* g = (const void*)g_pw_zero;
            if (m < p.M && ch < p.cin) {
                int sidx = 0;
                if (p.nsrc == 2 && ch >= p.src0_ch) {
                    sidx = 1;
                    ch -= p.src0_ch;
                }
                const T* sp = (const T*)p.sptr[sidx];
                if (sidx == 0 ? a.dense0 : a.dense1) {
                    g = sp + (long long)m * p.scs[sidx] + ch;
                } else {
                    const int b = m / p.ohw, pix = m - b * p.ohw;
                    const int y = pix / p.out_w, x = pix - y * p.out_w;
                    const int up = p.sup[sidx];
                    g = sp + b * p.sbs[sidx] + ((long long)(y >> up) * p.sw[sidx] + (x >> up)) * p.scs[sidx] + ch;
                }
            }
            glds16(g, base + 64 * 16 * (wave + 4 * i));
        }
    };

    f32x4 acc[FR][FC];
    auto zero_acc = [&]() {
#pragma unroll
        for (int i = 0; i < FR; ++i)
#pragma unroll
            for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    zero_acc();

    auto compute = [&](int st) {
        const int kc = st % a.nkc;
        const char* A = wl + kc * CPS * TN * 16;
        const char* B = ring + (st % NB) * BUF;
#pragma unroll
        for (int sl = 0; sl < KS; ++sl) {
            const int chunk = sl * 4 + fq, sw_ = 2 * fq + sl;
            uint4 af[FR], bf[FC];
#pragma unroll
            for (int i = 0; i < FR; ++i) {
                const int r = wr * 64 + i * 16 + frow;
                af[i] = *(const uint4*)(A + (chunk * TN + (r ^ sw_)) * 16);
            }
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                const int r = wc * WTM + j * 16 + frow;
                bf[j] = *(const uint4*)(B + (chunk * TM + (r ^ sw_)) * 16);
            }
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) Mma<T>::run(acc[i][j], af[i], bf[j]);
        }
    };

    const bool staged = p.vec16 && !p.dst_f32 && (TN * OES) % 16 == 0;
    auto epilogue = [&](int st) {
        const int m0 = (pstart + (st / a.nkc) * pstep) * TM;
        if (staged) {
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                const int pl = wc * WTM + j * 16 + frow;
#pragma unroll
                for (int i = 0; i < FR; ++i) {
                    const int nl = wr * 64 + i * 16 + fq * 4;
                    T t[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        t[r] = from_f32<T>(apply_act<sizeof(T) == 4>(acc[i][j][r] + lbias[nl + r], p.act));
                    char* d = stg + pl * OROW + nl * OES;
                    if constexpr (OES == 2) {
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
            pw_barrier();
            constexpr int CPO = TN * OES / 16;
            const int ncols = min(TN, p.cout - n0) * OES / 16;
            for (int q = tid; q < TM * CPO; q += 256) {
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
                const uint4 u = *(const uint4*)(stg + r * OROW + c * 16);
                *(uint4*)((char*)p.dst + (off + n0) * OES + c * 16) = u;
            }
        } else {
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                const int m = m0 + wc * WTM + j * 16 + frow;
                if (m >= p.M) continue;
                const int b = m / p.ohw, pix = m - b * p.ohw;
                const int oy = pix / p.out_w, ox = pix - oy * p.out_w;
#pragma unroll
                for (int i = 0; i < FR; ++i) {
                    const int nl = wr * 64 + i * 16 + fq * 4, n = n0 + nl;
                    if (n >= p.cout) continue;
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + lbias[nl + r];
                    store4<T>(p, v, n, b, pix, ox, oy);  // no residual on this path: no loads
                }
            }
        }
    };

    constexpr int D = NB - 1;  // stages in flight ahead of the one being computed
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (d < nstages) issue(d);
    for (int st = 0; st < nstages; ++st) {
        // stage st landed: at most min(D-1, stages issued after it) younger stages may fly
        const int younger = min(D - 1, nstages - 1 - st);
        if constexpr (D >= 3) {
            if (younger >= 2) pw_wait_vm<2 * G>();
            else if (younger == 1) pw_wait_vm<G>();
            else pw_wait_vm<0>();
        } else if constexpr (D == 2) {
            if (younger >= 1) pw_wait_vm<G>();
            else pw_wait_vm<0>();
        } else {
            pw_wait_vm<0>();
        }
        pw_barrier();  // all waves' parts landed; stage st-1's slot and the staging tile are free
        if (st + D < nstages) issue(st + D);
        compute(st);
        if (st % a.nkc == a.nkc - 1) {
            epilogue(st);
            zero_acc();
        }
    }
}

template <typename T, int TN, int TM, int KS, int NB, int WBYTES>
static int launch_pw(const ConvParams& p, const PwArgs& a0, hipStream_t st) {
    constexpr int es = sizeof(T);
    constexpr int CPS = 4 * KS;
    constexpr int lds = WBYTES + NB * TM * CPS * 16 + TM * (TN * es + 16) + TN * 4;
    if constexpr (lds > 160 * 1024) {
        set_error("conv_pw variant needs more than 160 KiB of LDS");
        return YXH_EUNSUPPORTED;
    } else {
    PwArgs a = a0;
    a.ntn = (p.cout + TN - 1) / TN;
    a.ntiles = (p.M + TM - 1) / TM;
    const int kst = CPS * (16 / es);
    a.nkc = (p.cin + kst - 1) / kst;
    if ((long long)a.nkc * kst * TN * es > WBYTES) {
        set_error("conv_pw: %d x %d weights exceed the %d-byte LDS slice", TN, a.nkc * kst, WBYTES);
        return YXH_EUNSUPPORTED;
    }
    const int occ = max(1, (160 * 1024) / lds);
    const long long want = (long long)a.ntiles * a.ntn;
    long long blocks = (long long)256 * occ;
    blocks = blocks / a.ntn * a.ntn;  // whole channel-tile groups
    if (blocks > want) blocks = want;
    if (blocks < a.ntn) blocks = a.ntn;
    hipLaunchKernelGGL((conv_pw<T, TN, TM, KS, NB, WBYTES>), dim3((unsigned)blocks), dim3(256), 0, st, p, a);
    YXH_CHECK_LAUNCH("conv_pw launch");
    return YXH_OK;
    }
}

template <typename T, int TN, int TM, int NB>
static int pw_pick(const ConvParams& p, int ks, const PwArgs& a, hipStream_t st) {
    // smallest resident-weight slice that holds TN x Cin (16 or 64 KiB)
    const int kst = 4 * ks * (16 / (int)sizeof(T));
    const long long wbytes = (long long)((p.cin + kst - 1) / kst) * kst * TN * (long long)sizeof(T);
    if (wbytes <= 16 * 1024)
        return ks == 2 ? launch_pw<T, TN, TM, 2, NB, 16 * 1024>(p, a, st) : launch_pw<T, TN, TM, 1, NB, 16 * 1024>(p, a, st);
    return ks == 2 ? launch_pw<T, TN, TM, 2, NB, 64 * 1024>(p, a, st) : launch_pw<T, TN, TM, 1, NB, 64 * 1024>(p, a, st);
}

template <typename T>
static int pw_dispatch_t(int id, const ConvParams& p, int ks, const PwArgs& a, hipStream_t st) {
    // id -> (TN, TM, NB); ks = 64/128-byte K stages
    switch (id) {
        case 1: return pw_pick<T, 64, 64, 3>(p, ks, a, st);
        case 2: return pw_pick<T, 64, 128, 3>(p, ks, a, st);
        case 3: return pw_pick<T, 128, 64, 3>(p, ks, a, st);
        case 4: return pw_pick<T, 128, 128, 3>(p, ks, a, st);
        case 5: return pw_pick<T, 64, 64, 4>(p, ks, a, st);
        case 6: return pw_pick<T, 128, 64, 4>(p, ks, a, st);
        default: set_error("conv_pw tile id %d", id); return YXH_EINVAL;
    }
}

int conv_pw_dispatch(int dtype, int id, const ConvParams& p, int ks, hipStream_t st) {
    if (p.taps != 1 || p.stride != 1 || p.pad != 0 || p.res) {
        set_error("conv_pw needs a 1x1 stride-1 conv without residual");
        return YXH_EUNSUPPORTED;
    }
    PwArgs a{};
    a.dense0 = !p.sup[0] && p.sw[0] == p.out_w && p.sbs[0] == (long long)p.ohw * p.scs[0];
    a.dense1 = p.nsrc == 2 && !p.sup[1] && p.sw[1] == p.out_w && p.sbs[1] == (long long)p.ohw * p.scs[1];
    if (dtype == YXH_BF16) return pw_dispatch_t<bf16>(id, p, ks, a, st);
    if (dtype == YXH_F16) return pw_dispatch_t<f16>(id, p, ks, a, st);
    set_error("conv_pw is built for bf16/f16 only");
    return YXH_EUNSUPPORTED;
}

}  // namespace yxh
