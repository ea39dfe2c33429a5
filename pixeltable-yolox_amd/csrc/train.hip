// Training-side kernels of the YOLOX hot path on gfx950 (MI355X): everything the
// backward pass of YoloxModule needs besides the data-gradient convolutions (those
// run on the forward conv kernels with transposed/flipped weights, yxh_pack_dgrad_weight,
// and a zero-dilated source for stride 2).
//
//  bn_stats        : BatchNorm2d training statistics (network_blocks.py:44-49 BaseConv.bn,
//                    eps/momentum from config.py:162-166): per-channel shifted sums in a
//                    fixed-order two-stage reduction, then mean / invstd / folded
//                    scale+shift and the running-stat update (unbiased var, momentum).
//  bn_act_fwd      : y*scale+shift -> act (SiLU/ReLU/LReLU) (+ Bottleneck residual,
//                    network_blocks.py:97-99) into a channel-slice view.
//  bn_act_bwd      : act' and BatchNorm backward: dgamma = sum dz*xhat, dbeta = sum dz,
//                    dx = gamma*invstd*(dz - dbeta/M - xhat*dgamma/M).
//  conv_wgrad      : dW[n][c][ky][kx] = sum_pixels dY[n] * X[c](tap) on MFMA: both
//                    operands are pixel-major (NHWC), so the loader transposes 16-byte
//                    chunks in registers (v_perm) and the LDS image is the forward
//                    kernel's [K chunk][row] layout with K = pixels; split over pixel
//                    ranges, fp32 atomics into the weight gradient.
//  spp_bwd         : max_pool2d(5/9/13, s1) backward (first max in row-major scan, as
//                    torch) + the identity branch of SPPBottleneck's concat.
//  upsample_bwd    : nn.Upsample(nearest x2) backward (2x2 sums), accumulated.
//  channel_sum     : bias gradients of the head's pred convs.
#include <cstdlib>

#include "conv_common.hpp"

namespace yxh {

// A strided NHWC view (yxh_src): pixel m = b*HW + pix -> b*bs + pix*cs elements.
struct TView {
    const void* ptr;
    int C, cs, HW;
    long long bs;
};

__device__ __forceinline__ long long vofs(const TView& v, int m) {
    if (v.bs == (long long)v.HW * v.cs) return (long long)m * v.cs;  // images back to back: no (b, pix) split
    const int b = m / v.HW, pix = m - b * v.HW;
    return (long long)b * v.bs + (long long)pix * v.cs;
}

template <typename T, int N>
__device__ __forceinline__ void load_f(const T* p, float (&o)[N]) {
    if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int q = 0; q < N; q += 4) {
            const float4 u = *(const float4*)(p + q);
            o[q] = u.x; o[q + 1] = u.y; o[q + 2] = u.z; o[q + 3] = u.w;
        }
    } else {
        static_assert(N % 8 == 0, "16-bit chunks");
#pragma unroll
        for (int q = 0; q < N; q += 8) {
            const uint4 u = *(const uint4*)(p + q);
            T t[8];
            __builtin_memcpy(t, &u, 16);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[q + e] = to_f32(t[e]);
        }
    }
}

template <typename T, int N>
__device__ __forceinline__ void store_f(T* p, const float (&o)[N]) {
    if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int q = 0; q < N; q += 4) *(float4*)(p + q) = make_float4(o[q], o[q + 1], o[q + 2], o[q + 3]);
    } else {
#pragma unroll
        for (int q = 0; q < N; q += 8) {
            T t[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] = from_f32<T>(o[q + e]);
            uint4 u;
            __builtin_memcpy(&u, t, 16);
            *(uint4*)(p + q) = u;
        }
    }
}

// d act(z) / dz
template <bool PRECISE>
__device__ __forceinline__ float act_grad(float z, int act) {
    switch (act) {
        case YXH_ACT_SILU: {
            const float s = PRECISE ? 1.0f / (1.0f + expf(-z)) : __builtin_amdgcn_rcpf(1.0f + __expf(-z));
            return s * (1.0f + z * (1.0f - s));
        }
        case YXH_ACT_RELU: return z > 0.0f ? 1.0f : 0.0f;
        case YXH_ACT_LRELU: return z > 0.0f ? 1.0f : 0.1f;
        default: return 1.0f;
    }
}

// ------------------------------------------------------------------ reductions
// Stage 1: block b reduces rows [b*rpb, (b+1)*rpb) into partial[b][2][C].
// Thread = (row lane, channel chunk of EPC channels); rows stride by the row lanes.
enum { RED_STATS = 0, RED_BWD = 1, RED_SUM = 2 };

struct RedArgs {
    TView x;          // activation (T): y for STATS/BWD, x for SUM
    TView g;          // fp32 gradient (BWD)
    const float* st;  // stats [4][C] = mean, invstd, scale, shift (BWD)
    int act, M, rpb;
    float* partial;
};

template <typename T, int MODE>
__global__ __launch_bounds__(256) void chan_reduce(RedArgs a) {
    constexpr int EPC = Chunk<T>::N;
    // one staging buffer for both sums in turn (8 KiB at 16 bits): beside the side stream's weight
    // gradients (up to ~140 KiB of LDS per CU) a 16 KiB block often found no room on a CU
    __shared__ float red[256 * EPC];
    // blockIdx.y = channel group of up to 256 16-byte chunks (yolox_x fp32: 1280 channels)
    const int C = a.x.C, cg = blockIdx.y * 256 * EPC, CL = min(C - cg, 256 * EPC), nch = CL / EPC;
    const int tid = threadIdx.x;
    const int q = tid % nch, rl = tid / nch, rpi = 256 / nch;
    float s1[EPC], s2[EPC], sh[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) s1[e] = s2[e] = sh[e] = 0.0f;
    const int c0 = cg + q * EPC;
    const T* xp = (const T*)a.x.ptr;
    if (MODE == RED_STATS && rl < rpi) {
        load_f<T, EPC>(xp + c0, sh);  // shift = pixel 0 (cancellation guard)
        if (blockIdx.x == 0 && rl == 0)
#pragma unroll
            for (int e = 0; e < EPC; ++e) a.partial[(long long)gridDim.x * 2 * C + c0 + e] = sh[e];
    }
    float sc[EPC], sf[EPC], mu[EPC], is[EPC];
    if (MODE == RED_BWD) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
            mu[e] = a.st[c0 + e];
            is[e] = a.st[C + c0 + e];
            sc[e] = a.st[2 * C + c0 + e];
            sf[e] = a.st[3 * C + c0 + e];
        }
    }
    const int r0 = blockIdx.x * a.rpb, r1 = min(a.M, r0 + a.rpb);
    auto accum = [&](const float (&v)[EPC], const float (&gv)[EPC]) {
        if (MODE == RED_STATS) {
#pragma unroll
            for (int e = 0; e < EPC; ++e) {
                const float d = v[e] - sh[e];
                s1[e] += d;
                s2[e] += d * d;
            }
        } else if (MODE == RED_SUM) {
#pragma unroll
            for (int e = 0; e < EPC; ++e) s1[e] += v[e];
        } else {
#pragma unroll
            for (int e = 0; e < EPC; ++e) {
                const float z = v[e] * sc[e] + sf[e];
                const float dz = gv[e] * act_grad<sizeof(T) == 4>(z, a.act);
                s1[e] += dz;
                s2[e] += dz * ((v[e] - mu[e]) * is[e]);
            }
        }
    };
    // U rows in flight per thread: all loads first, then the rows in order (the same
    // fixed summation order as one row at a time).  BWD holds y, the fp32 gradient and four
    // coefficient rows per channel: at U = 4 the 16-bit form took 159 VGPRs (3 waves per SIMD, so
    // the 1024-block grid ran in two rounds: the slowest kernel of the configs[4] step's main
    // stream); fp32 (4 channels per 16-byte chunk) fits 91 at U = 4
    constexpr int U = MODE == RED_BWD && sizeof(T) == 2 ? 2 : 4;
    if (rl < rpi) {
        int r = r0 + rl;
        for (; r + (U - 1) * rpi < r1; r += U * rpi) {
            float v[U][EPC], gv[U][EPC] = {};
#pragma unroll
            for (int u = 0; u < U; ++u) {
                load_f<T, EPC>(xp + vofs(a.x, r + u * rpi) + c0, v[u]);
                if (MODE == RED_BWD) load_f<float, EPC>((const float*)a.g.ptr + vofs(a.g, r + u * rpi) + c0, gv[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) accum(v[u], gv[u]);
        }
        for (; r < r1; r += rpi) {
            float v[EPC], gv[EPC] = {};
            load_f<T, EPC>(xp + vofs(a.x, r) + c0, v);
            if (MODE == RED_BWD) load_f<float, EPC>((const float*)a.g.ptr + vofs(a.g, r) + c0, gv);
            accum(v, gv);
        }
    }
    // thread t < C sums channel t over the row lanes (fixed order: deterministic), Σ1 then Σ2
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (k) __syncthreads();  // every thread is done reading the Σ1 stage
#pragma unroll
        for (int e = 0; e < EPC; ++e) red[tid * EPC + e] = k ? s2[e] : s1[e];
        __syncthreads();
        for (int c = tid; c < CL; c += 256) {
            const int qq = c / EPC, e = c - qq * EPC;
            float t = 0.0f;
            for (int l = 0; l < rpi; ++l) t += red[(l * nch + qq) * EPC + e];
            a.partial[((long long)blockIdx.x * 2 + k) * C + cg + c] = t;
        }
    }
}

struct FinArgs {
    const float* partial;  // [nblk][2][C] (+ [C] shift row for STATS)
    int nblk, C, M, mode;
    const float *gamma, *beta;
    float *rmean, *rvar;
    float eps, momentum;
    float* stats;        // STATS out [4][C] = mean, invstd, scale, shift
    float *out0, *out1;  // BWD: dgamma, dbeta; SUM: out0
    const float* st_in;  // BWD: the forward's stats [4][C]
    float* coef;         // BWD out [3][C]: dx = k1*dz + k2*(y - mean) + k3
};

// 4 channels per block, a wave per channel: each lane sums its strided share of the
// per-block partials in double (eight independent chains, so the loads of eight rows are in
// flight at once: the kernel is latency-bound, <= 512 partials per channel), then a
// fixed-order tree over the lanes: deterministic.
__global__ __launch_bounds__(256) void chan_finalize(FinArgs f) {
    __shared__ double red[2][256];
    const int j = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + j;
    // eight independent chains: the <= 512 partials of a channel (red_blocks) arrive in ONE round of
    // loads per lane instead of two dependent rounds
    constexpr int U = 8;
    double a1[U], a2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a1[u] = a2[u] = 0.0;
    if (c < f.C) {
        const long long rs = 2LL * f.C;  // partial row stride (one block's [2][C])
        const float* p0 = f.partial + c;
        for (int b = lane; b < f.nblk; b += 64 * U) {
            float v1[U], v2[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int bb = b + 64 * u;
                v1[u] = bb < f.nblk ? p0[(long long)bb * rs] : 0.0f;
                v2[u] = bb < f.nblk ? p0[(long long)bb * rs + f.C] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                a1[u] += v1[u];
                a2[u] += v2[u];
            }
        }
    }
    red[0][threadIdx.x] = ((a1[0] + a1[1]) + (a1[2] + a1[3])) + ((a1[4] + a1[5]) + (a1[6] + a1[7]));
    red[1][threadIdx.x] = ((a2[0] + a2[1]) + (a2[2] + a2[3])) + ((a2[4] + a2[5]) + (a2[6] + a2[7]));
    __syncthreads();
    for (int s = 32; s > 0; s >>= 1) {
        if (lane < s) {
            red[0][threadIdx.x] += red[0][threadIdx.x + s];
            red[1][threadIdx.x] += red[1][threadIdx.x + s];
        }
        __syncthreads();
    }
    if (lane != 0 || c >= f.C) return;
    double t1, t2;
    t1 = red[0][threadIdx.x];
    t2 = red[1][threadIdx.x];
    if (f.mode == RED_STATS) {
        const double m1 = t1 / f.M;
        const double mean = (double)f.partial[(long long)f.nblk * 2 * f.C + c] + m1;
        double var = t2 / f.M - m1 * m1;
        if (var < 0) var = 0;
        const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
        const float g = f.gamma ? f.gamma[c] : 1.0f, be = f.beta ? f.beta[c] : 0.0f;
        const float scale = g * invstd;
        f.stats[c] = (float)mean;
        f.stats[f.C + c] = invstd;
        f.stats[2 * f.C + c] = scale;
        f.stats[3 * f.C + c] = be - (float)mean * scale;
        if (f.rmean) {
            const float mo = f.momentum;
            f.rmean[c] = (1.0f - mo) * f.rmean[c] + mo * (float)mean;
            const double unb = f.M > 1 ? var * f.M / (f.M - 1) : var;
            f.rvar[c] = (1.0f - mo) * f.rvar[c] + mo * (float)unb;
        }
    } else if (f.mode == RED_BWD) {
        f.out0[c] = (float)t2;  // dgamma = sum dz * xhat
        f.out1[c] = (float)t1;  // dbeta = sum dz
        const float is = f.st_in[f.C + c], inv_m = 1.0f / (float)f.M;
        const float k1 = (f.gamma ? f.gamma[c] : 1.0f) * is;
        f.coef[c] = k1;
        f.coef[f.C + c] = -k1 * is * ((float)t2 * inv_m);
        f.coef[2 * f.C + c] = -k1 * ((float)t1 * inv_m);
    } else {
        f.out0[c] = (float)t1;
    }
}

// ------------------------------------------------------------------ elementwise
template <typename T>
__global__ __launch_bounds__(256) void bn_act_fwd(TView y, const float* st, int act, TView res, TView out, int M) {
    constexpr int EPC = Chunk<T>::N;
    const int C = y.C, nch = C / EPC;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)M * nch) return;
    const int m = (int)(idx / nch), c0 = (int)(idx - (long long)m * nch) * EPC;
    float v[EPC], sc[EPC], sf[EPC];
    load_f<T, EPC>((const T*)y.ptr + vofs(y, m) + c0, v);
    load_f<float, EPC>(st + 2 * C + c0, sc);
    load_f<float, EPC>(st + 3 * C + c0, sf);
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
        const float z = v[e] * sc[e] + sf[e];
        // training keeps the IEEE-divide SiLU on every dtype: the SimOTA assignment
        // downstream is discrete, so the bf16/f16 step stays bit-stable across builds
        v[e] = (act == YXH_ACT_SILU && sizeof(T) != 4) ? z / (1.0f + __expf(-z)) : apply_act<sizeof(T) == 4>(z, act);
    }
    if (res.ptr) {
        float r[EPC];
        load_f<T, EPC>((const T*)res.ptr + vofs(res, m) + c0, r);
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] += r[e];
    }
    store_f<T, EPC>((T*)out.ptr + vofs(out, m) + c0, v);
}

// dx = k1*dz + k2*(y - mean) + k3 with the per-channel coefficients chan_finalize derived
// from dgamma / dbeta (BatchNorm's backward with batch statistics).
template <typename T>
__global__ __launch_bounds__(256) void bn_act_bwd_apply(TView y, TView g, const float* st, const float* coef,
                                                       int act, int M, T* dx) {
    constexpr int EPC = Chunk<T>::N;
    const int C = y.C, nch = C / EPC;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)M * nch) return;
    const int m = (int)(idx / nch), c0 = (int)(idx - (long long)m * nch) * EPC;
    float v[EPC], gv[EPC], o[EPC], mu[EPC], sc[EPC], sf[EPC], k1[EPC], k2[EPC], k3[EPC];
    load_f<T, EPC>((const T*)y.ptr + vofs(y, m) + c0, v);
    load_f<float, EPC>((const float*)g.ptr + vofs(g, m) + c0, gv);
    load_f<float, EPC>(st + c0, mu);
    load_f<float, EPC>(st + 2 * C + c0, sc);
    load_f<float, EPC>(st + 3 * C + c0, sf);
    load_f<float, EPC>(coef + c0, k1);
    load_f<float, EPC>(coef + C + c0, k2);
    load_f<float, EPC>(coef + 2 * C + c0, k3);
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
        const float z = v[e] * sc[e] + sf[e];
        const float dz = gv[e] * act_grad<sizeof(T) == 4>(z, act);
        o[e] = k1[e] * dz + k2[e] * (v[e] - mu[e]) + k3[e];
    }
    store_f<T, EPC>(dx + (long long)m * C + c0, o);
}

// ------------------------------------------------------------------ weight gradient
struct WgradParams {
    int in_h, in_w, out_h, out_w, cin, cout, kh, kw, stride, pad, ohw, M;
    int nsrc, src0_ch, B;
    const void* sptr[2];
    int scs[2], sw[2], sup[2];
    long long sbs[2];
    const void* dy;
    int dycs;
    long long dybs;
    float* dw;
    int cin_store;
    int sps, nst;  // stages per split, total pixel stages
    int ntc;       // channel tiles per tap
    int dych;      // channels of the dy view (loads past them read the zero chunk)
    float* ws;     // fp32 tiles 17-20: per-split partial dW (yxh_wgrad_desc.workspace), or null
    long long ws_elems;
};

__device__ __attribute__((aligned(16))) uint4 g_wg_zero[4];

// In-register transpose of an EPC x EPC block of T: a[e] = EPC channels of pixel e ->
// a[j] = EPC pixels of channel j.
__device__ __forceinline__ void transpose_chunks(uint4 (&a)[8]) {  // 16-bit elements
    uint32_t w[8][4];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        w[e][0] = a[e].x; w[e][1] = a[e].y; w[e][2] = a[e].z; w[e][3] = a[e].w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t sel = (j & 1) ? 0x07060302u : 0x05040100u;
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = __builtin_amdgcn_perm(w[2 * q + 1][j >> 1], w[2 * q][j >> 1], sel);
        a[j] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}
__device__ __forceinline__ void transpose_chunks(uint4 (&a)[4]) {  // 32-bit elements
    uint4 b[4];
    b[0] = make_uint4(a[0].x, a[1].x, a[2].x, a[3].x);
    b[1] = make_uint4(a[0].y, a[1].y, a[2].y, a[3].y);
    b[2] = make_uint4(a[0].z, a[1].z, a[2].z, a[3].z);
    b[3] = make_uint4(a[0].w, a[1].w, a[2].w, a[3].w);
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = b[j];
}

// LDS row placement of the wgrad image: the chunk XOR of the forward kernel plus
// (r >> 3) & 7 on the low bits.  A loader lane writes 8 consecutive rows of one chunk and
// neighbouring lanes are 8 rows apart, so without the second term every lane of a
// ds_write_b128 hits the same 32-bank group; with it 8 lanes cover all banks.  A fragment
// read (16 consecutive rows, one chunk) stays a permutation of one 256-byte block.
__device__ __forceinline__ int wg_row(int r, int sw) { return r ^ sw ^ ((r >> 3) & 7); }

template <typename T, int TN, int TM, int WR, int WC, int KS>
__global__ __launch_bounds__(256) void conv_wgrad(WgradParams p) {
    constexpr int EPC = Chunk<T>::N;
    constexpr int CPR = 4 * KS;           // 16-byte chunks (of EPC pixels) per row per stage
    static_assert(CPR * EPC > 0, "stage");
    constexpr int NA = (TN / EPC) * CPR;  // transpose items: A = dY rows (cout)
    constexpr int NB = (TM / EPC) * CPR;  //                  B = X rows (cin of the tap)
    constexpr int NIT = (NA + NB + 255) / 256;
    constexpr int WTN = TN / WR, WTM = TM / WC;
    constexpr int FR = WTN / 16, FC = WTM / 16;
    constexpr int A_BYTES = TN * CPR * 16, B_BYTES = TM * CPR * 16;
    constexpr int BUF = A_BYTES + B_BYTES;
    static_assert(WR * WC == 4 && FR >= 1 && FC >= 1, "tile");
    __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WC, wc = wave % WC;
    const int n0 = blockIdx.y * TN;
    const int tap = blockIdx.z / p.ntc, c0 = (blockIdx.z - tap * p.ntc) * TM;
    const int ky = tap / p.kw, kx = tap - ky * p.kw;
    const int st0 = blockIdx.x * p.sps, st1 = min(p.nst, st0 + p.sps);

    uint4 rg[NIT][EPC];
    // K runs over "runs": EPC consecutive output pixels of one output row (rows padded to
    // a multiple of EPC), so a run is one (b, oy, ox0) decomposition and its input pixels
    // for the tap are one input row at stride `stride`.  Loads are branch-free: invalid
    // lanes read a zero chunk.
    const int rpr = (p.out_w + EPC - 1) / EPC, rpi = rpr * p.out_h;
    auto gload = [&](int stg) {
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
            const int it = tid + 256 * i;
            if (it >= NA + NB) continue;
            const bool isa = it < NA;
            const int jt = isa ? it : it - NA;
            const int rows = isa ? TN : TM;
            const int ci = jt % (rows / EPC), pc = jt / (rows / EPC);
            const int R = stg * CPR + pc;
            const int b = R / rpi, rem = R - b * rpi;
            const int oy = rem / rpr, ox0 = (rem - oy * rpr) * EPC;
            const bool run_ok = b < p.B;
            const T* zero = (const T*)g_wg_zero;
            if (isa) {
                const int n = n0 + ci * EPC;
                const bool ok = run_ok && n < p.cout;
                const T* base = (const T*)p.dy + (ok ? (long long)b * p.dybs + n : 0);
                const int o0 = (oy * p.out_w + ox0) * p.dycs;
#pragma unroll
                for (int e = 0; e < EPC; ++e) {
                    const bool v = ok && ox0 + e < p.out_w;
                    rg[i][e] = *(const uint4*)(v ? base + o0 + e * p.dycs : zero);
                }
            } else {
                int c = c0 + ci * EPC;
                int s = 0;
                if (p.nsrc == 2 && c >= p.src0_ch) {
                    s = 1;
                    c -= p.src0_ch;
                }
                const int iy = oy * p.stride - p.pad + ky;
                const bool ok = run_ok && c0 + ci * EPC < p.cin && iy >= 0 && iy < p.in_h;
                const int up = p.sup[s], scs = p.scs[s];
                const T* base = (const T*)p.sptr[s] + (ok ? (long long)b * p.sbs[s] + c : 0);
                const int rowoff = (iy >> up) * p.sw[s];
#pragma unroll
                for (int e = 0; e < EPC; ++e) {
                    const int ix = (ox0 + e) * p.stride - p.pad + kx;
                    const bool v = ok && ox0 + e < p.out_w && ix >= 0 && ix < p.in_w;
                    rg[i][e] = *(const uint4*)(v ? base + (rowoff + (ix >> up)) * scs : zero);
                }
            }
        }
    };
    auto lstore = [&](int buf) {
        char* A = smem + buf * BUF;
        char* B = A + A_BYTES;
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
            const int it = tid + 256 * i;
            if (it >= NA + NB) continue;
            transpose_chunks(rg[i]);
            const bool isa = it < NA;
            const int jt = isa ? it : it - NA;
            const int rows = isa ? TN : TM;
            const int ci = jt % (rows / EPC), pc = jt / (rows / EPC);
            const int sw_ = 2 * (pc & 3) + (pc >> 2);
            char* base = isa ? A : B;
#pragma unroll
            for (int j = 0; j < EPC; ++j) {
                const int r = ci * EPC + j;
                *(uint4*)(base + (pc * rows + wg_row(r, sw_)) * 16) = rg[i][j];
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
        for (int s = 0; s < KS; ++s) {
            const int chunk = s * 4 + fq, sw_ = 2 * fq + s;
            uint4 af[FR], bf[FC];
#pragma unroll
            for (int i = 0; i < FR; ++i) af[i] = *(const uint4*)(A + (chunk * TN + wg_row(wr * WTN + i * 16 + frow, sw_)) * 16);
#pragma unroll
            for (int j = 0; j < FC; ++j) bf[j] = *(const uint4*)(B + (chunk * TM + wg_row(wc * WTM + j * 16 + frow, sw_)) * 16);
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) Mma<T>::run(acc[i][j], af[i], bf[j]);
        }
    };

    if (st0 < st1) {
        gload(st0);
        lstore(0);
        __syncthreads();
        for (int k = st0; k < st1; ++k) {
            const int cur = (k - st0) & 1;
            if (k + 1 < st1) gload(k + 1);
            compute(cur);
            if (k + 1 < st1) lstore(cur ^ 1);
            __syncthreads();
        }
    }
    // dW (torch layout [cout][cin_store][kh][kw]) += acc
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) {
            const int c = c0 + wc * WTM + j * 16 + frow;
            if (c >= p.cin_store) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n0 + wr * WTN + i * 16 + fq * 4 + r;
                if (n < p.cout) {
                    const long long e = (((long long)n * p.cin_store + c) * p.kh + ky) * p.kw + kx;
                    if (p.ws) p.ws[(long long)blockIdx.x * p.cout * p.cin_store * p.kh * p.kw + e] = acc[i][j][r];
                    else atomicAdd(p.dw + e, acc[i][j][r]);
                }
            }
        }
}

// ------------------------------------------------------------------ weight gradient, all nine taps
// fp32 3x3 (pad 1, stride S) weight gradient with the nine taps of one block sharing its
// staged operands: conv_wgrad stages dy and x once PER TAP (nine blocks re-read the same
// pixels; the 320x320 stem took 0.9 ms at 1.5 TB/s of re-reads).  Here a block owns
// dW[n0, n0+TN) x [c0, c0+TC) x 9 taps and walks pixel tiles of TY output rows x 16
// columns of one image:
//  * dy tile -> LDS transposed, [TN][TM] (pixel-major rows: an MFMA K step = 4 pixels);
//    x halo tile ((TY-1)*S+3 rows x 15*S+3 columns) -> LDS transposed, [TC][row][col];
//    next tile's global loads are in registers while this tile computes;
//  * per output row: the A fragments (dy) are read once and serve all nine taps; the B
//    fragment of tap (ky, kx) is the halo row ty*S + ky at columns tx*S + kx;
//  * wave (wn, wc) owns a TN/WN x TC/WC slice of every tap: no cross-wave reduction;
//    the block's totals go to dW (torch layout) with fp32 atomics (dW pre-zeroed).
// v_mfma_f32_16x16x4f32 (Mma<float>): 4 MFMAs per 16-pixel row and fragment pair.
template <int S, int TN, int TC, int WN, int WC, int TY>
__global__ __launch_bounds__(64 * WN * WC) void conv_wgrad9(WgradParams p, int tiles_x, int tiles_y, int tpb) {
    constexpr int NT = 64 * WN * WC, TX = 16, TM = TX * TY;
    constexpr int HX = (TX - 1) * S + 3, HY = (TY - 1) * S + 3;
    constexpr int DYS = TM + 4;        // dyT row stride (floats; 16-byte aligned rows)
    constexpr int XRS = HX + 1;        // xT row stride
    constexpr int XCS = HY * XRS + 4;  // xT channel stride
    constexpr int WTN = TN / WN, WTC = TC / WC, FRN = WTN / 16, FRC = WTC / 16;
    constexpr int N4 = TN / 4, C4 = TC / 4;
    constexpr int NDY = TM * N4, NX = HY * HX * C4;
    constexpr int IDY = (NDY + NT - 1) / NT, IX = (NX + NT - 1) / NT;
    static_assert(FRN >= 1 && FRC >= 1 && WTN % 16 == 0 && WTC % 16 == 0, "tile");
    __shared__ __attribute__((aligned(16))) float dyT[TN * DYS];
    __shared__ __attribute__((aligned(16))) float xT[TC * XCS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wn = wave / WC, wc = wave % WC;
    const int n0 = blockIdx.y * TN, c0 = blockIdx.z * TC;
    const int per_img = tiles_y * tiles_x;
    const int T = p.B * per_img;
    const int t0 = blockIdx.x * tpb, t1 = min(T, t0 + tpb);
    const int OH = p.out_h, OW = p.out_w;
    const float* dyp = (const float*)p.dy;
    const float* xp = (const float*)p.sptr[0];
    const int scs = p.scs[0], sw = p.sw[0];

    float4 rdy[IDY], rx[IX];
    auto gload = [&](int t) {
        const int b = t / per_img, r = t - b * per_img;
        const int tyi = r / tiles_x, txi = r - tyi * tiles_x;
        const int oy0 = tyi * TY, ox0 = txi * TX;
#pragma unroll
        for (int i = 0; i < IDY; ++i) {
            const int q = tid + NT * i;
            const int pl = q / N4, n = n0 + 4 * (q - pl * N4);
            const int oy = oy0 + pl / TX, ox = ox0 + pl % TX;
            const bool ok = q < NDY && oy < OH && ox < OW && n < p.dych;
            rdy[i] = ok ? *(const float4*)(dyp + (long long)b * p.dybs + (long long)(oy * OW + ox) * p.dycs + n)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < IX; ++i) {
            const int q = tid + NT * i;
            const int hp = q / C4, c = c0 + 4 * (q - hp * C4);
            const int hy = hp / HX, hx = hp - hy * HX;
            const int iy = oy0 * S - 1 + hy, ix = ox0 * S - 1 + hx;
            const bool ok = q < NX && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w && c < p.cin;
            rx[i] = ok ? *(const float4*)(xp + (long long)b * p.sbs[0] + (long long)(iy * sw + ix) * scs + c)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int i = 0; i < IDY; ++i) {
            const int q = tid + NT * i;
            if (q >= NDY) continue;
            const int pl = q / N4, n = 4 * (q - pl * N4);
            dyT[(n + 0) * DYS + pl] = rdy[i].x;
            dyT[(n + 1) * DYS + pl] = rdy[i].y;
            dyT[(n + 2) * DYS + pl] = rdy[i].z;
            dyT[(n + 3) * DYS + pl] = rdy[i].w;
        }
#pragma unroll
        for (int i = 0; i < IX; ++i) {
            const int q = tid + NT * i;
            if (q >= NX) continue;
            const int hp = q / C4, c = 4 * (q - hp * C4);
            const int hy = hp / HX, hx = hp - hy * HX;
            const int o = hy * XRS + hx;
            xT[(c + 0) * XCS + o] = rx[i].x;
            xT[(c + 1) * XCS + o] = rx[i].y;
            xT[(c + 2) * XCS + o] = rx[i].z;
            xT[(c + 3) * XCS + o] = rx[i].w;
        }
    };

    f32x4 acc[9][FRN][FRC];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < FRN; ++i)
#pragma unroll
            for (int j = 0; j < FRC; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int frow = lane & 15, fq = lane >> 4;

    auto compute = [&]() {
        for (int ty = 0; ty < TY; ++ty) {
            uint4 af[FRN];
#pragma unroll
            for (int i = 0; i < FRN; ++i)
                af[i] = *(const uint4*)&dyT[(wn * WTN + i * 16 + frow) * DYS + ty * TX + 4 * fq];
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
#pragma unroll
                    for (int j = 0; j < FRC; ++j) {
                        const float* xr = &xT[(wc * WTC + j * 16 + frow) * XCS + (ty * S + ky) * XRS + 4 * fq * S + kx];
                        const uint4 bf = make_uint4(__float_as_uint(xr[0]), __float_as_uint(xr[S]),
                                                    __float_as_uint(xr[2 * S]), __float_as_uint(xr[3 * S]));
#pragma unroll
                        for (int i = 0; i < FRN; ++i) Mma<float>::run(acc[ky * 3 + kx][i][j], af[i], bf);
                    }
                }
        }
    };

    if (t0 < t1) {
        gload(t0);
        lstore();
        __syncthreads();
        for (int t = t0; t < t1; ++t) {
            if (t + 1 < t1) gload(t + 1);
            compute();
            __syncthreads();
            if (t + 1 < t1) {
                lstore();
                __syncthreads();
            }
        }
    }
    // dW (torch layout [cout][cin_store][3][3]) += acc
#pragma unroll
    for (int i = 0; i < FRN; ++i)
#pragma unroll
        for (int j = 0; j < FRC; ++j) {
            const int c = c0 + wc * WTC + j * 16 + frow;
            if (c >= p.cin_store) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n0 + wn * WTN + i * 16 + fq * 4 + r;
                if (n >= p.cout) continue;
                const long long e = ((long long)n * p.cin_store + c) * 9;
                if (p.ws) {
                    float* d = p.ws + (long long)blockIdx.x * p.cout * p.cin_store * 9 + e;
#pragma unroll
                    for (int t = 0; t < 9; ++t) d[t] = acc[t][i][j][r];
                } else {
#pragma unroll
                    for (int t = 0; t < 9; ++t) atomicAdd(p.dw + e + t, acc[t][i][j][r]);
                }
            }
        }
}

__global__ __launch_bounds__(256) void wgrad_reduce(const float* ws, int splits, long long ne, float* dw);

// Per-split partials (yxh_wgrad_desc.workspace): the split count a launcher wants, capped so every
// split's partial dW fits the workspace and `cap_elems` floats (tiles 1-24: 16 MiB, beyond which
// writing and summing the partials cost more than the extra blocks gained; the nine-tap 16-bit
// tiles 25-28 hold all nine taps per split and take 64 MiB, or wide 3x3s get ~100 blocks); p.ws is
// cleared when not even one split fits (atomics).
static long long ws_cap_splits(WgradParams& p, long long splits, long long cap_elems = 4LL << 20) {
    if (!p.ws) return splits;
    const long long ne = (long long)p.cout * p.cin_store * p.kh * p.kw;
    const long long cap = std::min<long long>(p.ws_elems, cap_elems) / ne;
    if (cap < 1) {
        p.ws = nullptr;
        return splits;
    }
    return std::min(splits, cap);
}

// dW += the splits' partials, summed in split order (deterministic)
static int ws_reduce(const WgradParams& p, long long splits, hipStream_t st) {
    if (!p.ws) return YXH_OK;
    const long long ne = (long long)p.cout * p.cin_store * p.kh * p.kw;
    hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st, (const float*)p.ws,
                       (int)splits, ne, p.dw);
    YXH_CHECK_LAUNCH("wgrad_reduce");
    return YXH_OK;
}

template <int S, int TN, int TC, int WN, int WC, int TY>
int launch_wgrad9_t(WgradParams p, hipStream_t st) {
    if (p.kh != 3 || p.kw != 3 || p.pad != 1 || p.stride != S || p.nsrc != 1 || p.sup[0] || p.sw[0] != p.in_w) {
        set_error("wgrad tiles 11-16 (all nine taps per block) need a 3x3 pad-1 stride-%d conv over one plain source", S);
        return YXH_EUNSUPPORTED;
    }
    if (p.cin % 4 || p.dych % 4 || p.dycs % 4 || p.scs[0] % 4) {
        set_error("wgrad tiles 11-16: channels must be whole 4-float chunks");
        return YXH_EUNSUPPORTED;
    }
    const int tiles_x = (p.out_w + 15) / 16, tiles_y = (p.out_h + TY - 1) / TY;
    const long long T = (long long)p.B * tiles_x * tiles_y;
    const int ntn = (p.cout + TN - 1) / TN, ntc = (p.cin + TC - 1) / TC;
    YXH_CHECK_ARG(T < (1LL << 31) && ntn < 65536 && ntc < 65536, "wgrad grid");
    // about two blocks per CU over the grid, at least two pixel tiles per block
    long long splits = (512 + (long long)ntn * ntc - 1) / ((long long)ntn * ntc);
    if (splits > (T + 1) / 2) splits = (T + 1) / 2;
    splits = ws_cap_splits(p, splits);
    if (splits < 1) splits = 1;
    const int tpb = (int)((T + splits - 1) / splits);
    splits = (T + tpb - 1) / tpb;
    hipLaunchKernelGGL((conv_wgrad9<S, TN, TC, WN, WC, TY>), dim3((unsigned)splits, ntn, ntc), dim3(64 * WN * WC), 0,
                       st, p, tiles_x, tiles_y, tpb);
    YXH_CHECK_LAUNCH("conv_wgrad9");
    return ws_reduce(p, splits, st);
}

// ------------------------------------------------------------------ weight gradient, LDS-DMA + transposed reads
// bf16/f16 variant (tile ids 5-10, TN and TM in {64, 128}): both operands land in LDS in
// their natural pixel-major layout by LDS-DMA (global_load_lds_dwordx4: one 16-byte
// channel chunk per lane, the zero chunk for padding taps and the pixel tail), and the
// MFMA fragments come out pixel(K)-major through gfx950's ds_read_b64_tr_b16 -- no
// register staging and no in-register transpose, so the K loop is DMA issue + LDS reads
// + MFMA over an NBUF-deep ring with counted vmcnt waits and raw barriers.  K = linear
// output pixels, 64 per stage; each lane's DMA rows advance incrementally (no division
// in the loop).  Row images are [pixel][chunk ^ f(pixel)]: the transposed reads of a
// 32-lane half (4 consecutive rows, two blocks 8 rows apart) cover all 64 banks once.
typedef short wg_i16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint2 lds_read_tr16(const char* ptr) {
    const auto q = (__attribute__((address_space(3))) wg_i16x4*)(const_cast<char*>(ptr));
    return __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(q));
}

template <int NCH>
__device__ __forceinline__ int wg2_swz(int row) {
    if constexpr (NCH == 16) return ((row & 3) << 2) | ((row >> 2) & 3);
    else return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2);
}

__device__ __forceinline__ void wg2_glds16(const void* g, void* l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wg2_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void wg2_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

struct Wg2Pix {
    int b, oy, ox;
};

template <typename T, int TN, int TM, int NBUF>
__global__ __launch_bounds__(256) void conv_wgrad2(WgradParams p) {
    constexpr int KP = 64;                     // output pixels per stage (two 32-deep K slabs)
    constexpr int NCA = TN / 8, NCB = TM / 8;  // 16-byte chunks per pixel row
    constexpr int RBA = NCA * 16, RBB = NCB * 16;
    constexpr int A_BYTES = KP * RBA, B_BYTES = KP * RBB, BUF = A_BYTES + B_BYTES;
    constexpr int PWA = A_BYTES / 4096, PWB = B_BYTES / 4096;  // 1 KiB DMA pieces per wave per stage
    constexpr int PW = PWA + PWB;
    constexpr int WTN = TN / 2, WTM = TM / 2, FR = WTN / 16, FC = WTM / 16;
    static_assert(PWA >= 1 && PWB >= 1 && sizeof(T) == 2 && (NBUF == 2 || NBUF == 3), "tile");
    __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const int n0 = blockIdx.y * TN;
    const int tap = blockIdx.z / p.ntc, c0 = (blockIdx.z - tap * p.ntc) * TM;
    const int ky = tap / p.kw, kx = tap - ky * p.kw;
    const int st0 = blockIdx.x * p.sps;
    const int nst = min(p.nst, st0 + p.sps) - st0;
    if (nst <= 0) return;

    // this lane's DMA slots: piece k of an image holds bytes [1024k, 1024k + 1024)
    int rowA[PWA], chA[PWA], rowB[PWB], chB[PWB];
#pragma unroll
    for (int a = 0; a < PWA; ++a) {
        const int byte = (wave * PWA + a) * 1024 + lane * 16;
        rowA[a] = byte / RBA;
        chA[a] = ((byte % RBA) >> 4) ^ wg2_swz<NCA>(rowA[a]);
    }
#pragma unroll
    for (int q = 0; q < PWB; ++q) {
        const int byte = (wave * PWB + q) * 1024 + lane * 16;
        rowB[q] = byte / RBB;
        chB[q] = ((byte % RBB) >> 4) ^ wg2_swz<NCB>(rowB[q]);
    }
    Wg2Pix sa[PWA], sb[PWB];
    auto init = [&](Wg2Pix& s, int row) {
        const long long m = (long long)st0 * KP + row;
        s.b = (int)(m / p.ohw);
        const int pix = (int)(m - (long long)s.b * p.ohw);
        s.oy = pix / p.out_w;
        s.ox = pix - s.oy * p.out_w;
    };
    auto adv = [&](Wg2Pix& s) {
        s.ox += KP;
        while (s.ox >= p.out_w) {
            s.ox -= p.out_w;
            if (++s.oy == p.out_h) {
                s.oy = 0;
                ++s.b;
            }
        }
    };
#pragma unroll
    for (int a = 0; a < PWA; ++a) init(sa[a], rowA[a]);
#pragma unroll
    for (int q = 0; q < PWB; ++q) init(sb[q], rowB[q]);

    const T* dyp = (const T*)p.dy;
    const void* zero = (const void*)g_wg_zero;
    auto issue = [&](int buf) {
        char* A = smem + buf * BUF;
        char* Bm = A + A_BYTES;
#pragma unroll
        for (int a = 0; a < PWA; ++a) {
            const int n = n0 + chA[a] * 8;
            const void* g = zero;
            if (sa[a].b < p.B && n < p.dych)
                g = dyp + (long long)sa[a].b * p.dybs + (long long)(sa[a].oy * p.out_w + sa[a].ox) * p.dycs + n;
            wg2_glds16(g, A + (wave * PWA + a) * 1024);
        }
#pragma unroll
        for (int q = 0; q < PWB; ++q) {
            int c = c0 + chB[q] * 8;
            const int iy = sb[q].oy * p.stride - p.pad + ky, ix = sb[q].ox * p.stride - p.pad + kx;
            const void* g = zero;
            if (sb[q].b < p.B && c < p.cin && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w) {
                int si = 0;
                if (p.nsrc == 2 && c >= p.src0_ch) {
                    si = 1;
                    c -= p.src0_ch;
                }
                const int up = p.sup[si];
                g = (const T*)p.sptr[si] + (long long)sb[q].b * p.sbs[si] +
                    ((long long)(iy >> up) * p.sw[si] + (ix >> up)) * p.scs[si] + c;
            }
            wg2_glds16(g, Bm + (wave * PWB + q) * 1024);
        }
#pragma unroll
        for (int a = 0; a < PWA; ++a) adv(sa[a]);
#pragma unroll
        for (int q = 0; q < PWB; ++q) adv(sb[q]);
    };

    // transposed-read addresses (image-relative, K slab 0): lane 4q+p of a 16-lane group
    // supplies row q of the 4-row block, columns 4p..4p+3; it receives its own column
    const int g4 = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    int offA[2][FR], offB[2][FC];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int row = 8 * g4 + 4 * h + q4;
#pragma unroll
        for (int i = 0; i < FR; ++i) {
            const int ch = ((wr * WTN + i * 16) >> 3) + (p4 >> 1);
            offA[h][i] = row * RBA + 16 * (ch ^ wg2_swz<NCA>(row)) + 8 * (p4 & 1);
        }
#pragma unroll
        for (int j = 0; j < FC; ++j) {
            const int ch = ((wc * WTM + j * 16) >> 3) + (p4 >> 1);
            offB[h][j] = row * RBB + 16 * (ch ^ wg2_swz<NCB>(row)) + 8 * (p4 & 1);
        }
    }

    f32x4 acc[FR][FC];
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](int buf) {
        const char* A = smem + buf * BUF;
        const char* Bm = A + A_BYTES;
#pragma unroll
        for (int s = 0; s < KP / 32; ++s) {
            uint4 af[FR], bf[FC];
#pragma unroll
            for (int i = 0; i < FR; ++i) {
                const uint2 lo = lds_read_tr16(A + s * 32 * RBA + offA[0][i]);
                const uint2 hi = lds_read_tr16(A + s * 32 * RBA + offA[1][i]);
                af[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
            }
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                const uint2 lo = lds_read_tr16(Bm + s * 32 * RBB + offB[0][j]);
                const uint2 hi = lds_read_tr16(Bm + s * 32 * RBB + offB[1][j]);
                bf[j] = make_uint4(lo.x, lo.y, hi.x, hi.y);
            }
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) Mma<T>::run(acc[i][j], af[i], bf[j]);
        }
    };

    constexpr int D = NBUF - 1;  // stages in flight ahead of the one being computed
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (d < nst) issue(d);
    for (int k = 0; k < nst; ++k) {
        if constexpr (D == 2) {
            if (k + 1 < nst) wg2_wait_vm<PW>();  // stage k landed; stage k+1 may still fly
            else wg2_wait_vm<0>();
        } else {
            wg2_wait_vm<0>();
        }
        wg2_barrier();  // every wave's pieces landed; compute(k-1) done -> its buffer is free
        if (k + D < nst) issue((k + D) % NBUF);
        compute(k % NBUF);
    }
    // dW (torch layout [cout][cin_store][kh][kw]) += acc
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) {
            const int c = c0 + wc * WTM + j * 16 + (lane & 15);
            if (c >= p.cin_store) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n0 + wr * WTN + i * 16 + (lane >> 4) * 4 + r;
                if (n < p.cout) {
                    const long long e = (((long long)n * p.cin_store + c) * p.kh + ky) * p.kw + kx;
                    if (p.ws) p.ws[(long long)blockIdx.x * p.cout * p.cin_store * p.kh * p.kw + e] = acc[i][j][r];
                    else atomicAdd(p.dw + e, acc[i][j][r]);
                }
            }
        }
}

// ------------------------------------------------------------------ fp32 weight gradient
// dW[n][c][tap] += sum over output pixels p of dY[p][n] * X[in(p, tap)][c] for fp32 convs (any
// kh x kw, stride, pad; the 1x1 and 3x3 BaseConvs of the training step).  Both operands are
// pixel-major, which is exactly the k-major operand form of v_mfma_f32_16x16x4_f32 (lane l:
// A[l % 16][l / 16] = dY[p0 + l / 16][n0 + l % 16], B likewise from X at the tap's input pixel,
// zero outside the image): no transposes.  A block owns a TN x TC tile of ONE tap over a range of
// KP-pixel stages (split-K over pixels); per stage both slabs are staged through LDS by 16-byte
// register loads (rows padded by 16 floats: the four 16-lane row groups of a ds_read_b32 hit
// distinct banks), double-buffered.  With a workspace each split stores its partial dW plainly
// and wgrad_reduce sums the splits in a fixed order (deterministic, no cross-XCD atomics);
// without one the partials go out as fp32 atomics (dW pre-zeroed, as for conv_wgrad).
template <int TN, int TC, int WN, int WC, int KP>
__global__ __launch_bounds__(256) void wgrad_f32(WgradParams p) {
    static_assert(WN * WC == 4, "4 waves");
    constexpr int WTN = TN / WN, WTC = TC / WC, FN = WTN / 16, FC = WTC / 16;
    constexpr int TNP = TN + 16, TCP = TC + 16;
    constexpr int ASZ = KP * TNP, BSZ = KP * TCP;
    constexpr int ACH = KP * TN / 4, BCH = KP * TC / 4, AL = (ACH + 255) / 256, BL = (BCH + 255) / 256;
    __shared__ __attribute__((aligned(16))) float lds[2][ASZ + BSZ];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wn = wave % WN, wc = wave / WN;
    const int taps = p.kh * p.kw;
    const int tap = (int)blockIdx.z % taps, ct = (int)blockIdx.z / taps;
    const int ty = tap / p.kw, tx = tap - ty * p.kw;
    const int n0 = blockIdx.y * TN, c0 = ct * TC;
    const int st0 = blockIdx.x * p.sps, st1 = min(p.nst, st0 + p.sps);
    const int M = p.M, ohw = p.ohw, ow = p.out_w, cout = p.cout, cin = p.cin;
    const float* dy = (const float*)p.dy;
    const bool dy_dense = p.dybs == (long long)ohw * p.dycs;

    float4 ra[AL], rb[BL];
    auto gload = [&](int st) {
        const int pb = st * KP;
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            const int row = q / (TN / 4), col = q - row * (TN / 4);
            const int m = pb + row, n = n0 + col * 4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < ACH && m < M && n < cout) {
                long long off;
                if (dy_dense) {
                    off = (long long)m * p.dycs;
                } else {
                    const int b = m / ohw;
                    off = (long long)b * p.dybs + (long long)(m - b * ohw) * p.dycs;
                }
                v = *(const float4*)(dy + off + n);
            }
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            const int row = q / (TC / 4), col = q - row * (TC / 4);
            const int m = pb + row, c = c0 + col * 4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < BCH && m < M && c < cin) {
                const int b = m / ohw, pix = m - b * ohw;
                const int oy = pix / ow, ox = pix - oy * ow;
                const int iy = oy * p.stride + ty - p.pad, ix = ox * p.stride + tx - p.pad;
                if ((unsigned)iy < (unsigned)p.in_h && (unsigned)ix < (unsigned)p.in_w) {
                    const int s = (p.nsrc > 1 && c >= p.src0_ch) ? 1 : 0;
                    const int cc = s ? c - p.src0_ch : c;
                    const int spix = p.sup[s] ? (iy >> 1) * p.sw[s] + (ix >> 1) : iy * p.sw[s] + ix;
                    v = *(const float4*)((const float*)p.sptr[s] + (long long)b * p.sbs[s] + (long long)spix * p.scs[s] + cc);
                }
            }
            rb[i] = v;
        }
    };
    auto lstore = [&](int buf) {
        float* A = lds[buf];
        float* Bm = lds[buf] + ASZ;
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            const int row = q / (TN / 4), col = q - row * (TN / 4);
            if (q < ACH) *(float4*)(A + row * TNP + col * 4) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            const int row = q / (TC / 4), col = q - row * (TC / 4);
            if (q < BCH) *(float4*)(Bm + row * TCP + col * 4) = rb[i];
        }
    };

    f32x4 acc[FN][FC];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int kr = lane >> 4, kc = lane & 15;
    if (st0 < st1) {
        gload(st0);
        lstore(0);
        __syncthreads();
    }
    int buf = 0;
    for (int st = st0; st < st1; ++st) {
        const bool more = st + 1 < st1;
        if (more) gload(st + 1);
        const float* A = lds[buf] + wn * WTN + kc;
        const float* Bm = lds[buf] + ASZ + wc * WTC + kc;
#pragma unroll
        for (int kk = 0; kk < KP / 4; ++kk) {
            float a[FN], b[FC];
#pragma unroll
            for (int i = 0; i < FN; ++i) a[i] = A[(4 * kk + kr) * TNP + 16 * i];
#pragma unroll
            for (int j = 0; j < FC; ++j) b[j] = Bm[(4 * kk + kr) * TCP + 16 * j];
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (more) lstore(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    // D[m][n] of fragment (i, j): lane holds rows 4 (lane / 16) + r, column lane % 16
    float* out = p.ws ? p.ws + (long long)blockIdx.x * p.cout * p.cin_store * taps : p.dw;
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) {
            const int c = c0 + wc * WTC + 16 * j + kc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n0 + wn * WTN + 16 * i + 4 * kr + r;
                if (n >= cout || c >= p.cin_store) continue;
                float* d = out + ((long long)n * p.cin_store + c) * taps + tap;
                if (p.ws) *d = acc[i][j][r];
                else unsafeAtomicAdd(d, acc[i][j][r]);
            }
        }
}

// fp32 3x3 weight gradient with all nine taps per block: a stage is a row segment of KP output
// pixels (image b, row oy, columns ox0 .. ox0 + KP); dY[KP][TN] and the three input rows it
// reads, X[3][(KP - 1) s + 3][TC] (zero outside the image), are staged once, and every tap's
// B operand is a shifted view of the X rows: dY and X are read once per stage instead of once
// per tap.  acc[9][FN][FC] stays in registers for the block's pixel range; partials as wgrad_f32.
template <int TN, int TC, int S, int KP>
__global__ __launch_bounds__(256) void wgrad9t_f32(WgradParams p, int nseg) {
    constexpr int WN = 2, WC = 2;
    constexpr int WTN = TN / WN, WTC = TC / WC, FN = WTN / 16, FC = WTC / 16;
    constexpr int XW = (KP - 1) * S + 3, TNP = TN + 16, TCP = TC + 16;
    constexpr int ASZ = KP * TNP, BSZ = 3 * XW * TCP;
    constexpr int ACH = KP * TN / 4, BCH = 3 * XW * TC / 4, AL = (ACH + 255) / 256, BL = (BCH + 255) / 256;
    __shared__ __attribute__((aligned(16))) float lds[2][ASZ + BSZ];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wn = wave % WN, wc = wave / WN;
    const int n0 = blockIdx.y * TN, c0 = blockIdx.z * TC;
    const int st0 = blockIdx.x * p.sps, st1 = min(p.nst, st0 + p.sps);
    const int oh = p.out_h, ow = p.out_w, cout = p.cout, cin = p.cin;
    const float* dy = (const float*)p.dy;

    float4 ra[AL], rb[BL];
    auto gload = [&](int st) {
        const int seg = st % nseg, r = st / nseg;
        const int b = r / oh, oy = r - b * oh, ox0 = seg * KP;
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            const int row = q / (TN / 4), col = q - row * (TN / 4);
            const int ox = ox0 + row, n = n0 + col * 4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < ACH && ox < ow && n < cout)
                v = *(const float4*)(dy + (long long)b * p.dybs + (long long)(oy * ow + ox) * p.dycs + n);
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            const int row = q / (TC / 4), col = q - row * (TC / 4);  // row = ty * XW + xx
            const int ty = row / XW, xx = row - ty * XW;
            const int iy = oy * S + ty - 1, ix = ox0 * S + xx - 1, c = c0 + col * 4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < BCH && c < cin && (unsigned)iy < (unsigned)p.in_h && (unsigned)ix < (unsigned)p.in_w) {
                const int s = (p.nsrc > 1 && c >= p.src0_ch) ? 1 : 0;
                const int cc = s ? c - p.src0_ch : c;
                const int spix = p.sup[s] ? (iy >> 1) * p.sw[s] + (ix >> 1) : iy * p.sw[s] + ix;
                v = *(const float4*)((const float*)p.sptr[s] + (long long)b * p.sbs[s] + (long long)spix * p.scs[s] + cc);
            }
            rb[i] = v;
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            if (q < ACH) *(float4*)(lds[buf] + (q / (TN / 4)) * TNP + (q % (TN / 4)) * 4) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            if (q < BCH) *(float4*)(lds[buf] + ASZ + (q / (TC / 4)) * TCP + (q % (TC / 4)) * 4) = rb[i];
        }
    };

    f32x4 acc[9][FN][FC];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FC; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int kr = lane >> 4, kc = lane & 15;
    if (st0 < st1) {
        gload(st0);
        lstore(0);
        __syncthreads();
    }
    int buf = 0;
    for (int st = st0; st < st1; ++st) {
        const bool more = st + 1 < st1;
        if (more) gload(st + 1);
        const float* A = lds[buf] + wn * WTN + kc;
        const float* Bm = lds[buf] + ASZ + wc * WTC + kc;
#pragma unroll
        for (int kk = 0; kk < KP / 4; ++kk) {
            float a[FN];
#pragma unroll
            for (int i = 0; i < FN; ++i) a[i] = A[(4 * kk + kr) * TNP + 16 * i];
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int xrow = (t / 3) * XW + (4 * kk + kr) * S + (t % 3);
                float b[FC];
#pragma unroll
                for (int j = 0; j < FC; ++j) b[j] = Bm[xrow * TCP + 16 * j];
#pragma unroll
                for (int i = 0; i < FN; ++i)
#pragma unroll
                    for (int j = 0; j < FC; ++j)
                        acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[t][i][j], 0, 0, 0);
            }
        }
        if (more) lstore(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    float* out = p.ws ? p.ws + (long long)blockIdx.x * p.cout * p.cin_store * 9 : p.dw;
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) {
            const int c = c0 + wc * WTC + 16 * j + kc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n0 + wn * WTN + 16 * i + 4 * kr + r;
                if (n >= cout || c >= p.cin_store) continue;
                float* d = out + ((long long)n * p.cin_store + c) * 9;
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    if (p.ws) d[t] = acc[t][i][j][r];
                    else unsafeAtomicAdd(d + t, acc[t][i][j][r]);
                }
            }
        }
}

// bf16/f16 3x3 weight gradient with all nine taps per block (tiles 25-30): wgrad9t_f32's
// staging -- a stage is a row segment of KP output pixels; dY[KP][TN] and the three input rows
// X[3][(KP - 1) s + 3][TC] it reads are copied once into LDS in their natural pixel-major layout
// (rows padded by 16 bytes) -- with the 16-bit MFMA operands (8 consecutive pixels of one channel
// per lane) read out pixel-transposed by ds_read_b64_tr_b16.  Each lane of a transposed read
// names its own pixel row, so tap (ky, kx)'s B operand is the X row ky * XW + p * s + kx of each
// pixel p: stride and shift cost nothing, and dY / X are read once per stage instead of once per
// tap (tiles 1-10 stage both operands per tap: nine reads of each).
template <typename T, int TN, int TC, int S, int KP>
__global__ __launch_bounds__(256, (TN * TC <= 64 * 64 && KP == 32 && S == 1) ? 2 : 1) void wgrad9t_h(WgradParams p, int nseg) {
    constexpr int WTN = TN / 2, WTC = TC / 2, FN = WTN / 16, FC = WTC / 16;
    // row pitches: the 8 pixel rows one 32-lane half reads (stride S apart) land on distinct
    // 8-bank windows -- pitch / 4 an odd multiple of 8 banks (mod 64) per S rows
    constexpr int XW = (KP - 1) * S + 3, RA = TN * 2 + 32, RB = TC * 2 + (S == 1 ? 32 : 16);
    constexpr int ASZ = KP * RA, BSZ = 3 * XW * RB;
    constexpr int ACH = KP * TN / 8, BCH = 3 * XW * TC / 8, AL = (ACH + 255) / 256, BL = (BCH + 255) / 256;
    static_assert(sizeof(T) == 2 && KP % 32 == 0 && FN >= 1 && FC >= 1, "tile");
    __shared__ __attribute__((aligned(16))) char lds[2][ASZ + BSZ];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wn = wave & 1, wc = wave >> 1;
    // XCD-aware order: the dispatcher deals linear block ids to the 8 XCDs round-robin; the
    // ntn x ntc blocks of one split (same pixels, so the same dY / X lines) get consecutive
    // logical ids on one XCD and share its L2 instead of fetching the lines once per XCD
    const int nblk = gridDim.x * gridDim.y * gridDim.z;
    const int bid = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
    const int tc_ = lid % gridDim.z, tn_ = (lid / gridDim.z) % gridDim.y, split = lid / (gridDim.z * gridDim.y);
    const int n0 = tn_ * TN, c0 = tc_ * TC;
    const int st0 = split * p.sps, st1 = min(p.nst, st0 + p.sps);
    const int oh = p.out_h, ow = p.out_w, cin = p.cin;
    const T* dy = (const T*)p.dy;

    uint4 ra[AL], rb[BL];
    auto gload = [&](int st) {
        const int seg = st % nseg, r = st / nseg;
        const int b = r / oh, oy = r - b * oh, ox0 = seg * KP;
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            const int row = q / (TN / 8), col = q - row * (TN / 8);
            const int ox = ox0 + row, n = n0 + col * 8;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (q < ACH && ox < ow && n < p.dych)
                v = *(const uint4*)(dy + (long long)b * p.dybs + (long long)(oy * ow + ox) * p.dycs + n);
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            const int row = q / (TC / 8), col = q - row * (TC / 8);  // row = ty * XW + xx
            const int ty = row / XW, xx = row - ty * XW;
            const int iy = oy * S + ty - 1, ix = ox0 * S + xx - 1, c = c0 + col * 8;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (q < BCH && c < cin && (unsigned)iy < (unsigned)p.in_h && (unsigned)ix < (unsigned)p.in_w) {
                const int s = (p.nsrc > 1 && c >= p.src0_ch) ? 1 : 0;
                const int cc = s ? c - p.src0_ch : c;
                const int spix = p.sup[s] ? (iy >> 1) * p.sw[s] + (ix >> 1) : iy * p.sw[s] + ix;
                v = *(const uint4*)((const T*)p.sptr[s] + (long long)b * p.sbs[s] + (long long)spix * p.scs[s] + cc);
            }
            rb[i] = v;
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int q = tid + 256 * i;
            if (q < ACH) *(uint4*)(lds[buf] + (q / (TN / 8)) * RA + (q % (TN / 8)) * 16) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int q = tid + 256 * i;
            if (q < BCH) *(uint4*)(lds[buf] + ASZ + (q / (TC / 8)) * RB + (q % (TC / 8)) * 16) = rb[i];
        }
    };

    f32x4 acc[9][FN][FC];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FC; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // transposed reads: lane 4q + p of a 16-lane group names pixel row q of a 4-row block and
    // columns 4p .. 4p + 3; it receives its own column (lane % 16) over the four rows.  K slot
    // 8g + 4h + q of a 32-pixel slab holds pixel 16h + 4g + q (any bijection serves, A and B
    // alike): a 32-lane half's read then covers 8 consecutive pixel rows
    const int g4 = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int colA = (wn * WTN + 4 * p4) * 2, colB = (wc * WTC + 4 * p4) * 2;
    if (st0 < st1) {
        gload(st0);
        lstore(0);
        __syncthreads();
    }
    int buf = 0;
    for (int st = st0; st < st1; ++st) {
        const bool more = st + 1 < st1;
        if (more) gload(st + 1);
        const char* A = lds[buf] + colA;
        const char* Bm = lds[buf] + ASZ + colB;
#pragma unroll
        for (int kk = 0; kk < KP / 32; ++kk) {
            const int pr0 = 32 * kk + 4 * g4 + q4, pr1 = pr0 + 16;
            uint4 af[FN];
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const uint2 lo = lds_read_tr16(A + pr0 * RA + 32 * i);
                const uint2 hi = lds_read_tr16(A + pr1 * RA + 32 * i);
                af[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
            }
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int x0 = (t / 3) * XW + pr0 * S + (t % 3), x1 = x0 + 16 * S;
                uint4 bf[FC];
#pragma unroll
                for (int j = 0; j < FC; ++j) {
                    const uint2 lo = lds_read_tr16(Bm + x0 * RB + 32 * j);
                    const uint2 hi = lds_read_tr16(Bm + x1 * RB + 32 * j);
                    bf[j] = make_uint4(lo.x, lo.y, hi.x, hi.y);
                }
#pragma unroll
                for (int i = 0; i < FN; ++i)
#pragma unroll
                    for (int j = 0; j < FC; ++j) Mma<T>::run(acc[t][i][j], af[i], bf[j]);
            }
        }
        if (more) lstore(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    float* out = p.ws ? p.ws + (long long)split * p.cout * p.cin_store * 9 : p.dw;
    const int kr = lane >> 4, kc = lane & 15;
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) {
            const int c = c0 + wc * WTC + 16 * j + kc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n0 + wn * WTN + 16 * i + 4 * kr + r;
                if (n >= p.cout || c >= p.cin_store) continue;
                float* d = out + ((long long)n * p.cin_store + c) * 9;
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    if (p.ws) d[t] = acc[t][i][j][r];
                    else unsafeAtomicAdd(d + t, acc[t][i][j][r]);
                }
            }
        }
}

// dW[i] += sum over the splits of ws[split][i], in split order (deterministic)
__global__ __launch_bounds__(256) void wgrad_reduce(const float* ws, int splits, long long ne, float* dw) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= ne) return;
    float s = 0.0f;
    for (int k = 0; k < splits; ++k) s += ws[(long long)k * ne + i];
    dw[i] += s;
}

// dgrad weights: w [cout][cin][kh][kw] fp32 -> [c_count][kh][kw][cout_pad] of T, taps
// flipped (ky -> kh-1-ky), input channels [c_begin, c_begin + c_count).
template <typename T>
__global__ __launch_bounds__(256) void pack_dgrad(const float* w, int cout, int cin, int kh, int kw, int c_begin,
                                                  int c_count, int cout_pad, T* out) {
    const long long total = (long long)c_count * kh * kw * cout_pad;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int n = (int)(idx % cout_pad);
    const int t = (int)((idx / cout_pad) % (kh * kw));
    const int c = (int)(idx / ((long long)cout_pad * kh * kw));
    const int ky = t / kw, kx = t - ky * kw;
    float v = 0.0f;
    if (n < cout) v = w[(((long long)n * cin + c_begin + c) * kh + (kh - 1 - ky)) * kw + (kw - 1 - kx)];
    out[idx] = from_f32<T>(v);
}

// Every repack of a training step in one launch: block b belongs to the last job whose
// block0 <= b (binary search over the job table, which stays in L2); element order and
// values as fold_bn_pack without BN (kind FWD) and pack_dgrad (kind DGRAD).
template <typename T>
__global__ __launch_bounds__(256) void pack_batch(const yxh_pack_job* jobs, int njobs) {
    const int b = blockIdx.x;
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (jobs[mid].block0 <= b) lo = mid;
        else hi = mid - 1;
    }
    const yxh_pack_job& j = jobs[lo];
    const long long idx = (long long)(b - j.block0) * 256 + threadIdx.x;
    const int taps = j.kh * j.kw;
    if (j.kind == YXH_PACK_FWD) {
        const long long total = (long long)j.cout * taps * j.pad;
        if (idx >= total) return;
        const int c = (int)(idx % j.pad);
        const int t = (int)((idx / j.pad) % taps);
        const int n = (int)(idx / ((long long)j.pad * taps));
        const int ky = t / j.kw, kx = t - ky * j.kw;
        const float v = c < j.cin ? j.w[(((long long)n * j.cin + c) * j.kh + ky) * j.kw + kx] : 0.0f;
        ((T*)j.out)[idx] = from_f32<T>(v);
        if (t == 0 && c == 0 && j.bias_out) j.bias_out[n] = j.cb ? j.cb[n] : 0.0f;
    } else {
        const long long total = (long long)j.c_count * taps * j.pad;
        if (idx >= total) return;
        const int n = (int)(idx % j.pad);
        const int t = (int)((idx / j.pad) % taps);
        const int c = (int)(idx / ((long long)j.pad * taps));
        const int ky = t / j.kw, kx = t - ky * j.kw;
        float v = 0.0f;
        if (n < j.cout) v = j.w[(((long long)n * j.cin + j.c_begin + c) * j.kh + (j.kh - 1 - ky)) * j.kw + (j.kw - 1 - kx)];
        ((T*)j.out)[idx] = from_f32<T>(v);
    }
}

// ------------------------------------------------------------------ SPP / upsample backward
// Block = (CPB channels, image), 1024 threads: the plane lives in LDS.  Per pool radius r (2, 4, 6):
// horizontal pass -> first max column hcol of each row window; vertical pass -> first max row brow
// among those = torch's argmax (first maximum in row-major scan, -inf padding): output (oy, ox)
// routes its gradient to pixel (brow, hcol[brow][ox]).  Every input pixel then GATHERS those
// gradients separably (fixed order, no atomics: deterministic): G1[y][ox] = the outputs of column
// ox whose argmax row is y (2r + 1 candidates), then pixel (y, x) sums the G1[y][ox] whose row-window
// max sits in column x (2r + 1 more) -- 2 (2r + 1) LDS reads per pixel instead of (2r + 1)^2.
// dx = dcat[:, :c] + the three gathers.  (The round-4 form gathered over the whole square window
// with one wave per SIMD: 3.4 ms of the configs[4] step's main stream for yolox_x's 40x40x640 SPP.)
template <typename T, int CPB>
__global__ __launch_bounds__(1024) void spp_bwd(TView cat, int H, int W, int c, const float* dcat, float* dx,
                                                int B) {
    extern __shared__ __attribute__((aligned(16))) char sm[];
    const int HW = H * W, n = HW * CPB;
    unsigned short* brow = (unsigned short*)sm;  // [3][n] argmax row of output q
    unsigned short* hcol = brow + 3 * n;         // [3][n] first max column of row y's window around x
    float* pl = (float*)(hcol + 3 * n);          // plane, then the staged output gradients of pool k
    float* hv = pl + n;                          // row-window max, then G1
    float* acc = hv + n;                         // the input gradient being gathered
    const int c0 = blockIdx.x * CPB, b = blockIdx.y, nt = blockDim.x;
    const T* xb = (const T*)cat.ptr + (long long)b * cat.bs;
    const float* db = dcat + (long long)b * HW * 4 * c;
    for (int q = threadIdx.x; q < n; q += nt) {
        const int pix = q / CPB, j = q - pix * CPB;
        const bool in = c0 + j < c;
        pl[q] = in ? to_f32(xb[(long long)pix * cat.cs + c0 + j]) : 0.0f;
        acc[q] = in ? db[(long long)pix * 4 * c + c0 + j] : 0.0f;
    }
    __syncthreads();
    for (int k = 0; k < 3; ++k) {
        const int r = 2 + 2 * k;
        for (int q = threadIdx.x; q < n; q += nt) {
            const int pix = q / CPB, j = q - pix * CPB;
            const int y = pix / W, x = pix - y * W;
            float best = 0.0f;
            int bc = -1;
            for (int xx = max(0, x - r); xx <= min(W - 1, x + r); ++xx) {
                const float v = pl[(y * W + xx) * CPB + j];
                if (bc < 0 || v > best) {
                    best = v;
                    bc = xx;
                }
            }
            hv[q] = best;
            hcol[k * n + q] = (unsigned short)bc;
        }
        __syncthreads();
        for (int q = threadIdx.x; q < n; q += nt) {
            const int pix = q / CPB, j = q - pix * CPB;
            const int y = pix / W, x = pix - y * W;
            float best = 0.0f;
            int br = -1;
            for (int yy = max(0, y - r); yy <= min(H - 1, y + r); ++yy) {
                const float v = hv[(yy * W + x) * CPB + j];
                if (br < 0 || v > best) {
                    best = v;
                    br = yy;
                }
            }
            brow[k * n + q] = (unsigned short)br;
        }
        __syncthreads();
    }
    // the plane is dead: per pool, stage its output gradients, gather by columns, then by rows
    for (int k = 0; k < 3; ++k) {
        const int r = 2 + 2 * k;
        const unsigned short* bk = brow + k * n;
        const unsigned short* hk = hcol + k * n;
        for (int q = threadIdx.x; q < n; q += nt) {
            const int pix = q / CPB, j = q - pix * CPB;
            pl[q] = c0 + j < c ? db[(long long)pix * 4 * c + (k + 1) * c + c0 + j] : 0.0f;
        }
        __syncthreads();
        for (int q = threadIdx.x; q < n; q += nt) {  // G1[y][ox]
            const int pix = q / CPB, j = q - pix * CPB;
            const int y = pix / W, ox = pix - y * W;
            float g = 0.0f;
            for (int oy = max(0, y - r); oy <= min(H - 1, y + r); ++oy) {
                const int o = (oy * W + ox) * CPB + j;
                if (bk[o] == y) g += pl[o];
            }
            hv[q] = g;
        }
        __syncthreads();
        for (int q = threadIdx.x; q < n; q += nt) {
            const int pix = q / CPB, j = q - pix * CPB;
            const int y = pix / W, x = pix - y * W;
            float g = 0.0f;
            for (int ox = max(0, x - r); ox <= min(W - 1, x + r); ++ox) {
                const int o = (y * W + ox) * CPB + j;
                if (hk[o] == x) g += hv[o];
            }
            acc[q] += g;
        }
        __syncthreads();
    }
    for (int q = threadIdx.x; q < n; q += nt) {
        const int pix = q / CPB, j = q - pix * CPB;
        if (c0 + j < c) dx[((long long)b * HW + pix) * c + c0 + j] = acc[q];
    }
}

__global__ __launch_bounds__(256) void upsample_bwd(const float* g, int B, int h, int w, int C, float* dst) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    const int nc4 = C / 4;
    if (idx >= (long long)B * h * w * nc4) return;
    const int c = (int)(idx % nc4) * 4;
    const long long m = idx / nc4;
    const int b = (int)(m / ((long long)h * w)), pix = (int)(m - (long long)b * h * w);
    const int y = pix / w, x = pix - y * w;
    const float* gb = g + (long long)b * 4 * h * w * C;
    float4 s = *(float4*)(dst + m * C + c);
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
            const float4 u = *(const float4*)(gb + ((long long)(2 * y + dy) * 2 * w + 2 * x + dx) * C + c);
            s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
        }
    *(float4*)(dst + m * C + c) = s;
}

// ================================================================== host
namespace {

int esz(int dt) { return dt == YXH_F32 ? 4 : 2; }

TView tview(const yxh_src* s, int C) {
    TView v;
    v.ptr = s ? s->ptr : nullptr;
    v.C = C;
    v.cs = s ? s->cstride : 0;
    v.HW = s ? s->h * s->w : 1;
    v.bs = s ? s->bstride : 0;
    return v;
}

bool a16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int check_view(const yxh_src* s, int dt, const char* what) {
    YXH_CHECK_ARG(s && s->ptr, "%s: null view", what);
    const int epc = 16 / esz(dt);
    YXH_CHECK_ARG(a16(s->ptr) && s->channels > 0 && s->channels % epc == 0 && s->cstride % epc == 0 &&
                      s->bstride % epc == 0 && s->h > 0 && s->w > 0,
                  "%s: view not 16-byte aligned / chunked (channels %d, cstride %d)", what, s->channels, s->cstride);
    return YXH_OK;
}

constexpr int kRedMaxBlocks = 1024;

// Reduction blocks: ~8 rows per thread, at most YXH_RED_BLOCKS (default 512: two 4-wave blocks
// per CU, one round; chan_finalize then reads 512 partials per channel instead of 1024 -- it is
// latency-bound on the strided partial rows and runs once per BatchNorm per pass)
int red_cap() {
    static const int cap = [] {
        const char* e = getenv("YXH_RED_BLOCKS");
        const int v = e ? atoi(e) : 512;
        return v < 1 ? 1 : v > kRedMaxBlocks ? kRedMaxBlocks : v;
    }();
    return cap;
}

int red_blocks(int M, int C, int dt, int* rpb) {
    const int nch = C / (16 / esz(dt));
    const int rpi = nch >= 256 ? 1 : 256 / nch;
    // ~8 rows per thread (2-4 in flight).  (~32 rows per thread left 4x fewer partials for chan_finalize
    // but too few blocks in flight for the mid-size fp32 maps: configs[2] 570 -> 527 img/s, round 5)
    int nblk = (int)(((long long)M + rpi * 8 - 1) / (rpi * 8));
    const int cap = red_cap();
    nblk = nblk < 1 ? 1 : (nblk > cap ? cap : nblk);
    *rpb = (M + nblk - 1) / nblk;
    return (M + *rpb - 1) / *rpb;
}

template <int MODE>
int launch_reduce(int dt, const RedArgs& a, int nblk, hipStream_t st) {
    const int per = 256 * (16 / esz(dt));  // channels per group (256 chunks)
    const dim3 grid(nblk, (a.x.C + per - 1) / per);
    if (dt == YXH_BF16) hipLaunchKernelGGL((chan_reduce<bf16, MODE>), grid, dim3(256), 0, st, a);
    else if (dt == YXH_F16) hipLaunchKernelGGL((chan_reduce<f16, MODE>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((chan_reduce<float, MODE>), grid, dim3(256), 0, st, a);
    YXH_CHECK_LAUNCH("chan_reduce");
    return YXH_OK;
}

}  // namespace

// partials [nblk][2][C] + the stats shift row [C] + the backward coefficients [3][C]
size_t reduce_workspace(int C) { return (size_t)(kRedMaxBlocks * 2 + 4) * C * sizeof(float); }

namespace {

int run_reduce(int mode, int dt, int B, const yxh_src* x, const yxh_src* g, const float* stats, int act,
               void* ws, size_t ws_bytes, FinArgs f, hipStream_t st) {
    const int C = x->channels;
    YXH_CHECK_ARG(B > 0, "batch %d", B);
    YXH_CHECK_ARG(C > 0 && C % (16 / esz(dt)) == 0, "reduction: %d channels not in 16-byte chunks", C);
    YXH_CHECK_ARG(ws && ws_bytes >= reduce_workspace(C), "reduction workspace too small");
    RedArgs a{};
    a.x = tview(x, C);
    a.g = tview(g, C);
    a.st = stats;
    a.act = act;
    const long long M = (long long)B * x->h * x->w;
    YXH_CHECK_ARG(M < (1LL << 31), "too many pixels");
    a.M = (int)M;
    const int nblk = red_blocks(a.M, C, dt, &a.rpb);
    a.partial = (float*)ws;
    int rc = mode == RED_STATS ? launch_reduce<RED_STATS>(dt, a, nblk, st)
             : mode == RED_BWD ? launch_reduce<RED_BWD>(dt, a, nblk, st)
                               : launch_reduce<RED_SUM>(dt, a, nblk, st);
    if (rc) return rc;
    f.partial = (const float*)ws;
    f.nblk = nblk;
    f.C = C;
    f.M = a.M;
    f.mode = mode;
    hipLaunchKernelGGL(chan_finalize, dim3((C + 3) / 4), dim3(256), 0, st, f);
    YXH_CHECK_LAUNCH("chan_finalize");
    return YXH_OK;
}

}  // namespace

int bn_stats(int dt, int B, const yxh_src* y, const float* gamma, const float* beta, float* rmean, float* rvar,
             float eps, float momentum, float* stats, void* ws, size_t ws_bytes, hipStream_t st) {
    if (int rc = check_view(y, dt, "bn_stats y")) return rc;
    YXH_CHECK_ARG(stats, "bn_stats: null stats");
    YXH_CHECK_ARG(!rmean == !rvar, "running mean/var must both be given or both NULL");
    FinArgs f{};
    f.gamma = gamma;
    f.beta = beta;
    f.rmean = rmean;
    f.rvar = rvar;
    f.eps = eps;
    f.momentum = momentum;
    f.stats = stats;
    return run_reduce(RED_STATS, dt, B, y, nullptr, nullptr, 0, ws, ws_bytes, f, st);
}

int bn_act_fwd_launch(int dt, int B, const yxh_src* y, const float* stats, int act, const yxh_src* res,
                      const yxh_src* out, hipStream_t st) {
    if (int rc = check_view(y, dt, "bn_act_fwd y")) return rc;
    if (int rc = check_view(out, dt, "bn_act_fwd out")) return rc;
    if (res && res->ptr)
        if (int rc = check_view(res, dt, "bn_act_fwd residual")) return rc;
    const int C = y->channels;
    YXH_CHECK_ARG(out->channels == C && out->h == y->h && out->w == y->w, "bn_act_fwd: out view shape");
    YXH_CHECK_ARG(!res || !res->ptr || (res->channels == C && res->h == y->h && res->w == y->w),
                  "bn_act_fwd: residual view shape");
    YXH_CHECK_ARG(stats && a16(stats) && B > 0, "bn_act_fwd: stats (16-byte aligned) / batch");
    const long long M = (long long)B * y->h * y->w;
    const long long total = M * (C / (16 / esz(dt)));
    TView r = tview(res && res->ptr ? res : nullptr, C);
    dim3 grid((unsigned)((total + 255) / 256));
#define YXH_BNF(T) hipLaunchKernelGGL(bn_act_fwd<T>, grid, dim3(256), 0, st, tview(y, C), stats, act, r, tview(out, C), (int)M)
    if (dt == YXH_BF16) YXH_BNF(bf16);
    else if (dt == YXH_F16) YXH_BNF(f16);
    else YXH_BNF(float);
#undef YXH_BNF
    YXH_CHECK_LAUNCH("bn_act_fwd");
    return YXH_OK;
}

int bn_act_bwd_launch(int dt, int B, const yxh_src* y, const yxh_src* dout, const float* stats, const float* gamma,
                      int act, float* dgamma, float* dbeta, void* dx, void* ws, size_t ws_bytes, hipStream_t st) {
    if (int rc = check_view(y, dt, "bn_act_bwd y")) return rc;
    if (int rc = check_view(dout, YXH_F32, "bn_act_bwd dout")) return rc;
    const int C = y->channels;
    YXH_CHECK_ARG(dout->channels == C && dout->h == y->h && dout->w == y->w, "bn_act_bwd: dout view shape");
    YXH_CHECK_ARG(stats && dgamma && dbeta && dx && a16(dx), "bn_act_bwd: null / unaligned outputs");
    YXH_CHECK_ARG(a16(stats), "bn_act_bwd: stats not 16-byte aligned");
    FinArgs f{};
    f.out0 = dgamma;
    f.out1 = dbeta;
    f.gamma = gamma;
    f.st_in = stats;
    float* coef = (float*)ws + (size_t)(kRedMaxBlocks * 2 + 1) * C;
    f.coef = coef;
    if (int rc = run_reduce(RED_BWD, dt, B, y, dout, stats, act, ws, ws_bytes, f, st)) return rc;
    const long long M = (long long)B * y->h * y->w;
    const long long total = M * (C / (16 / esz(dt)));
    dim3 grid((unsigned)((total + 255) / 256));
#define YXH_BNB(T)                                                                                                 \
    hipLaunchKernelGGL(bn_act_bwd_apply<T>, grid, dim3(256), 0, st, tview(y, C), tview(dout, C), stats, coef, act, \
                       (int)M, (T*)dx)
    if (dt == YXH_BF16) YXH_BNB(bf16);
    else if (dt == YXH_F16) YXH_BNB(f16);
    else YXH_BNB(float);
#undef YXH_BNB
    YXH_CHECK_LAUNCH("bn_act_bwd_apply");
    return YXH_OK;
}

int channel_sum_launch(int dt, int B, const yxh_src* x, float* out, void* ws, size_t ws_bytes, hipStream_t st) {
    if (int rc = check_view(x, dt, "channel_sum x")) return rc;
    YXH_CHECK_ARG(out, "channel_sum: null out");
    FinArgs f{};
    f.out0 = out;
    return run_reduce(RED_SUM, dt, B, x, nullptr, nullptr, 0, ws, ws_bytes, f, st);
}

namespace {

// Blocks a weight-gradient grid aims for (splits x tiles): YXH_WGRAD_BLOCKS, default 512 = two per CU.
// The weight gradients run on a side stream beside the data-gradient chain; a grid that fills every
// CU's registers leaves the main stream's BatchNorm reductions no room until its blocks retire.
int wgrad_target_blocks() {
    static const int v = [] {
        const char* e = getenv("YXH_WGRAD_BLOCKS");
        const int x = e ? atoi(e) : 512;
        return x < 64 ? 64 : x > 4096 ? 4096 : x;
    }();
    return v;
}

template <typename T, int TN, int TM, int WR, int WC, int KS>
int launch_wgrad_t(WgradParams p, hipStream_t st) {
    constexpr int EPC = Chunk<T>::N;
    constexpr int KP = 4 * KS * EPC;
    const int ntn = (p.cout + TN - 1) / TN;
    p.ntc = (p.cin + TM - 1) / TM;
    const int ntap = p.kh * p.kw;
    p.nst = (int)(((long long)p.B * p.out_h * ((p.out_w + EPC - 1) / EPC) + 4 * KS - 1) / (4 * KS));
    (void)KP;
    // ~2 blocks per CU over the whole grid; at least 8 stages per split
    const long long tiles = (long long)ntn * ntap * p.ntc;
    long long splits = (wgrad_target_blocks() + tiles - 1) / tiles;
    const long long max_splits = (p.nst + 7) / 8;
    if (splits > max_splits) splits = max_splits;
    splits = ws_cap_splits(p, splits);
    if (splits < 1) splits = 1;
    p.sps = (int)((p.nst + splits - 1) / splits);
    splits = (p.nst + p.sps - 1) / p.sps;
    YXH_CHECK_ARG(ntap * p.ntc < 65536 && ntn < 65536, "wgrad grid");
    hipLaunchKernelGGL((conv_wgrad<T, TN, TM, WR, WC, KS>), dim3((unsigned)splits, ntn, ntap * p.ntc), dim3(256), 0,
                       st, p);
    YXH_CHECK_LAUNCH("conv_wgrad");
    return ws_reduce(p, splits, st);
}

template <typename T, int TN, int TM, int NBUF>
int launch_wgrad2_t(WgradParams p, hipStream_t st) {
    if constexpr (sizeof(T) != 2) {
        set_error("wgrad tiles 5-10 (LDS-DMA + transposed LDS reads) are built for bf16/f16 only");
        return YXH_EUNSUPPORTED;
    } else {
        constexpr int KP = 64;
        constexpr int LDS = NBUF * KP * (TN + TM) * 2;
        const int ntn = (p.cout + TN - 1) / TN;
        p.ntc = (p.cin + TM - 1) / TM;
        const int ntap = p.kh * p.kw;
        p.nst = (int)(((long long)p.M + KP - 1) / KP);
        const long long tiles = (long long)ntn * ntap * p.ntc;
        const int occ = (160 * 1024) / LDS;
        long long splits = (256LL * (occ < 1 ? 1 : occ) + tiles - 1) / tiles;  // about one wave of blocks
        const long long max_splits = (p.nst + 3) / 4;                           // >= 4 stages per split
        if (splits > max_splits) splits = max_splits;
        splits = ws_cap_splits(p, splits);
        if (splits < 1) splits = 1;
        p.sps = (int)((p.nst + splits - 1) / splits);
        splits = (p.nst + p.sps - 1) / p.sps;
        YXH_CHECK_ARG(ntap * p.ntc < 65536 && ntn < 65536, "wgrad grid");
        hipLaunchKernelGGL((conv_wgrad2<T, TN, TM, NBUF>), dim3((unsigned)splits, ntn, ntap * p.ntc), dim3(256), 0,
                           st, p);
        YXH_CHECK_LAUNCH("conv_wgrad2");
        return ws_reduce(p, splits, st);
    }
}

template <int TN, int TC, int WN, int WC, int KP>
int launch_wgrad_f32(WgradParams p, hipStream_t st) {
    if ((p.nsrc > 1 && p.src0_ch % 4) || p.dycs % 4 || p.dybs % 4 || p.cin % 4) {
        set_error("wgrad tiles 17-20: 16-byte channel chunks");
        return YXH_EUNSUPPORTED;
    }
    const int taps = p.kh * p.kw;
    const int ntn = (p.cout + TN - 1) / TN, ntc = (p.cin + TC - 1) / TC;
    p.nst = (int)(((long long)p.M + KP - 1) / KP);
    const long long tiles = (long long)ntn * ntc * taps;
    long long splits = (wgrad_target_blocks() + tiles - 1) / tiles;  // about two blocks per CU
    const long long max_splits = (p.nst + 3) / 4;  // >= 4 stages per split
    if (splits > max_splits) splits = max_splits;
    splits = ws_cap_splits(p, splits);
    if (splits < 1) splits = 1;
    p.sps = (int)((p.nst + splits - 1) / splits);
    splits = (p.nst + p.sps - 1) / p.sps;
    YXH_CHECK_ARG(ntn < 65536 && ntc * taps < 65536, "wgrad grid");
    hipLaunchKernelGGL((wgrad_f32<TN, TC, WN, WC, KP>), dim3((unsigned)splits, ntn, ntc * taps), dim3(256), 0, st, p);
    YXH_CHECK_LAUNCH("wgrad_f32");
    return ws_reduce(p, splits, st);
}

template <int TN, int TC, int S, int KP>
int launch_wgrad9t_f32(WgradParams p, hipStream_t st) {
    if (p.kh != 3 || p.kw != 3 || p.stride != S || p.pad != 1) {
        set_error("wgrad tiles 21-24 (fp32, nine taps per block) need a 3x3 pad-1 conv of stride %d", S);
        return YXH_EUNSUPPORTED;
    }
    if ((p.nsrc > 1 && p.src0_ch % 4) || p.dycs % 4 || p.dybs % 4 || p.cin % 4) {
        set_error("wgrad tiles 21-24: 16-byte channel chunks");
        return YXH_EUNSUPPORTED;
    }
    const int nseg = (p.out_w + KP - 1) / KP;
    const int ntn = (p.cout + TN - 1) / TN, ntc = (p.cin + TC - 1) / TC;
    p.nst = p.B * p.out_h * nseg;
    const long long tiles = (long long)ntn * ntc;
    long long splits = (wgrad_target_blocks() + tiles - 1) / tiles;
    const long long max_splits = (p.nst + 3) / 4;
    if (splits > max_splits) splits = max_splits;
    splits = ws_cap_splits(p, splits);
    if (splits < 1) splits = 1;
    p.sps = (int)((p.nst + splits - 1) / splits);
    splits = (p.nst + p.sps - 1) / p.sps;
    YXH_CHECK_ARG(ntn < 65536 && ntc < 65536, "wgrad grid");
    hipLaunchKernelGGL((wgrad9t_f32<TN, TC, S, KP>), dim3((unsigned)splits, ntn, ntc), dim3(256), 0, st, p, nseg);
    YXH_CHECK_LAUNCH("wgrad9t_f32");
    return ws_reduce(p, splits, st);
}

template <typename T, int TN, int TC, int S, int KP>
int launch_wgrad9t_h(WgradParams p, hipStream_t st) {
    if constexpr (sizeof(T) != 2) {
        set_error("wgrad tiles 25-28 (nine taps per block, transposed LDS reads) are built for bf16/f16 only");
        return YXH_EUNSUPPORTED;
    } else {
        if (p.kh != 3 || p.kw != 3 || p.stride != S || p.pad != 1) {
            set_error("wgrad tiles 25-28 (nine taps per block) need a 3x3 pad-1 conv of stride %d", S);
            return YXH_EUNSUPPORTED;
        }
        // 16-byte channel chunks everywhere (conv_wgrad_launch checks the views; src0_ch too)
        if (p.nsrc > 1 && p.src0_ch % 8) {
            set_error("wgrad tiles 25-28: 16-byte channel chunks");
            return YXH_EUNSUPPORTED;
        }
        const int nseg = (p.out_w + KP - 1) / KP;
        const int ntn = (p.cout + TN - 1) / TN, ntc = (p.cin + TC - 1) / TC;
        p.nst = p.B * p.out_h * nseg;
        const long long tiles = (long long)ntn * ntc;
        long long splits = (wgrad_target_blocks() + tiles - 1) / tiles;
        const long long max_splits = (p.nst + 3) / 4;
        if (splits > max_splits) splits = max_splits;
        splits = ws_cap_splits(p, splits, 16LL << 20);
        if (splits < 1) splits = 1;
        p.sps = (int)((p.nst + splits - 1) / splits);
        splits = (p.nst + p.sps - 1) / p.sps;
        YXH_CHECK_ARG(ntn < 65536 && ntc < 65536, "wgrad grid");
        hipLaunchKernelGGL((wgrad9t_h<T, TN, TC, S, KP>), dim3((unsigned)splits, ntn, ntc), dim3(256), 0, st, p, nseg);
        YXH_CHECK_LAUNCH("wgrad9t_h");
        return ws_reduce(p, splits, st);
    }
}

template <typename T>
int wgrad_tile(int tile, const WgradParams& p, hipStream_t st) {
    // default: 64 x 64 (cout x cin), 2 x 2 waves; 4 slabs (bf16: 128 pixels) per stage
    switch (tile) {
        case 0:  // by shape: the smallest tile that covers cout, wide tiles for wide layers
            if (p.cout <= 16) return wgrad_tile<T>(4, p, st);
            if (p.cout <= 32) return wgrad_tile<T>(3, p, st);
            if (p.cout >= 128 && p.cin >= 128) return wgrad_tile<T>(2, p, st);
            return wgrad_tile<T>(1, p, st);
        case 1: return sizeof(T) == 4 ? launch_wgrad_t<T, 64, 64, 2, 2, 2>(p, st) : launch_wgrad_t<T, 64, 64, 2, 2, 4>(p, st);
        case 2: return launch_wgrad_t<T, 128, 128, 2, 2, 2>(p, st);
        case 3: return launch_wgrad_t<T, 32, 64, 1, 4, 2>(p, st);
        case 4: return launch_wgrad_t<T, 16, 64, 1, 4, 2>(p, st);
        case 5: return launch_wgrad2_t<T, 128, 128, 3>(p, st);
        case 6: return launch_wgrad2_t<T, 128, 128, 2>(p, st);
        case 7: return launch_wgrad2_t<T, 64, 64, 3>(p, st);
        case 8: return launch_wgrad2_t<T, 64, 64, 2>(p, st);
        case 9: return launch_wgrad2_t<T, 128, 64, 3>(p, st);
        case 10: return launch_wgrad2_t<T, 64, 128, 3>(p, st);
        case 11: case 12: case 13: case 14: case 15: case 16:
            if constexpr (sizeof(T) != 4) {
                set_error("wgrad tiles 11-16 (all nine taps per block) are built for fp32 only");
                return YXH_EUNSUPPORTED;
            } else {
                const bool s2 = p.stride == 2;
                switch (tile) {
                    case 11: return s2 ? launch_wgrad9_t<2, 32, 32, 2, 2, 4>(p, st) : launch_wgrad9_t<1, 32, 32, 2, 2, 8>(p, st);
                    case 12: return s2 ? launch_wgrad9_t<2, 64, 32, 2, 2, 4>(p, st) : launch_wgrad9_t<1, 64, 32, 2, 2, 8>(p, st);
                    case 13: return s2 ? launch_wgrad9_t<2, 64, 64, 2, 2, 2>(p, st) : launch_wgrad9_t<1, 64, 64, 2, 2, 4>(p, st);
                    case 14: return s2 ? launch_wgrad9_t<2, 32, 16, 2, 1, 4>(p, st) : launch_wgrad9_t<1, 32, 16, 2, 1, 8>(p, st);
                    case 15: return s2 ? launch_wgrad9_t<2, 32, 32, 2, 2, 2>(p, st) : launch_wgrad9_t<1, 32, 32, 2, 2, 4>(p, st);
                    default: return s2 ? launch_wgrad9_t<2, 64, 16, 4, 1, 4>(p, st) : launch_wgrad9_t<1, 64, 16, 4, 1, 8>(p, st);
                }
            }
        case 17: case 18: case 19: case 20:
            if constexpr (sizeof(T) != 4) {
                set_error("wgrad tiles 17-20 (k-major MFMA operands) are built for fp32 only");
                return YXH_EUNSUPPORTED;
            } else {
                switch (tile) {
                    case 17: return launch_wgrad_f32<64, 64, 2, 2, 32>(p, st);
                    case 18: return launch_wgrad_f32<128, 128, 2, 2, 16>(p, st);
                    case 19: return launch_wgrad_f32<128, 64, 2, 2, 32>(p, st);
                    default: return launch_wgrad_f32<64, 128, 2, 2, 32>(p, st);
                }
            }
        case 21: case 22: case 23: case 24:
            if constexpr (sizeof(T) != 4) {
                set_error("wgrad tiles 21-24 (nine taps per block, k-major operands) are built for fp32 only");
                return YXH_EUNSUPPORTED;
            } else {
                const bool s2 = p.stride == 2;
                switch (tile) {
                    case 21: return s2 ? launch_wgrad9t_f32<64, 64, 2, 16>(p, st) : launch_wgrad9t_f32<64, 64, 1, 16>(p, st);
                    case 22: return s2 ? launch_wgrad9t_f32<64, 64, 2, 8>(p, st) : launch_wgrad9t_f32<64, 64, 1, 32>(p, st);
                    case 23: return s2 ? launch_wgrad9t_f32<32, 64, 2, 16>(p, st) : launch_wgrad9t_f32<32, 64, 1, 16>(p, st);
                    default: return s2 ? launch_wgrad9t_f32<64, 32, 2, 16>(p, st) : launch_wgrad9t_f32<64, 32, 1, 16>(p, st);
                }
            }
        case 25: case 26: case 27: case 28: case 29: case 30: {
            const bool s2 = p.stride == 2;
            switch (tile) {
                // 160 x 32 / 32 x 160 (round 5): yolox_x's 160-channel 3x3s in whole tiles (64 x 64 covers
                // 160 x 160 with 3 x 3 tiles = 1.44x the MFMA work), five 16-row fragments per wave
                case 29: return s2 ? launch_wgrad9t_h<T, 160, 32, 2, 32>(p, st) : launch_wgrad9t_h<T, 160, 32, 1, 32>(p, st);
                case 30: return s2 ? launch_wgrad9t_h<T, 32, 160, 2, 32>(p, st) : launch_wgrad9t_h<T, 32, 160, 1, 32>(p, st);
                case 25: return s2 ? launch_wgrad9t_h<T, 64, 64, 2, 32>(p, st) : launch_wgrad9t_h<T, 64, 64, 1, 32>(p, st);
                case 26: return s2 ? launch_wgrad9t_h<T, 128, 64, 2, 32>(p, st) : launch_wgrad9t_h<T, 128, 64, 1, 32>(p, st);
                case 27:  // stride 2 would stage 13 chunks per lane beside 288 accumulators: spills
                    if (s2) {
                        set_error("wgrad tile 27 is stride-1 only");
                        return YXH_EUNSUPPORTED;
                    }
                    return launch_wgrad9t_h<T, 64, 128, 1, 32>(p, st);
                default: return s2 ? launch_wgrad9t_h<T, 64, 64, 2, 64>(p, st) : launch_wgrad9t_h<T, 64, 64, 1, 64>(p, st);
            }
        }
        default: set_error("wgrad tile %d", tile); return YXH_EINVAL;
    }
}

}  // namespace

int conv_wgrad_launch(const yxh_wgrad_desc* d, hipStream_t st) {
    YXH_CHECK_ARG(d, "null descriptor");
    const int dt = d->dtype;
    YXH_CHECK_ARG(dt == YXH_F32 || dt == YXH_BF16 || dt == YXH_F16, "wgrad dtype %d", dt);
    const int epc = 16 / esz(dt);
    YXH_CHECK_ARG(d->batch > 0 && d->cin > 0 && d->cout > 0 && d->kh > 0 && d->kw > 0 && d->stride > 0,
                  "wgrad geometry");
    YXH_CHECK_ARG((d->in_h + 2 * d->pad - d->kh) / d->stride + 1 == d->out_h &&
                      (d->in_w + 2 * d->pad - d->kw) / d->stride + 1 == d->out_w,
                  "wgrad output size mismatch");
    YXH_CHECK_ARG(d->nsrc == 1 || d->nsrc == 2, "nsrc %d", d->nsrc);
    int chs = 0;
    for (int s = 0; s < d->nsrc; ++s) {
        const yxh_src& q = d->src[s];
        YXH_CHECK_ARG(q.ptr && a16(q.ptr) && q.channels % epc == 0 && q.cstride % epc == 0 && q.bstride % epc == 0,
                      "wgrad src%d alignment / channels", s);
        YXH_CHECK_ARG(q.upsample == 0 || q.upsample == 1, "wgrad src%d upsample %d", s, q.upsample);
        YXH_CHECK_ARG((q.h << q.upsample) == d->in_h && (q.w << q.upsample) == d->in_w, "wgrad src%d spatial", s);
        chs += q.channels;
    }
    YXH_CHECK_ARG(chs == d->cin, "wgrad source channels %d != cin %d", chs, d->cin);
    const yxh_src& g = d->dy;
    YXH_CHECK_ARG(g.ptr && a16(g.ptr) && g.channels % epc == 0 && g.channels >= d->cout && g.cstride % epc == 0 &&
                      g.bstride % epc == 0 && g.h == d->out_h && g.w == d->out_w && g.upsample == 0,
                  "wgrad dy view (channels %d must cover cout %d in %d-element chunks)", g.channels, d->cout, epc);
    YXH_CHECK_ARG(d->dw && d->cin_store > 0 && d->cin_store <= d->cin, "wgrad dw / cin_store");
    WgradParams p{};
    p.in_h = d->in_h; p.in_w = d->in_w; p.out_h = d->out_h; p.out_w = d->out_w;
    p.cin = d->cin; p.cout = d->cout; p.kh = d->kh; p.kw = d->kw; p.stride = d->stride; p.pad = d->pad;
    p.ohw = d->out_h * d->out_w;
    const long long M = (long long)d->batch * p.ohw;
    YXH_CHECK_ARG(M < (1LL << 31), "too many pixels");
    p.M = (int)M;
    p.B = d->batch;
    YXH_CHECK_ARG((long long)d->out_h * d->out_w * g.cstride < (1LL << 31) &&
                      (long long)d->src[0].h * d->src[0].w * d->src[0].cstride < (1LL << 31),
                  "wgrad: per-image offsets exceed 32 bits");
    p.nsrc = d->nsrc;
    p.src0_ch = d->src[0].channels;
    for (int s = 0; s < d->nsrc; ++s) {
        p.sptr[s] = d->src[s].ptr;
        p.scs[s] = d->src[s].cstride;
        p.sbs[s] = d->src[s].bstride;
        p.sw[s] = d->src[s].w;
        p.sup[s] = d->src[s].upsample;
    }
    p.dy = g.ptr;
    p.dycs = g.cstride;
    p.dybs = g.bstride;
    p.dw = d->dw;
    p.cin_store = d->cin_store;
    p.dych = g.channels;
    YXH_CHECK_ARG(!d->workspace || a16(d->workspace), "wgrad workspace alignment");
    p.ws = (float*)d->workspace;
    p.ws_elems = d->workspace ? d->workspace_bytes / 4 : 0;
    if (dt == YXH_BF16) return wgrad_tile<bf16>(d->tile, p, st);
    if (dt == YXH_F16) return wgrad_tile<f16>(d->tile, p, st);
    return wgrad_tile<float>(d->tile, p, st);
}

int pack_dgrad_launch(const float* w, int cout, int cin, int kh, int kw, int c_begin, int c_count, int cout_pad, int dt,
                      void* out, hipStream_t st) {
    YXH_CHECK_ARG(w && out && a16(out), "pack_dgrad: null / unaligned");
    YXH_CHECK_ARG(cout > 0 && cin > 0 && kh > 0 && kw > 0 && c_begin >= 0 && c_count > 0 && c_begin + c_count <= cin &&
                      cout_pad >= cout,
                  "pack_dgrad geometry");
    const long long total = (long long)c_count * kh * kw * cout_pad;
    dim3 grid((unsigned)((total + 255) / 256));
    if (dt == YXH_BF16) hipLaunchKernelGGL(pack_dgrad<bf16>, grid, dim3(256), 0, st, w, cout, cin, kh, kw, c_begin, c_count, cout_pad, (bf16*)out);
    else if (dt == YXH_F16) hipLaunchKernelGGL(pack_dgrad<f16>, grid, dim3(256), 0, st, w, cout, cin, kh, kw, c_begin, c_count, cout_pad, (f16*)out);
    else if (dt == YXH_F32) hipLaunchKernelGGL(pack_dgrad<float>, grid, dim3(256), 0, st, w, cout, cin, kh, kw, c_begin, c_count, cout_pad, (float*)out);
    else {
        set_error("pack_dgrad dtype %d", dt);
        return YXH_EINVAL;
    }
    YXH_CHECK_LAUNCH("pack_dgrad");
    return YXH_OK;
}

int pack_batch_launch(const yxh_pack_job* jobs, int njobs, int total_blocks, int dt, hipStream_t st) {
    YXH_CHECK_ARG(jobs && njobs > 0 && total_blocks > 0, "pack_batch: empty job table");
    if (dt == YXH_BF16) hipLaunchKernelGGL(pack_batch<bf16>, dim3(total_blocks), dim3(256), 0, st, jobs, njobs);
    else if (dt == YXH_F16) hipLaunchKernelGGL(pack_batch<f16>, dim3(total_blocks), dim3(256), 0, st, jobs, njobs);
    else if (dt == YXH_F32) hipLaunchKernelGGL(pack_batch<float>, dim3(total_blocks), dim3(256), 0, st, jobs, njobs);
    else {
        set_error("pack_batch dtype %d", dt);
        return YXH_EINVAL;
    }
    YXH_CHECK_LAUNCH("pack_batch");
    return YXH_OK;
}

int spp_bwd_launch(int dt, int B, const yxh_src* cat, int c, const float* dcat, float* dx, hipStream_t st) {
    YXH_CHECK_ARG(cat && cat->ptr && dcat && dx && B > 0 && c > 0 && cat->cstride >= 4 * c, "spp_bwd arguments");
    const int HW = cat->h * cat->w;
    // LDS per channel and pixel: brow + hcol u16 [3] each, plane / row max / gradient f32
    constexpr size_t kPer = 6 + 6 + 12;
    const int cpb = (size_t)HW * 4 * kPer <= 160 * 1024 ? 4 : (size_t)HW * 2 * kPer <= 160 * 1024 ? 2 : 1;
    const size_t lds = (size_t)HW * cpb * kPer;
    YXH_CHECK_ARG(lds <= 160 * 1024 && HW < 65536, "spp_bwd plane %dx%d too large for LDS", cat->h, cat->w);
    dim3 grid((c + cpb - 1) / cpb, B);
    TView v = tview(cat, c);
#define YXH_SPPB(T, P)                                                                                     \
    do {                                                                                                   \
        (void)hipFuncSetAttribute((const void*)spp_bwd<T, P>, hipFuncAttributeMaxDynamicSharedMemorySize,  \
                                  (int)lds);                                                               \
        hipLaunchKernelGGL((spp_bwd<T, P>), grid, dim3(1024), lds, st, v, cat->h, cat->w, c, dcat, dx, B); \
    } while (0)
#define YXH_SPPB_T(T)                 \
    do {                              \
        if (cpb == 4) YXH_SPPB(T, 4); \
        else if (cpb == 2) YXH_SPPB(T, 2); \
        else YXH_SPPB(T, 1);          \
    } while (0)
    if (dt == YXH_BF16) YXH_SPPB_T(bf16);
    else if (dt == YXH_F16) YXH_SPPB_T(f16);
    else YXH_SPPB_T(float);
#undef YXH_SPPB_T
#undef YXH_SPPB
    YXH_CHECK_LAUNCH("spp_bwd");
    return YXH_OK;
}

int upsample_bwd_launch(const float* g, int B, int h, int w, int C, float* dst, hipStream_t st) {
    YXH_CHECK_ARG(g && dst && a16(g) && a16(dst) && B > 0 && h > 0 && w > 0 && C > 0 && C % 4 == 0,
                  "upsample_bwd arguments");
    const long long total = (long long)B * h * w * (C / 4);
    hipLaunchKernelGGL(upsample_bwd, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, g, B, h, w, C, dst);
    YXH_CHECK_LAUNCH("upsample_bwd");
    return YXH_OK;
}

}  // namespace yxh
