// conv_ws1: weight-stationary persistent 1x1 conv (16-bit) over dense sources -- the
// 1x1 BaseConvs of CspLayer (network_blocks.py:160-183 conv1 | conv2 and conv3 over the
// concat), SPPBottleneck (:107-116), the PAFPN lateral / reduce convs (yolo_pafpn.py:58-64)
// and the head stems (yolo_head.py:52-56).
//
// The 1x1 form of conv_ws.hip: a block keeps its TN output channels x all of K in VGPRs
// for its life and walks pixel tiles of TM consecutive pixels of the flattened batch; per
// tile only the pixel rows land in LDS (LDS-DMA, two buffers), the next tile's rows fly
// while this tile computes, and the epilogue of tile k-1 is spread over tile k's MFMAs.
// Two sources (a channel concat) occupy two LDS regions of the same pixel stride, so every
// 1 KiB DMA reads one source; a K step (32 channels) lies inside one source.
#include "conv_common.hpp"
#include "lds_dma.hpp"

namespace yxh {

// V16: 16-byte epilogue stores -- channel fragments i and i + 1 of a pixel fragment are exchanged
// between lane rows by v_permlane16_swap so that every lane holds 8 consecutive channels of its
// pixel (half the store instructions and offset computations of the 8-byte form)
template <typename T, int CIN, int TM, int TN, int WN, int WK, int WM, int BPC, int NBUF, bool UP0, bool V16>
__global__ __launch_bounds__(64 * WN * WK * WM, BPC) void conv_ws1(ConvParams p, int ntiles, int ntn, int nwork,
                                                                    int ps, int l0, int l1) {
    static_assert(sizeof(T) == 2, "16-bit operands");
    constexpr int NW = WN * WK * WM;
    constexpr int NCB = CIN / 32, WCB = NCB / WK;
    constexpr int WTN = TN / WN, FR = WTN / 16;
    constexpr int WTM = TM / WM, FC = WTM / 16;
    constexpr int C16 = CIN / 8;
    // LDS image bound: two regions of TM pixels x ps 16-byte slots (ps padded up to 2 x odd,
    // at most 3 slots per region), each rounded up to whole 1 KiB wave-loads; a buffer holds
    // GB wave-loads of every wave (the ones past the image land zeros in the padding), so each
    // wave issues exactly GB DMAs per tile and the pipeline's vmcnt waits are constants.
    // NBUF buffers: NBUF - 1 tiles' rows in flight while one computes
    constexpr int LMAX = (TM * (C16 + 6) + 63) / 64 + 2, GB = (LMAX + NW - 1) / NW, HBYTES = GB * NW * 1024;
    constexpr int RBYTES = WK > 1 ? WN * WM * FR * FC * (WK - 1) * 1024 : 0;
    constexpr int SMEM = NBUF * HBYTES + RBYTES;
    static_assert(NBUF >= 2 && (NBUF - 1) * GB <= 63, "DMA pipeline depth");
    constexpr int FCO = (FC + WK - 1) / WK;
    constexpr int PD = FR * FC >= 8 ? 1 : FR * FC >= 4 ? 2 : 3;  // fragment-read distance in K steps
    static_assert(NCB % WK == 0 && WTN % 16 == 0 && WTM % 16 == 0, "tile");
    static_assert(FR * WCB * 4 <= (NW == 4 && BPC == 1 ? 288 : 160), "weights must stay in VGPRs");
    static_assert(SMEM <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wave % WN, wk = (wave / WN) % WK, wm = wave / (WN * WK);
    const int frow = lane & 15, fq = lane >> 4;
    const int bid = dma::xcd_remap(blockIdx.x, gridDim.x);
    const int nt = bid % ntn, worker = bid / ntn;
    const int n0 = nt * TN;
    const int tile = worker;
    if (tile >= ntiles) return;  // block-uniform
    const int M = p.M, cout = p.cout, dcs = p.dst_cs;
    const int c0 = p.src0_ch, ncb0 = c0 / 32;
    const int c1 = CIN - c0;

    uint32_t boff[FC];
#pragma unroll
    for (int j = 0; j < FC; ++j) boff[j] = (uint32_t)(((wm * FC + j) * 16 + frow) * ps * 16 + fq * 16);

    // per-lane DMA slot geometry: pixel of the tile | 16-byte chunk << 16 (-1: pad slot)
    int geo[GB];
#pragma unroll
    for (int i = 0; i < GB; ++i) {
        const int L = wave + NW * i;
        const int r = L < l0 ? 0 : 1;
        const int s = 64 * (L - r * l0) + lane;
        const int hp = s / ps, ch = s - hp * ps;
        const bool st = L < l0 + l1 && hp < TM && ch < (r ? c1 : c0) / 8;
        geo[i] = st ? (hp | (ch << 16)) : -1;
    }
    const uint32_t lds0 = dma::lds_addr(smem);
    // UP0: source 0 is read through a nearest x2 upsample (yxh_src.upsample = 1: the PAFPN's
    // upsampled lateral / reduce map in C3_p4 / C3_p3's conv1 | conv2, yolo_pafpn.py:98-112)
    const long long src0_elems = UP0 ? (long long)(M / p.ohw) * p.sbs[0] : (long long)M * p.scs[0];
    const dma::u32x4 srd0 = dma::srd(p.sptr[0], (uint32_t)(src0_elems * 2));
    const int ohw = p.ohw, ow = p.out_w, sw0 = p.sw[0];
    const long long sbs0 = p.sbs[0];
    const dma::u32x4 srd1 = dma::srd(p.nsrc > 1 ? p.sptr[1] : p.sptr[0],
                                     (uint32_t)((long long)M * (p.nsrc > 1 ? p.scs[1] : p.scs[0]) * 2));
    const int scs0 = p.scs[0], scs1 = p.nsrc > 1 ? p.scs[1] : 0;

    // tile t's rows into buffer kb; a tile past the end (t >= ntiles) loads zeros, so the count
    // of DMAs per wave and tile is always GB
    auto issue = [&](int t, int kb) {
        const int m0 = t * TM;
#pragma unroll
        for (int i = 0; i < GB; ++i) {
            const int L = wave + NW * i;
            {
                const int g = geo[i];
                const int m = m0 + (g & 0xffff);
                const bool ok = g >= 0 && m < M;
                const uint32_t ldsa = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(kb * HBYTES + L * 1024));
                const bool r0 = L < l0;  // wave-uniform: the DMA reads one source
                dma::u32x4 rs = r0 ? srd0 : srd1;
                rs.x = __builtin_amdgcn_readfirstlane(rs.x);
                rs.y = __builtin_amdgcn_readfirstlane(rs.y);
                rs.z = __builtin_amdgcn_readfirstlane(rs.z);
                rs.w = __builtin_amdgcn_readfirstlane(rs.w);
                long long e = (long long)m * (r0 ? scs0 : scs1);
                if (UP0 && r0) {  // pixel m = (b, y, x) reads source pixel (b, y / 2, x / 2)
                    const int b = m / ohw, rr = m - b * ohw, y = rr / ow, x = rr - y * ow;
                    e = b * sbs0 + ((long long)(y >> 1) * sw0 + (x >> 1)) * scs0;
                }
                const uint32_t voff = ok ? (uint32_t)((e + (g >> 16) * 8) * 2) : dma::kOob;
                dma::load16(rs, voff, 0u, ldsa);
            }
        }
    };

    // prologue: the first NBUF tiles' rows go out before the weights, which then load in the
    // order the first tile's K steps consume them (tile_step's FIRST waits for tile 0 only)
#pragma unroll
    for (int q = 0; q < NBUF; ++q) issue(tile + q * nwork, q);
    uint4 a[FR][WCB];
#pragma unroll
    for (int c = 0; c < WCB; ++c)
#pragma unroll
        for (int i = 0; i < FR; ++i) a[i][c] = ws_weight<T>(p, n0 + wn * WTN + i * 16, 0, 1, CIN, wk * WCB + c, lane);
    float bias[FR][4];
#pragma unroll
    for (int i = 0; i < FR; ++i) {
        const int n = n0 + wn * WTN + i * 16 + fq * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[i][r] = n + r < cout ? p.bias[n + r] : 0.0f;
    }

    const bool silu = p.act == YXH_ACT_SILU;
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const __amdgpu_buffer_rsrc_t dsrd =
        __builtin_amdgcn_make_buffer_rsrc(p.dst, (short)0, (int)((long long)M * dcs * 2), 0x00020000);
    auto epi_piece = [&](const int tprev, const f32x4 (&ap)[FR][FCO], const int o, const int i) {
        const int j = wk + WK * o;
        const int m = tprev * TM + (wm * FC + j) * 16 + frow;
        const int n = n0 + wn * WTN + i * 16 + fq * 4;
        const bool ok = j < FC && m < M && n < cout;
        const int od = ok ? (m * dcs + n) * 2 : (int)dma::kOob;
        const f32x4 x = ap[i][o] + f32x4{bias[i][0], bias[i][1], bias[i][2], bias[i][3]};
        const f32x4 v = silu ? yxh::silu4(x) : x;
        T t[4] = {from_f32<T>(v[0]), from_f32<T>(v[1]), from_f32<T>(v[2]), from_f32<T>(v[3])};
        u32x2 u;
        __builtin_memcpy(&u, t, 8);
        __builtin_amdgcn_raw_buffer_store_b64(u, dsrd, od, 0, 0);
    };

    // V16: one piece = pixel fragment o x channel fragments 2 ip, 2 ip + 1.  Before the swap lane (frow,
    // fq) holds channels 4 fq .. +4 of both fragments; v_permlane16_swap trades fragment 2 ip's values
    // of odd lane rows for fragment 2 ip + 1's of even ones, so row fq ends up with the 8 channels
    // 16 (fq & 1) + 8 (fq >> 1) .. +8 of the fragment pair (rows 0 / 2: fragment 2 ip, rows 1 / 3: 2 ip + 1)
    auto epi_piece16 = [&](const int tprev, const f32x4 (&ap)[FR][FCO], const int o, const int ip) {
        const int j = wk + WK * o;
        const int i0 = 2 * ip;
        const int m = tprev * TM + (wm * FC + j) * 16 + frow;
        const int n = n0 + wn * WTN + i0 * 16 + (fq & 1) * 16 + (fq >> 1) * 8;
        const bool ok = j < FC && m < M && n < cout;
        const int od = ok ? (m * dcs + n) * 2 : (int)dma::kOob;
        uint32_t w[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = i0 + h;
            const f32x4 x = ap[i][o] + f32x4{bias[i][0], bias[i][1], bias[i][2], bias[i][3]};
            const uint2 pk = pack4<T>(silu ? yxh::silu4(x) : x);  // two paired conversions
            w[h][0] = pk.x;
            w[h][1] = pk.y;
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const auto r = __builtin_amdgcn_permlane16_swap(w[0][q], w[1][q], false, false);
            w[0][q] = r[0];
            w[1][q] = r[1];
        }
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 u = {w[0][0], w[0][1], w[1][0], w[1][1]};
        __builtin_amdgcn_raw_buffer_store_b128(u, dsrd, od, 0, 0);
    };

    f32x4 accp[FR][FCO];
    static_assert(!V16 || FR % 2 == 0, "16-byte epilogue pairs channel fragments");
    constexpr int NP = V16 ? FR / 2 * FCO : FR * FCO;  // epilogue pieces
    constexpr int PFR = V16 ? FR / 2 : FR;             // pieces per pixel fragment
    // K steps between pieces: a 16-byte piece carries two fragments' epilogue, so it rides every other
    // step while the K loop has room (the 8-byte pieces: every step)
    constexpr int PSP = V16 && 2 * NP <= WCB ? 2 : 1;
    auto piece = [&](const int tprev, const f32x4 (&ap)[FR][FCO], const int q) {
        if constexpr (V16) epi_piece16(tprev, ap, q / PFR, q % PFR);
        else epi_piece(tprev, ap, q / FR, q % FR);
    };
    auto tile_step = [&](const int t, const int k, const int tprev, auto epi, auto first) -> int {
        constexpr bool EPI = decltype(epi)::value;
        constexpr bool FIRST = decltype(first)::value;
        const int kb = k % NBUF;
        const int next = t + nwork;
        // vmcnt retires in issue order.  FIRST: tiles 1 .. NBUF-1 and the weights went out after
        // tile 0's rows; later steps: at least tiles k+1 .. k+NBUF-2 did (GB DMAs each)
        if constexpr (FIRST) {
            constexpr int younger = (NBUF - 1) * GB + FR * WCB;
            dma::wait_vm<(younger < 63 ? younger : 63)>();
        } else {
            dma::wait_vm<(NBUF - 2) * GB>();
        }
        dma::barrier();
        // the buffer of tile k-1 is free: tile k + NBUF - 1 into it (the prologue issued tile NBUF-1)
        if (!FIRST) issue(t + (NBUF - 1) * nwork, (k + NBUF - 1) % NBUF);

        f32x4 acc[FR][FC];
#pragma unroll
        for (int i = 0; i < FR; ++i)
#pragma unroll
            for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        const char* hb = smem + kb * HBYTES;
        // pixel fragments read PD K steps ahead (conv_ws.hip: about 8 MFMAs of cover)
        uint4 bf[PD + 1][FC];
        auto load_b = [&](int s, uint4 (&d)[FC]) {
            const int cg = wk * WCB + s;
            const int so = cg < ncb0 ? cg * 64 : l0 * 1024 + (cg - ncb0) * 64;
#pragma unroll
            for (int j = 0; j < FC; ++j) d[j] = *(const uint4*)(hb + boff[j] + so);
        };
#pragma unroll
        for (int q = 0; q < PD; ++q)
            if (q < WCB) load_b(q, bf[q]);
        __builtin_amdgcn_sched_group_barrier(0x100, FC * (PD < WCB ? PD : WCB), 0);
#pragma unroll
        for (int s = 0; s < WCB; ++s) {
            if (s + PD < WCB) load_b(s + PD, bf[(s + PD) % (PD + 1)]);
#pragma unroll
            for (int j = 0; j < FC; ++j)  // pixel-fragment-major (conv_ws.hip): more cover for the next reads
#pragma unroll
                for (int i = 0; i < FR; ++i) Mma<T>::run(acc[i][j], a[i][s], bf[s % (PD + 1)][j]);
            if constexpr (EPI)
                if (s % PSP == 0 && s / PSP < NP) piece(tprev, accp, s / PSP);
            if (s + PD < WCB) __builtin_amdgcn_sched_group_barrier(0x100, FC, 0);
#pragma unroll
            for (int m = 0; m < FR * FC; ++m) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if constexpr (EPI) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
            }
        }
        if constexpr (EPI)
#pragma unroll
            for (int q = (WCB + PSP - 1) / PSP; q < NP; ++q) piece(tprev, accp, q);

        if constexpr (WK > 1) {
            char* red = smem + NBUF * HBYTES;  // past every row buffer (NBUF - 1 tiles are in flight)
            const int grp = wm * WN + wn;
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) {
                    const int own = j % WK;
                    if (own != wk) {
                        const int slot = wk < own ? wk : wk - 1;
                        *(f32x4*)(red + (((grp * FR + i) * FC + j) * (WK - 1) + slot) * 1024 + lane * 16) = acc[i][j];
                    }
                }
            dma::barrier();
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j)
                    if (j % WK == wk) {
                        f32x4 v = acc[i][j];
#pragma unroll
                        for (int o = 0; o < WK - 1; ++o)
                            v += *(const f32x4*)(red + (((grp * FR + i) * FC + j) * (WK - 1) + o) * 1024 + lane * 16);
                        accp[i][j / WK] = v;
                    }
        } else {
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) accp[i][j] = acc[i][j];
        }
        return next;
    };

    int cur = tile;
    int next = tile_step(cur, 0, 0, std::false_type{}, std::true_type{});
    int k = 1;
    for (; next < ntiles; ++k) {
        const int prev = cur;
        cur = next;
        next = tile_step(cur, k, prev, std::true_type{}, std::false_type{});
    }
#pragma unroll
    for (int q = 0; q < NP; ++q) piece(cur, accp, q);
    dma::wait_vm<0>();  // the zero-filling DMAs of tiles past the end land before the LDS is released
}

template <typename T, int CIN, int TM, int TN, int WN, int WK, int WM, int BPC = 1, int NBUF = 2, bool UP0 = false>
static int launch_ws1(const ConvParams& p, hipStream_t st) {
    if (p.cin != CIN) {
        set_error("conv_ws1 variant built for %d input channels", CIN);
        return YXH_EUNSUPPORTED;
    }
    const int c0 = p.src0_ch, c1 = CIN - c0;
    // UP0 variants: source 0 upsampled x2 (nearest), source 1 dense; the others: dense sources
    const bool srcs_ok = UP0 ? (p.nsrc == 2 && p.sup[0] == 1 && p.sup[1] == 0 && p.sw[0] * 2 == p.out_w &&
                                p.sw[1] == p.out_w && p.sbs[1] == (long long)p.ohw * p.scs[1] &&
                                (long long)(p.M / p.ohw) * p.sbs[0] * 2 < (1LL << 31))
                             : (bool)p.src_dense;
    if (!srcs_ok || !p.dst_dense || p.dst_f32 || p.accum || p.res || p.pw1 || p.grp2 ||
        (p.act != YXH_ACT_SILU && p.act != YXH_ACT_NONE) || p.cout % 8 || c0 % 32 || c1 % 32 ||
        (p.nsrc == 1) != (c1 == 0)) {
        set_error("conv_ws1: dense 1x1 over 32-channel-aligned sources, 16-bit dst, SiLU/no activation, %d input channels",
                  CIN);
        return YXH_EUNSUPPORTED;
    }
    const long long M = p.M;
    if (M * p.scs[0] * 2 >= (1LL << 31) || (p.nsrc > 1 && M * p.scs[1] * 2 >= (1LL << 31)) ||
        M * p.dst_cs * 2 >= (1LL << 31)) {
        set_error("conv_ws1: tensors exceed 31-bit byte offsets");
        return YXH_EUNSUPPORTED;
    }
    // one pixel stride for both regions, 2 x odd 16-byte slots (conflict-free fragment reads)
    int ps = std::max(c0, c1) / 8;
    ps += (6 - ps % 4) % 4;
    const int l0 = (TM * ps + 63) / 64, l1 = c1 ? (TM * ps + 63) / 64 : 0;
    if (l0 + l1 > (TM * (CIN / 8 + 6) + 63) / 64 + 2) {
        set_error("conv_ws1: source split %d + %d does not fit the LDS image", c0, c1);
        return YXH_EUNSUPPORTED;
    }
    const long long ntiles = (M + TM - 1) / TM;
    const int ntn = (p.cout + TN - 1) / TN;
    const int nwork = (int)std::min<long long>(ntiles, std::max(1, p.cus * BPC / ntn));
    constexpr bool PAIRS = (TN / WN / 16) % 2 == 0;  // channel fragments per wave even: 16-byte stores
    if (p.v16_req && !PAIRS) {
        set_error("conv_ws1 tile has no 16-byte epilogue (an odd number of channel fragments per wave)");
        return YXH_EUNSUPPORTED;
    }
    if (PAIRS && p.v16_req && p.vec16)  // (conv.hip: v16_req = the odd tile codes)
        hipLaunchKernelGGL((conv_ws1<T, CIN, TM, TN, WN, WK, WM, BPC, NBUF, UP0, PAIRS>), dim3((unsigned)(nwork * ntn)),
                           dim3(64 * WN * WK * WM), 0, st, p, (int)ntiles, ntn, nwork, ps, l0, l1);
    else
        hipLaunchKernelGGL((conv_ws1<T, CIN, TM, TN, WN, WK, WM, BPC, NBUF, UP0, false>), dim3((unsigned)(nwork * ntn)),
                           dim3(64 * WN * WK * WM), 0, st, p, (int)ntiles, ntn, nwork, ps, l0, l1);
    YXH_CHECK_LAUNCH("conv_ws1 launch");
    return YXH_OK;
}

template <typename T>
static int ws1_dispatch_t(int id, const ConvParams& p, hipStream_t st) {
    // id -> (CIN, TM, TN, WN, WK, WM[, blocks per CU])
    switch (id) {
        case 1: return launch_ws1<T, 64, 128, 64, 2, 1, 2, 2>(p, st);
        case 2: return launch_ws1<T, 64, 256, 64, 2, 1, 4, 1>(p, st);
        case 3: return launch_ws1<T, 128, 64, 128, 4, 1, 1, 2>(p, st);
        case 4: return launch_ws1<T, 128, 128, 64, 2, 1, 2, 1>(p, st);  // 80 KiB of LDS: one block per CU
        case 5: return launch_ws1<T, 256, 64, 128, 4, 1, 1, 2>(p, st);
        case 6: return launch_ws1<T, 256, 64, 64, 2, 1, 2, 2>(p, st);
        case 7: return launch_ws1<T, 512, 32, 128, 4, 1, 1, 1>(p, st);
        case 8: return launch_ws1<T, 512, 64, 64, 2, 2, 2, 1>(p, st);
        case 9: return launch_ws1<T, 1024, 32, 64, 2, 2, 2, 1>(p, st);
        case 10: return launch_ws1<T, 256, 128, 128, 4, 1, 2, 1>(p, st);
        // deeper row pipelines (3-4 buffers: 2-3 tiles in flight), smaller tiles: the 1x1s were
        // latency-bound at one tile in flight (2-5x a copy of the same bytes, tools/pw_probe.py)
        case 11: return launch_ws1<T, 64, 64, 64, 2, 1, 2, 2, 4>(p, st);
        case 12: return launch_ws1<T, 128, 64, 128, 4, 1, 1, 1, 4>(p, st);
        case 13: return launch_ws1<T, 256, 32, 128, 4, 1, 1, 1, 4>(p, st);
        case 14: return launch_ws1<T, 256, 64, 128, 4, 1, 1, 1, 3>(p, st);
        case 15: return launch_ws1<T, 512, 32, 128, 4, 1, 1, 1, 3>(p, st);
        case 16: return launch_ws1<T, 512, 32, 64, 2, 2, 2, 1, 3>(p, st);
        case 17: return launch_ws1<T, 1024, 16, 64, 4, 1, 1, 1, 4>(p, st);
        case 18: return launch_ws1<T, 64, 128, 64, 2, 1, 2, 1, 3>(p, st);
        // [upsampled x2 | dense] sources: C3_p4's conv1 | conv2 (256 up + 256 @40x40 -> 256) and
        // C3_p3's (128 up + 128 @80x80 -> 128)
        case 19: return launch_ws1<T, 512, 32, 128, 4, 1, 1, 1, 3, true>(p, st);
        case 20: return launch_ws1<T, 512, 64, 64, 2, 2, 2, 1, 2, true>(p, st);
        case 21: return launch_ws1<T, 256, 64, 128, 4, 1, 1, 2, 2, true>(p, st);
        case 22: return launch_ws1<T, 256, 32, 128, 4, 1, 1, 1, 4, true>(p, st);
        // every output channel in one block (round 5): the 40x40 / 20x20 1x1s with 256 outputs read
        // their input ONCE instead of once per 128- / 64-channel slice (the re-read through LDS-DMA
        // was most of their time: 2.5-5.5x a copy of their bytes, profiles/r04/pw_probe_r4.txt);
        // 128 weight registers per wave (K split two ways past 256 input channels)
        // (two 4-wave blocks per CU / eight-wave blocks hold 256 registers per lane: 32-pixel tiles spilled)
        case 23: return launch_ws1<T, 256, 32, 256, 4, 1, 1, 1, 3>(p, st);
        case 24: return launch_ws1<T, 256, 64, 256, 4, 1, 1, 1, 3>(p, st);
        case 25: return launch_ws1<T, 512, 16, 256, 4, 2, 1, 1, 4>(p, st);
        case 26: return launch_ws1<T, 512, 16, 256, 4, 2, 1, 1, 4, true>(p, st);
        case 27: return launch_ws1<T, 128, 64, 256, 4, 1, 1, 1, 3>(p, st);
        case 28: return launch_ws1<T, 1024, 32, 128, 4, 2, 1, 1, 2>(p, st);
        default: set_error("conv_ws1 tile id %d", id); return YXH_EINVAL;
    }
}

int conv_ws1_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st) {
    if (p.taps != 1 || p.stride != 1 || p.pad != 0) {
        set_error("conv_ws1 needs a 1x1 s1 conv");
        return YXH_EUNSUPPORTED;
    }
    if (dtype == YXH_BF16) return ws1_dispatch_t<bf16>(id, p, st);
    if (dtype == YXH_F16) return ws1_dispatch_t<f16>(id, p, st);
    set_error("conv_ws1 is built for bf16/f16");
    return YXH_EUNSUPPORTED;
}

}  // namespace yxh
