// conv_ws: weight-stationary 3x3 conv (stride 1 or 2, pad 1) for 16-bit types.
// Reference: network_blocks.py:48-49 (BaseConv, ksize 3) as used by darknet.py:148-156
// (stage downsampling), network_blocks.py:77-99 (Bottleneck conv2), yolo_pafpn.py:55-80
// (bu_conv1/2) and yolo_head.py:57-104 (cls/reg convs).
//
// conv_r3 / conv_r3h stream the weights of their TN output channels through LDS for
// every pixel tile, and that weight DMA is what bounds them. Here a block
// is persistent and keeps its weights in VGPRs for its whole life: it loads them once,
// then walks pixel tiles. Per tile the only DMA is the input halo and the only LDS reads
// are the pixel fragments (half a ds_read_b128 per MFMA at FR = 2).
//
// Block: NW = WN x WK x WM waves. Wave (wn, wk, wm) holds output channels
// n0 + wn*WTN .. +WTN (FR = WTN/16 fragments) x input channel blocks wk*WCB .. +WCB
// (32 channels each) x all nine taps = FR*9*WCB*4 VGPRs, and computes pixel fragments
// wm*FC .. +FC of the TX x TY output tile. WK > 1 splits K: partial sums meet in LDS and
// each of the WK waves finishes every WK-th pixel fragment.
// Halo image in LDS: pixel (hy, hx) at hp = hy*HXP + hx, PS 16-byte slots per pixel.
// PS = 2 x odd (stride 1) / odd (stride 2) and HXP = TX mod 8 when fragments cross tile
// rows make the 16 pixels of a fragment hit distinct bank groups of ds_read_b128.
// Two halo buffers: tile k+1 lands by LDS-DMA while tile k computes.
#include "conv_common.hpp"
#include "lds_dma.hpp"

// Probe builds only (tools/ws_split.sh): 1 = no epilogue stores, 2 = no halo DMA after the
// first tile, 3 = both
#ifndef YXH_WS_PROBE
#define YXH_WS_PROBE 0
#endif

// probe builds: the fragment-read distance of the 8-MFMA-step tiles (0 = the default, 1)
#ifndef YXH_WS_PD8
#define YXH_WS_PD8 0
#endif

#ifndef YXH_WS_NPIN
#define YXH_WS_NPIN 48
#endif

// 1 (default): in the one-wave-per-SIMD tiles the activation is a compile-time property of the tile
// loop (one copy of the loop for SiLU, one for none, picked once per block), so no epilogue piece
// branches around its SiLU: the branch split every epilogue step into a basic block of its own, and
// the SiLU's exp / rcp ran with no MFMA beside them (head level-0 tile 109 -> 102 us).  The 256-register
// tiles keep the runtime test: a second loop copy spills them
#ifndef YXH_WS_ACT_CT
#define YXH_WS_ACT_CT 1
#endif

namespace yxh {

namespace {

// the value must live in AGPRs here (an empty asm with an "a" operand): the register allocator
// then keeps it there and the MFMAs read it in place
// a stationary weight fragment of a conv whose CR input channels are not a multiple of 32: row
// pieces of the [cout][9][CR] weights, zero past CR (the halo holds zeros there too)
template <typename T, int CR>
__device__ __forceinline__ uint4 ws_weight_padk(const ConvParams& p, int n_first, int tap, int kb, int lane) {
    const int frow = lane & 15, fq = lane >> 4;
    const int ch = kb * 32 + fq * 8;
    if (ch >= CR) return make_uint4(0, 0, 0, 0);
    const int n = min(n_first + frow, p.cout - 1);
    return *(const uint4*)((const T*)p.w + ((long long)n * 9 + tap) * CR + ch);
}

__device__ __forceinline__ void pin_agpr(uint4& v) {
    typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
    u32x4v t = {v.x, v.y, v.z, v.w};
    asm volatile("" : "+a"(t));
    v = make_uint4(t.x, t.y, t.z, t.w);
}

constexpr int ws_ps(int c16, int s) {
    return s == 1 ? c16 + (6 - c16 % 4) % 4 : (c16 % 2 ? c16 : c16 + 1);
}
constexpr int ws_hxp(int tx, int s) {
    const int hx = (tx - 1) * s + 3;
    if (tx % 16 == 0) return hx;
    int h = hx;
    while (h % 8 != tx % 8) ++h;
    return h;
}

}  // namespace

// CR: the conv's real input channels when CIN (the K of the tile, a multiple of 32) pads them
// (yolox_x's 80-channel stage: CIN 96) -- the halo DMA zero-fills chunks past CR, the weight
// fragments past CR are zero
// A32: fp32 destination, written or (YXH_CONV_ACCUMULATE) added to -- the data gradient of a
// stride-1 3x3 conv in the training step (yolox_amd/train.py _dgrad: dy with the transposed,
// flipped weights into the input's fp32 gradient), no bias / activation / residual
template <typename T, int CIN, int S, int TX, int TY, int TN, int WN, int WK, int WM, int BPC, bool F1, int PGN = 0,
          int PGC = 0, int PGH = 0, int CR = CIN, bool A32 = false>
__global__ __launch_bounds__(64 * WN * WK * WM, BPC) void conv_ws(ConvParams p, int tiles_x, int tiles_y,
                                                                 int ntiles, int ntn, int nwork) {
    static_assert(sizeof(T) == 2, "16-bit operands");
    constexpr int NW = WN * WK * WM;
    constexpr int NCB = CIN / 32, WCB = NCB / WK;
    constexpr int WTN = TN / WN, FR = WTN / 16;
    constexpr int TM = TX * TY, WTM = TM / WM, FC = WTM / 16;
    constexpr int HX = (TX - 1) * S + 3, HY = (TY - 1) * S + 3, HXP = ws_hxp(TX, S);
    constexpr int C16 = CIN / 8, PS = ws_ps(C16, S), PSB = PS * 16;
    constexpr int SLOTS = HY * HXP * PS, LOADS = (SLOTS + 63) / 64, GB = (LOADS + NW - 1) / NW;
    // partial sums: fragment j of wave group (wn, wm) is finished by wave wk = j % WK; the
    // WK - 1 others each leave their part in a slot of their own
    constexpr int RBYTES = WK > 1 ? WN * WM * FR * FC * (WK - 1) * 1024 : 0;
    // residual tile staging (stride-1 variants: the Bottleneck's shortcut): TM pixels x TN
    // channels by LDS-DMA with the halo, one 16-byte pad slot per pixel row, a ring of three
    // (the epilogue of tile k-1 runs during tile k while tile k+1 lands)
    // Post conv (PGN > 0, yxh_conv_desc.post_weight): the tile's output Y stays in LDS in the
    // residual slot layout (ring slot = tile % 3: the residual DMA'd in at the tile's own step,
    // Y written over it in place by the epilogue pieces riding the next tile's MFMAs) and
    // Z = SiLU(W2 . [Y | X2] + b2) of PGN channels leaves instead, computed in pieces riding
    // the MFMAs of the tile after that; X2 = PGC channels of post_src DMA'd per tile (ring of 3)
    // Head form (PGH > 0 class fragments; YXH_CONV_GROUPS2): the same Y ring, and instead of a
    // bf16 post conv each group's block runs its level's preds over Y (group 0: PGH x 16 class
    // rows, group 1: the 5 reg | obj rows; weights in LDS) into decoded fp32 [B, A, 5 + C] rows
    constexpr bool PG = PGN > 0, HP = PGH > 0, PGY = PG || HP;
    constexpr int RS = TN / 8 + 1, RSLOTS = (S == 1 || PGY) ? TM * RS : 0;
    constexpr int RLOADS = (RSLOTS + 63) / 64, GR = (RLOADS + NW - 1) / NW, RTB = RLOADS * 1024;
    constexpr int NRING = 3;
    constexpr int XS = PGC / 8 + 1, XSLOTS = PG && PGC > 0 ? TM * XS : 0;
    constexpr int XLOADS = (XSLOTS + 63) / 64, GX = (XLOADS + NW - 1) / NW, XTB = XLOADS * 1024;
    constexpr int K2 = TN + PGC, KB2 = K2 / 32;
    constexpr int WN2 = PG ? (NW < PGN / 16 ? NW : PGN / 16) : 1, WM2 = NW / WN2;
    constexpr int NF2 = PG ? PGN / 16 / WN2 : 1, PF2 = TM / 16 / WM2;
    static_assert(!PG || (!F1 && TN % 32 == 0 && PGC % 32 == 0 && PGN % (16 * WN2) == 0 &&
                          NW % WN2 == 0 && (TM / 16) % WM2 == 0), "post-conv tile");
    static_assert(!HP || (!PG && !F1 && S == 1 && TN % 32 == 0), "head-form tile");
    constexpr int HROWS = HP ? PGH * 16 : 0, HBYTES_W = HROWS * RS * 16 + HROWS * 4;
    // fused Bottleneck (F1): t = act(W1 . x + b1) of the halo tile, computed into one more
    // halo-shaped LDS image that the 3x3 then reads; wave w computes t channels
    // 32 (w % NG) .. +32 of every R-th 16-pixel halo fragment
    constexpr int NG = CIN / 32, R1 = NW / NG, NPA = (HY * HXP + 15) / 16;
    constexpr int HBYTES = LOADS * 1024;
    constexpr int XOFF = 2 * HBYTES + RBYTES + NRING * RTB;
    constexpr int TOFF = XOFF + 3 * XTB;
    constexpr int HWOFF = TOFF + (F1 ? HBYTES : 0);
    constexpr int SMEM = HWOFF + HBYTES_W;
    static_assert(!F1 || (S == 1 && NW % NG == 0), "fused Bottleneck tile");
    constexpr int FCO = (FC + WK - 1) / WK;  // pixel fragments this wave finishes
    constexpr int NS = WCB * 9;              // K steps per tile (channel block x tap)
    constexpr int PD = YXH_WS_PD8 && FR * FC >= 8 ? YXH_WS_PD8 : FR * FC >= 8 ? 1 : FR * FC >= 4 ? 2 : 3;  // fragment-read distance in K steps
    static_assert(NCB % WK == 0 && WTN % 16 == 0 && WTM % 16 == 0 && TM % (16 * WM) == 0, "tile");
    // weights must stay in VGPRs: 160 of 256 (2 waves per SIMD), 288 of 512 (one 4-wave block per CU)
    static_assert(FR * 9 * WCB * 4 <= (NW == 4 && BPC == 1 ? 288 : 160), "weights must stay in VGPRs");
    static_assert(SMEM <= 160 * 1024 && SMEM * BPC <= 160 * 1024, "LDS (BPC blocks per CU must fit)");
    // 288-register weight sets (one 4-wave block per CU): the first NPIN weight fragments are pinned
    // to AGPRs where the first tile first reads them, and the MFMAs take them from there (gfx950's
    // MFMA reads A operands from AGPRs).  Left to itself the register allocator parks ~30 % of the
    // weights in AGPRs anyway and copies each back to VGPRs before every use (4 v_accvgpr_read +
    // an s_nop per 4 MFMAs in the K loop of the head level-0 tile).  48 fragments = 192 AGPRs
    // leave room for the accumulators; 56 / 64 made the allocator shuffle again (probe builds).
    constexpr int NPIN = !F1 && FR * 9 * WCB * 4 > 160 ? YXH_WS_NPIN : 0;  // (fused-Bottleneck tiles: spills)
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

    const int cin_ = p.cin, cout = p.cout, in_w = p.in_w, in_h = p.in_h, scs = p.scs[0];
    const int OH = p.out_h, OW = p.out_w, ohw = p.ohw;
    (void)cin_;

    // ---- this lane's LDS byte offsets of its pixel fragments at tap (0, 0), channel block 0
    uint32_t boff[FC];
#pragma unroll
    for (int j = 0; j < FC; ++j) {
        const int pl = (wm * FC + j) * 16 + frow;
        const int ty = pl / TX, tx = pl - ty * TX;
        boff[j] = (uint32_t)((ty * S * HXP + tx * S) * PSB + (wk * WCB * 4 + fq) * 16);
    }

    const uint32_t lds0 = dma::lds_addr(smem);
    const uint32_t bytes = (uint32_t)((long long)in_h * in_w * scs * 2);
    const int gsrc = p.grp2 && n0 >= cout / 2 ? CR : 0;  // YXH_CONV_GROUPS2: this half's source channels

    // per-lane halo slot geometry, fixed for the block's life: the slot's pixel (hy, hx)
    // in the halo and its source byte offset relative to the halo's top-left pixel
    int hrel[GB], hyx[GB];
#pragma unroll
    for (int i = 0; i < GB; ++i) {
        const int L = wave + NW * i;
        const int s = 64 * L + lane;
        const int hp = s / PS, c16 = s - hp * PS;
        const int hy = hp / HXP, hx = hp - hy * HXP;
        const bool st = L < LOADS && s < SLOTS && c16 < CR / 8 && hx < HX;
        hyx[i] = st ? (hy | (hx << 16)) : 0x7fff7fff;  // 0x7fff fails every range check
        hrel[i] = ((hy * in_w + hx) * scs + c16 * 8) * 2;
    }

    struct TileC { int b, oy0, ox0; };
    const unsigned txy = (unsigned)(tiles_x * tiles_y);
    auto coords = [&](int t) -> TileC {
        const unsigned b = (unsigned)t / txy, r = (unsigned)t - b * txy;
        const unsigned ty = r / (unsigned)tiles_x, tx = r - ty * (unsigned)tiles_x;
        return TileC{(int)b, (int)ty * TY, (int)tx * TX};
    };

    auto issue_halo = [&](const TileC& c, int kb) {
        const int iy0 = c.oy0 * S - 1, ix0 = c.ox0 * S - 1;
        const int base = (iy0 * in_w + ix0) * scs * 2;
        const dma::u32x4 rsrc = dma::srd((const T*)p.sptr[0] + (long long)c.b * p.sbs[0] + gsrc, bytes);
#pragma unroll
        for (int i = 0; i < GB; ++i) {
            const int L = wave + NW * i;
            if (LOADS % NW == 0 || i + 1 < GB || L < LOADS) {
                const int iy = iy0 + (hyx[i] & 0xffff), ix = ix0 + (hyx[i] >> 16);
                const bool ok = (unsigned)iy < (unsigned)in_h && (unsigned)ix < (unsigned)in_w;
                const uint32_t voff = ok ? (uint32_t)(base + hrel[i]) : dma::kOob;
                dma::load16(rsrc, voff, 0u, __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(kb * HBYTES + L * 1024)));
            }
        }
    };

    const bool silu = p.act == YXH_ACT_SILU;
    const bool has_res = p.res != nullptr;
    const bool pg_store = PG && p.pg_store;
    const uint32_t dbytes = (uint32_t)((long long)ohw * p.dst_cs * (A32 ? 4 : 2));
    const uint32_t rbytes = (uint32_t)((long long)ohw * p.res_cs * 2);
    const int dcs = p.dst_cs, rcs = p.res_cs;
    const uint32_t res_lds = lds0 + (uint32_t)(2 * HBYTES + RBYTES);

    // residual staging: per-lane slot geometry (pixel ty/tx of the tile, 8-channel chunk)
    int rgeo[GR > 0 ? GR : 1];
#pragma unroll
    for (int i = 0; i < GR; ++i) {
        const int L = wave + NW * i;
        const int sl = 64 * L + lane;
        const int pl = sl / RS, ch = sl - pl * RS;
        const int ty = pl / TX, tx = pl - ty * TX;
        const bool st = L < RLOADS && sl < RSLOTS && ch < TN / 8 && n0 + ch * 8 < cout;
        rgeo[i] = st ? (ty | (tx << 10) | (ch << 20)) : -1;
    }
    auto issue_res = [&](const TileC& c, int slot) {
        if constexpr (GR > 0) {
            const dma::u32x4 rsrc = dma::srd((const T*)p.res + (long long)c.b * p.res_bs, rbytes);
#pragma unroll
            for (int i = 0; i < GR; ++i) {
                const int L = wave + NW * i;
                if (RLOADS % NW == 0 || i + 1 < GR || L < RLOADS) {
                    const int g = rgeo[i];
                    const int oy = c.oy0 + (g & 1023), ox = c.ox0 + ((g >> 10) & 1023);
                    const bool ok = g >= 0 && oy < OH && ox < OW;
                    const uint32_t voff = ok ? (uint32_t)(((oy * OW + ox) * rcs + n0 + (g >> 20) * 8) * 2) : dma::kOob;
                    dma::load16(rsrc, voff, 0u, __builtin_amdgcn_readfirstlane(res_lds + (uint32_t)(slot * RTB + L * 1024)));
                }
            }
        }
    };

    // post conv second operand: per-lane slot geometry as the residual's, PGC channels
    int xgeo[GX > 0 ? GX : 1];
#pragma unroll
    for (int i = 0; i < GX; ++i) {
        const int L = wave + NW * i;
        const int sl = 64 * L + lane;
        const int pl = sl / XS, ch = sl - pl * XS;
        const int ty = pl / TX, tx = pl - ty * TX;
        const bool st = L < XLOADS && sl < XSLOTS && ch < PGC / 8;
        xgeo[i] = st ? (ty | (tx << 10) | (ch << 20)) : -1;
    }
    auto issue_x2 = [&](const TileC& c, int slot) {
        if constexpr (GX > 0) {
            const dma::u32x4 xsrc =
                dma::srd((const T*)p.pgs + (long long)c.b * p.pgs_bs, (uint32_t)((long long)ohw * p.pgs_cs * 2));
#pragma unroll
            for (int i = 0; i < GX; ++i) {
                const int L = wave + NW * i;
                if (XLOADS % NW == 0 || i + 1 < GX || L < XLOADS) {
                    const int g = xgeo[i];
                    const int oy = c.oy0 + (g & 1023), ox = c.ox0 + ((g >> 10) & 1023);
                    const bool ok = g >= 0 && oy < OH && ox < OW;
                    const uint32_t voff = ok ? (uint32_t)(((oy * OW + ox) * p.pgs_cs + (g >> 20) * 8) * 2) : dma::kOob;
                    dma::load16(xsrc, voff, 0u,
                                __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(XOFF + slot * XTB + L * 1024)));
                }
            }
        }
    };

    // ---- prologue: this tile's halo (+ residual) and the next tile's go out first, then the
    // weights behind them (the first tile waits only for the halos: see tile_step's FIRST)
    TileC cur = coords(tile), cnext{0, 0, 0}, prev{0, 0, 0}, prev2{0, 0, 0};
    issue_halo(cur, 0);
    if (!PGY && has_res) issue_res(cur, 0);
    if (tile + nwork < ntiles) {
        cnext = coords(tile + nwork);
        issue_halo(cnext, 1);
        if (!PGY && has_res) issue_res(cnext, 1);
    }

    const bool hgrp1 = HP && n0 >= cout / 2;
    const int hrows = HP ? (hgrp1 ? p.pg_cout2 : p.pg_cout) : 0;

    uint4 a1[F1 ? 2 : 1][F1 ? NG : 1];
    float b1[2][4];
    if constexpr (F1) {
        const T* w1 = (const T*)p.pw1;
        const int g = wave % NG;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int cb = 0; cb < NG; ++cb)
                a1[i][cb] = *(const uint4*)(w1 + (g * 32 + i * 16 + frow) * CIN + cb * 32 + fq * 8);
#pragma unroll
            for (int r = 0; r < 4; ++r) b1[i][r] = p.pb1[g * 32 + i * 16 + fq * 4 + r];
        }
    }

    // ---- stationary weights: a[i][tap][c] = 16 channels x 32 K of fragment i, loaded in the
    // order the first tile's K steps consume them (the compiler's per-use vmcnt waits then let
    // that tile's MFMAs start while the rest of the weights are still arriving)
    uint4 a[FR][9][WCB];
#pragma unroll
    for (int c = 0; c < WCB; ++c)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int i = 0; i < FR; ++i)
                a[i][tap][c] = CR == CIN ? ws_weight<T>(p, n0 + wn * WTN + i * 16, tap, 9, CIN, wk * WCB + c, lane)
                                         : ws_weight_padk<T, CR>(p, n0 + wn * WTN + i * 16, tap, wk * WCB + c, lane);
    float bias[FR][4];
#pragma unroll
    for (int i = 0; i < FR; ++i) {
        const int n = n0 + wn * WTN + i * 16 + fq * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[i][r] = n + r < cout ? p.bias[n + r] : 0.0f;
    }


    // post conv weights, stationary: wave w owns Z channels (w % WN2) * NF2 * 16 .. + NF2 * 16 and
    // pixel fragments (w / WN2) * PF2 .. + PF2 of the tile
    const int wn2 = wave % WN2, wm2 = wave / WN2;
    uint4 a2[PG ? NF2 : 1][PG ? KB2 : 1];
    float b2[PG ? NF2 : 1][4];
    if constexpr (PG) {
        const T* w2 = (const T*)p.pgw;
#pragma unroll
        for (int f = 0; f < NF2; ++f) {
            const int n = (wn2 * NF2 + f) * 16;
#pragma unroll
            for (int kb = 0; kb < KB2; ++kb) a2[f][kb] = *(const uint4*)(w2 + (long long)(n + frow) * K2 + kb * 32 + fq * 8);
#pragma unroll
            for (int r = 0; r < 4; ++r) b2[f][r] = p.pgb[n + fq * 4 + r];
        }
    }

    // epilogue of a finished tile: bias, SiLU, residual (from the LDS staging slot), 8-byte
    // stores of 4 channels through a buffer descriptor (an invalid pixel / channel carries an
    // out-of-range offset: no branch, so the scheduler can spread it over the next tile's
    // MFMAs); dispatch checks the dtype / alignment / activation this form assumes
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    struct EpiCtx { __amdgpu_buffer_rsrc_t dsrd; const char* rl; TileC c; };
    auto epi_ctx = [&](const TileC c, const int k) -> EpiCtx {
        char* db = (char*)p.dst + (long long)c.b * p.dst_bs * (A32 ? 4 : 2);
        return EpiCtx{__builtin_amdgcn_make_buffer_rsrc((void*)db, (short)0, (int)dbytes, 0x00020000),
                      smem + 2 * HBYTES + RBYTES + (k % NRING) * RTB, c};
    };
    // one (pixel fragment o, channel fragment i) piece of the epilogue; act_c: 0 = the runtime
    // activation, 1 = SiLU, 2 = none (YXH_WS_ACT_CT: fixed for the whole tile loop)
    auto epi_piece = [&](const EpiCtx& e, const f32x4 (&ap)[FR][FCO], const int o, const int i, auto act_c) {
        constexpr int AC = decltype(act_c)::value;
        const int j = wk + WK * o;
        const int pl = (wm * FC + j) * 16 + frow;
        const int ty = pl / TX, tx = pl - ty * TX;
        const int oy = e.c.oy0 + ty, ox = e.c.ox0 + tx;
        const int nl = wn * WTN + i * 16 + fq * 4, n = n0 + nl;
        const bool ok = j < FC && oy < OH && ox < OW && n < cout;
        if constexpr (A32) {  // fp32 data gradient: 16-byte read-add-store of 4 channels
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const int od4 = ok ? ((oy * OW + ox) * dcs + n) * 4 : (int)dma::kOob;
            f32x4 v = ap[i][o] + f32x4{bias[i][0], bias[i][1], bias[i][2], bias[i][3]};
            if (p.accum) v += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(e.dsrd, od4, 0, 0));
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), e.dsrd, od4, 0, 0);
            return;
        }
        const int od = ok ? ((oy * OW + ox) * dcs + n) * 2 : (int)dma::kOob;
        u32x2 rv = {0u, 0u};
        if constexpr (GR > 0) rv = *(const u32x2*)(e.rl + (pl * RS + (nl >> 3)) * 16 + (nl & 7) * 2);
        T rt[4];
        __builtin_memcpy(rt, &rv, 8);
        const f32x4 x = ap[i][o] + f32x4{bias[i][0], bias[i][1], bias[i][2], bias[i][3]};
        f32x4 v;
        if constexpr (AC == 1) v = yxh::silu4(x);
        else if constexpr (AC == 2) v = x;
        else v = silu ? yxh::silu4(x) : x;
        if (has_res) v = v + f32x4{to_f32(rt[0]), to_f32(rt[1]), to_f32(rt[2]), to_f32(rt[3])};
        T t[4] = {from_f32<T>(v[0]), from_f32<T>(v[1]), from_f32<T>(v[2]), from_f32<T>(v[3])};
        u32x2 u;
        __builtin_memcpy(&u, t, 8);
        if constexpr (PGY) {
            // Y stays in LDS, over this lane's own residual values (and, YXH_CONV_POST_STORE,
            // leaves for dst too: the next Bottleneck's input)
            *(u32x2*)(e.rl + (pl * RS + (nl >> 3)) * 16 + (nl & 7) * 2) = u;
            if (PG && pg_store) __builtin_amdgcn_raw_buffer_store_b64(u, e.dsrd, od, 0, 0);
        } else if (!(YXH_WS_PROBE & 1) || p.act == 12345) {
            __builtin_amdgcn_raw_buffer_store_b64(u, e.dsrd, od, 0, 0);
        }
    };
    auto epilogue = [&](const TileC c, const int k, const f32x4 (&ap)[FR][FCO], auto act_c) {
        const EpiCtx e = epi_ctx(c, k);
#pragma unroll
        for (int o = 0; o < FCO; ++o)
#pragma unroll
            for (int i = 0; i < FR; ++i) epi_piece(e, ap, o, i, act_c);
    };

    // Post work of a finished tile whose Y is complete in ring slot k % 3 (and X2 landed), as
    // independent pieces -- one 16-pixel fragment x one 16-row output fragment each -- that ride
    // the MFMA loop two tiles later (or run at the end):
    //  * PG: Z = SiLU(W2 . [Y | X2] + b2) (W2 stationary in VGPRs), 8-byte bf16 stores;
    //  * HP: the level's preds over Y (weights in LDS) decoded as head.hip's head_pred (same
    //    MFMA order, hardware exp2 / rcp), dword stores of the fp32 rows
    struct PostCtx { __amdgpu_buffer_rsrc_t srd; const char* ys; const char* xs; TileC c; };
    auto post_ctx = [&](const TileC c, const int k) -> PostCtx {
        PostCtx q;
        q.c = c;
        q.ys = smem + 2 * HBYTES + RBYTES + (k % NRING) * RTB;
        q.xs = smem + XOFF + (k % 3) * XTB;
        const int es = HP ? 4 : 2;
        q.srd = __builtin_amdgcn_make_buffer_rsrc((void*)((char*)p.pgd + (long long)c.b * p.pgd_bs * es), (short)0,
                                                  (int)((long long)ohw * p.pgd_cs * es), 0x00020000);
        return q;
    };
    constexpr int HPF = (TM / 16 + NW - 1) / NW;  // HP: pixel fragments per wave
    constexpr int NPU = PG ? PF2 * NF2 : HP ? HPF * PGH : 0;  // post pieces per wave per tile
    // a piece is split in two: its LDS operand reads (post_load) go out one K step before its
    // MFMAs / decode / stores (post_math), and the pieces are spread SP steps apart over the
    // tile's K loop, so no MFMA waits on a fresh LDS read and the reads do not bunch up
    constexpr int KBP = PG ? KB2 : HP ? 2 * (TN / 32) : 1;  // operand registers of one piece
    // (the head form keeps its pieces in the first steps, reads and MFMAs in one step: spread
    // out or split, the 288-register weight set spills)
    constexpr bool SPLIT = PG;
    constexpr int SP = SPLIT && NS / (NPU + 1) > 1 ? NS / (NPU + 1) : 1;
    auto post_skip = [&](const int u) -> bool {  // wave-uniform: a head piece with no rows
        if constexpr (HP) {
            const int pf = wave + NW * (u / PGH), f = u - PGH * (u / PGH);
            return pf >= TM / 16 || f >= (hgrp1 ? 1 : PGH);
        }
        return false;
    };
    auto post_load = [&](const PostCtx& q, const int u, uint4 (&ob)[KBP]) {
        if constexpr (PG) {
            const int pf = u / NF2;
            const int pl = (wm2 * PF2 + pf) * 16 + frow;
#pragma unroll
            for (int kb = 0; kb < KB2; ++kb)
                ob[kb] = kb < TN / 32 ? *(const uint4*)(q.ys + (pl * RS + kb * 4 + fq) * 16)
                                      : *(const uint4*)(q.xs + (pl * XS + (kb - TN / 32) * 4 + fq) * 16);
        } else if constexpr (HP) {
            if (post_skip(u)) return;
            const int pf = wave + NW * (u / PGH), f = u - PGH * (u / PGH);
            const char* wl = smem + HWOFF;
#pragma unroll
            for (int kb = 0; kb < TN / 32; ++kb) {
                ob[2 * kb] = *(const uint4*)(q.ys + ((pf * 16 + frow) * RS + kb * 4 + fq) * 16);
                ob[2 * kb + 1] = *(const uint4*)(wl + ((f * 16 + frow) * RS + kb * 4 + fq) * 16);
            }
        }
    };
    auto post_math = [&](const PostCtx& q, const int u, const uint4 (&ob)[KBP]) {
        if constexpr (PG) {
            const int pf = u / NF2, f = u - NF2 * (u / NF2);
            const int pl = (wm2 * PF2 + pf) * 16 + frow;
            f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kb = 0; kb < KB2; ++kb) Mma<T>::run(z, a2[f][kb], ob[kb]);
            const int ty = pl / TX, tx = pl - ty * TX;
            const int oy = q.c.oy0 + ty, ox = q.c.ox0 + tx;
            const int n = (wn2 * NF2 + f) * 16 + fq * 4;
            const f32x4 zs = yxh::silu4(z + f32x4{b2[f][0], b2[f][1], b2[f][2], b2[f][3]});
            T t[4] = {from_f32<T>(zs[0]), from_f32<T>(zs[1]), from_f32<T>(zs[2]), from_f32<T>(zs[3])};
            u32x2 uv;
            __builtin_memcpy(&uv, t, 8);
            const int od = oy < OH && ox < OW ? ((oy * OW + ox) * p.pgd_cs + n) * 2 : (int)dma::kOob;
            __builtin_amdgcn_raw_buffer_store_b64(uv, q.srd, od, 0, 0);
        } else if constexpr (HP) {
            if (post_skip(u)) return;
            const int pf = wave + NW * (u / PGH), f = u - PGH * (u / PGH);
            const float* bl = (const float*)(smem + HWOFF + HROWS * RS * 16);
            // z[pixel][channel] (Y the A operand): lane l holds pixel 4 (l >> 4) + r of the
            // fragment and channel l & 15, so each dword store writes 16 consecutive channels of
            // 4 rows (4 x 64 B) instead of 4 channels of 16 rows
            f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kb = 0; kb < TN / 32; ++kb) Mma<T>::run(z, ob[2 * kb], ob[2 * kb + 1]);
            const float st = p.pg_stride;
            const int ch = f * 16 + frow;
            const float bch = bl[ch];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int pl = pf * 16 + fq * 4 + r;
                const int ty = pl / TX, tx = pl - ty * TX;
                const int oy = q.c.oy0 + ty, ox = q.c.ox0 + tx;
                const bool okp = oy < OH && ox < OW;
                const int rowo = (oy * OW + ox) * p.pgd_cs + (hgrp1 ? 0 : 5);
                float v = z[r] + bch;
                if (hgrp1) {
                    if (ch < 2) v = (v + (float)(ch == 0 ? ox : oy)) * st;
                    else if (ch < 4) v = __builtin_amdgcn_exp2f(v * 1.4426950408889634f) * st;
                    else v = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-v * 1.4426950408889634f));
                } else {
                    v = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-v * 1.4426950408889634f));
                }
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), q.srd,
                                                      okp && ch < hrows ? (rowo + ch) * 4 : (int)dma::kOob, 0, 0);
            }
        }
    };
    auto post_piece = [&](const PostCtx& q, const int u) {
        uint4 ob[KBP];
        post_load(q, u, ob);
        post_math(q, u, ob);
    };
    auto post_all = [&](const PostCtx& q) {
#pragma unroll
        for (int u = 0; u < NPU; ++u) post_piece(q, u);
    };

    f32x4 accp[FR][FCO];  // owned fragments of the previous tile, waiting for their epilogue
    constexpr int NP = FR * FCO;  // epilogue pieces, one per K step while they last

    // one tile: wait for its halo, start tile k+1's halo (+ residual), MMA of tile k with the
    // epilogue of tile k-1 spread over it, then the K-split reduce of tile k into accp
    auto tile_step = [&](const TileC cur, const int tile, const int k, TileC& cnext, const TileC prev,
                         const TileC prev2, auto epi, auto post, auto first, auto act_c) -> int {
        constexpr bool EPI = decltype(epi)::value;
        constexpr bool POST = decltype(post)::value && PGY;
        constexpr bool FIRST = decltype(first)::value;
        const int kb = k & 1;
        const int next = tile + nwork;
        // FIRST: the halos (and residuals) went out before the weight loads, and vmcnt retires
        // in issue order, so once no more than the weight loads are pending they have landed
        if constexpr (FIRST) dma::wait_vm<(FR * 9 * WCB < 63 ? FR * 9 * WCB : 63)>();
        else dma::wait_vm<0>();
        dma::barrier();
        if (next < ntiles) {
            cnext = coords(next);
            if (!FIRST && !(YXH_WS_PROBE & 2)) {
                issue_halo(cnext, kb ^ 1);
                if (!PGY && has_res) issue_res(cnext, (k + 1) % 3);
            }
        }
        if constexpr (PGY) {  // this tile's residual / X2 (ring slot k % 3: its post runs two steps on)
            if (has_res) issue_res(cur, k % 3);
            issue_x2(cur, k % 3);
        }

        if constexpr (F1) {
            // Bottleneck conv1 over the halo: t = act(W1 . x + b1), zero outside the image
            // (it is the 3x3's zero padding), into the t image
            const char* hx_img = smem + kb * HBYTES;
            char* timg = smem + TOFF;
            const int g = wave % NG;
            for (int fa = wave / NG; fa < NPA; fa += R1) {
                const int hq = fa * 16 + frow;
                const int hpr = min(hq, HY * HXP - 1);
                f32x4 t2[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
                for (int cb = 0; cb < NG; ++cb) {
                    const uint4 xb = *(const uint4*)(hx_img + hpr * PSB + (cb * 4 + fq) * 16);
                    Mma<T>::run(t2[0], a1[0][cb], xb);
                    Mma<T>::run(t2[1], a1[1][cb], xb);
                }
                const int hy = hq / HXP, hx = hq - hy * HXP;
                const int iy = cur.oy0 - 1 + hy, ix = cur.ox0 - 1 + hx;
                const bool valid = hx < HX && (unsigned)iy < (unsigned)in_h && (unsigned)ix < (unsigned)in_w;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    T t[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float x = t2[i][q] + b1[i][q];
                        t[q] = from_f32<T>(valid ? (silu ? yxh::silu<false>(x) : x) : 0.0f);
                    }
                    u32x2 u;
                    __builtin_memcpy(&u, t, 8);
                    if (hq < HY * HXP) *(u32x2*)(timg + hq * PSB + (g * 32 + i * 16 + fq * 4) * 2) = u;
                }
            }
            dma::barrier();
        }

        f32x4 acc[FR][FC];
#pragma unroll
        for (int i = 0; i < FR; ++i)
#pragma unroll
            for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        const char* hb = F1 ? smem + TOFF : smem + kb * HBYTES;
        // K steps s = (channel block c, tap); the pixel fragments of step s + PD are read
        // before the MFMAs of step s, so the LDS latency hides behind PD steps of MFMAs (about
        // 8 MFMAs: one 4-MFMA step does not cover an LDS read under load; measured, PD 1 -> 2:
        // 80x80 128->128 76 -> 70 us, 40->20 s2 256->512 64 -> 57 us)
        uint4 bf[PD + 1][FC];
        auto load_b = [&](int s, uint4 (&d)[FC]) {
            const int c = s / 9, tap = s - 9 * (s / 9);
            const int ky = tap / 3, kx = tap - 3 * (tap / 3);
            const int so = (ky * HXP + kx) * PSB + c * 64;
#pragma unroll
            for (int j = 0; j < FC; ++j) d[j] = *(const uint4*)(hb + boff[j] + so);
        };
#pragma unroll
        for (int q = 0; q < PD; ++q)
            if (q < NS) load_b(q, bf[q]);
        __builtin_amdgcn_sched_group_barrier(0x100, FC * (PD < NS ? PD : NS), 0);
        EpiCtx e{};
        if constexpr (EPI) e = epi_ctx(prev, k - 1);
        PostCtx pc{};
        if constexpr (POST) pc = post_ctx(prev2, k - 2);
        uint4 pob[KBP];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (s + PD < NS) load_b(s + PD, bf[(s + PD) % (PD + 1)]);
            const int c = s / 9, tap = s - 9 * (s / 9);
            if constexpr (FIRST && NPIN > 0) {  // where each pinned fragment is first used
#pragma unroll
                for (int i = 0; i < FR; ++i)
                    if ((c * 9 + tap) * FR + i < NPIN) pin_agpr(a[i][tap][c]);
            }
            // pixel-fragment-major: fragment j's FR uses come together, so its register is free (and
            // the next step's read into it can issue) FR * (FC - 1) MFMAs before that read's first use
            // (channel-major freed every fragment only in the step's last FC MFMAs: ~3 MFMAs of cover
            // for an LDS read at one wave per SIMD); each accumulator's K order is unchanged.  The
            // head-form tiles keep channel-major (fragment-major spilled their 288-register set)
            if constexpr (HP) {
#pragma unroll
                for (int i = 0; i < FR; ++i)
#pragma unroll
                    for (int j = 0; j < FC; ++j) Mma<T>::run(acc[i][j], a[i][tap][c], bf[s % (PD + 1)][j]);
            } else {
#pragma unroll
                for (int j = 0; j < FC; ++j)
#pragma unroll
                    for (int i = 0; i < FR; ++i) Mma<T>::run(acc[i][j], a[i][tap][c], bf[s % (PD + 1)][j]);
            }
            // piece s of the previous tile's epilogue rides on this step's MFMAs
            if constexpr (EPI)
                if (s < NP) epi_piece(e, accp, s / FR, s % FR, act_c);
            // ... and piece s of the post work of the tile before that
            // ... and the post work of the tile before that: piece u's operands are read in step
            // u * SP, its MFMAs and stores run in the next step
            if constexpr (POST && SPLIT) {
                if (s >= 1 && (s - 1) % SP == 0 && (s - 1) / SP < NPU) post_math(pc, (s - 1) / SP, pob);
                if (s % SP == 0 && s / SP < NPU) post_load(pc, s / SP, pob);
            } else if constexpr (POST) {
                if (s % SP == 0 && s / SP < NPU) post_piece(pc, s / SP);
            }
            // keep the one-step-ahead read distance (the scheduler would otherwise pull each
            // read down next to its first MFMA) and put two VALU ops in each MFMA's shadow
            if (s + PD < NS) __builtin_amdgcn_sched_group_barrier(0x100, FC, 0);  // DS reads
#pragma unroll
            for (int m = 0; m < FR * FC; ++m) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                if constexpr (EPI) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
            }
        }
        if constexpr (EPI)
#pragma unroll
            for (int q = NS; q < NP; ++q) epi_piece(e, accp, q / FR, q % FR, act_c);
        if constexpr (POST) {
            if (SPLIT && (NS - 1) % SP == 0 && (NS - 1) / SP < NPU) post_math(pc, (NS - 1) / SP, pob);
#pragma unroll
            for (int u = (NS + SP - 1) / SP; u < NPU; ++u) post_piece(pc, u);
        }

        // ---- K-split: partial sums of the fragments other waves finish go through LDS
        if constexpr (WK > 1) {
            char* red = smem + 2 * HBYTES;
            const int grp = wm * WN + wn;  // waves sharing (wn, wm)
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

    // the first tile is peeled off the loop: it consumes the weight loads, so the loop body
    // carries no compiler-visible pending load whose wait would also drain the halo DMA
    using act_rt = std::integral_constant<int, 0>;
    int next = tile_step(cur, tile, 0, cnext, cur, cur, std::false_type{}, std::false_type{}, std::true_type{}, act_rt{});
    // head form: this block's group's pred weights [rows][TN] (rows of RS 16-byte slots) and
    // biases -> LDS once, after the first tile (read from tile 2 on, behind tile 1's barriers);
    // rows past the group's count are zero
    if constexpr (HP) {
        const T* hw = (const T*)(hgrp1 ? p.pgw2 : p.pgw);
        const float* hb = hgrp1 ? p.pgb2 : p.pgb;
        char* wl = smem + HWOFF;
        for (int q = tid; q < HROWS * (TN / 8); q += 64 * NW) {
            const int r = q / (TN / 8), c = q - (TN / 8) * (q / (TN / 8));
            *(uint4*)(wl + (r * RS + c) * 16) = r < hrows ? *(const uint4*)(hw + (long long)r * TN + c * 8)
                                                          : make_uint4(0, 0, 0, 0);
        }
        for (int q = tid; q < HROWS; q += 64 * NW) ((float*)(wl + HROWS * RS * 16))[q] = q < hrows ? hb[q] : 0.0f;
    }

    // YXH_WS_ACT_CT: the tile loop once per activation in the one-wave-per-SIMD plain tiles (the
    // post / head forms and the 256-register tiles keep the runtime test below: a second copy of
    // their loop spills)
    constexpr bool ACT_CT = YXH_WS_ACT_CT && !A32 && !PGY && !F1 && NW == 4 && BPC == 1;
    if constexpr (ACT_CT) {
        auto tile_loop = [&](auto act_c) {
            int k = 1;
            for (; next < ntiles; ++k) {
                prev2 = prev;
                prev = cur;
                cur = cnext;
                next = tile_step(cur, next, k, cnext, prev, prev2, std::true_type{}, std::false_type{}, std::false_type{},
                                 act_c);
            }
            epilogue(cur, k - 1, accp, act_c);
        };
        if (silu) tile_loop(std::integral_constant<int, 1>{});
        else tile_loop(std::integral_constant<int, 2>{});
    } else {
        int k = 1;
        for (; next < ntiles; ++k) {
            prev2 = prev;
            prev = cur;
            cur = cnext;
            if (PGY && k >= 2)  // the post pieces of tile k - 2 ride this tile's MFMAs
                next = tile_step(cur, next, k, cnext, prev, prev2, std::true_type{}, std::integral_constant<bool, PGY>{},
                                 std::false_type{}, act_rt{});
            else
                next = tile_step(cur, next, k, cnext, prev, prev2, std::true_type{}, std::false_type{}, std::false_type{},
                                 act_rt{});
        }
        if constexpr (PGY) {  // the last tile's residual / X2 landed, the tile before it has its Y
            dma::wait_vm<0>();
            dma::barrier();
            if (k >= 2) post_all(post_ctx(prev, k - 2));
        }
        epilogue(cur, k - 1, accp, act_rt{});
        if constexpr (PGY) {
            dma::barrier();
            post_all(post_ctx(cur, k - 1));
        }
    }
    (void)ohw;
}

template <typename T, int CIN, int S, int TX, int TY, int TN, int WN, int WK, int WM, int BPC = 1, bool F1 = false,
          int PGN = 0, int PGC = 0, int PGH = 0, int CR = CIN, bool A32 = false>
static int launch_ws(const ConvParams& p, hipStream_t st) {
    if (p.stride != S || p.cin != CR) {
        set_error("conv_ws variant built for stride %d, %d input channels", S, CR);
        return YXH_EUNSUPPORTED;
    }
    if (CR != CIN && (p.grp2 || PGN > 0 || PGH > 0 || F1 || p.scs[0] % 8 || (uintptr_t)p.sptr[0] % 16)) {
        set_error("conv_ws padded-K variant (%d -> %d channels): plain conv over 16-byte pixel rows only", CR, CIN);
        return YXH_EUNSUPPORTED;
    }
    if (PGH > 0) {
        if (!p.grp2 || !p.pgw2 || p.cout != 2 * TN || (p.pg_cout + 15) / 16 != PGH) {
            set_error("conv_ws head-form tile: two groups of %d channels, %d class fragments", TN, PGH);
            return YXH_EUNSUPPORTED;
        }
    } else if ((p.pgw != nullptr) != (PGN > 0) || p.pgw2 || (p.pg_store && PGN == 0) ||
               (PGN > 0 && (p.pg_cout != PGN || p.pgs_ch != PGC || p.cout != TN))) {
        set_error(PGN > 0 ? "conv_ws post tile built for %d -> %d channels + a %d-channel post_src, post conv %d"
                          : "conv_ws plain tile with a post conv (%d -> %d, %d, %d)",
                  CIN, TN, PGC, PGN);
        return YXH_EUNSUPPORTED;
    }
    if (p.grp2 && (F1 || PGN > 0 || (p.cout / 2) % TN)) {
        set_error("conv_ws variant (%d input channels) cannot split its channel tiles over two groups", CIN);
        return YXH_EUNSUPPORTED;
    }
    if ((p.pw1 != nullptr) != F1) {
        set_error(F1 ? "conv_ws fused-Bottleneck variant (%d input channels) needs pre_weight"
                     : "conv_ws plain variant (%d input channels) with a pre_weight",
                  CIN);
        return YXH_EUNSUPPORTED;
    }
    if (A32) {
        if (!p.dst_f32 || p.act != YXH_ACT_NONE || p.res || p.grp2 || p.cout % 4 || ((uintptr_t)p.dst % 16) ||
            p.dst_cs % 4 || p.dst_bs % 4 || (long long)p.ohw * p.dst_cs * 4 >= (1LL << 31)) {
            set_error("conv_ws fp32-gradient tile: fp32 dst of 16-byte rows, no activation / residual");
            return YXH_EUNSUPPORTED;
        }
    } else if (p.dst_f32 || p.accum || (p.act != YXH_ACT_SILU && p.act != YXH_ACT_NONE) ||
        (!p.vec_store && PGN == 0 && PGH == 0) ||
        p.cout % 8 || (p.res && (S != 1 || ((uintptr_t)p.res % 16) || p.res_cs % 8 || p.res_bs % 8))) {
        set_error("conv_ws: 16-bit dst, SiLU/no activation, 8-byte aligned dst rows, 16-byte residual rows "
                  "(stride-1 variants) only");
        return YXH_EUNSUPPORTED;
    }
    const int tiles_x = (p.out_w + TX - 1) / TX, tiles_y = (p.out_h + TY - 1) / TY;
    const long long ntiles = (long long)tiles_x * tiles_y * (p.M / p.ohw);
    const int ntn = (p.cout + TN - 1) / TN;
    if (ntiles >= (1LL << 30)) {
        set_error("conv_ws: too many tiles");
        return YXH_EINVAL;
    }
    const int nwork = (int)std::min<long long>(ntiles, std::max(1, p.cus * BPC / ntn));
    hipLaunchKernelGGL((conv_ws<T, CIN, S, TX, TY, TN, WN, WK, WM, BPC, F1, PGN, PGC, PGH, CR, A32>), dim3((unsigned)(nwork * ntn)),
                       dim3(64 * WN * WK * WM), 0, st, p, tiles_x, tiles_y, (int)ntiles, ntn, nwork);
    YXH_CHECK_LAUNCH("conv_ws launch");
    return YXH_OK;
}

template <typename T>
static int ws_dispatch_t(int id, const ConvParams& p, hipStream_t st) {
    // id -> (CIN, stride, TX, TY, TN, WN, WK, WM[, blocks per CU])
    switch (id) {
        // 32 input channels: dark2 bottleneck 3x3 (160x160), dark2 downsample (s2 -> 64)
        case 1: return launch_ws<T, 32, 1, 16, 8, 32, 1, 1, 4>(p, st);
        case 2: return launch_ws<T, 32, 1, 16, 16, 32, 1, 1, 8>(p, st);
        case 3: return launch_ws<T, 32, 2, 16, 8, 64, 2, 1, 4>(p, st);
        case 4: return launch_ws<T, 32, 2, 16, 4, 64, 2, 1, 2, 2>(p, st);
        // 64 input channels: dark3 bottleneck 3x3 (80x80), dark3 downsample (s2 -> 128)
        case 5: return launch_ws<T, 64, 1, 16, 8, 64, 2, 1, 4>(p, st);
        case 6: return launch_ws<T, 64, 1, 16, 4, 64, 2, 1, 2, 2>(p, st);
        case 7: return launch_ws<T, 64, 2, 16, 4, 128, 4, 1, 2>(p, st);
        case 8: return launch_ws<T, 64, 2, 16, 2, 128, 4, 1, 1, 2>(p, st);
        // 128 input channels: 40x40 / 80x80 / 20x20 3x3s (dark4, PAFPN, head), s2 128 -> 128/256
        // ids 9 / 10 (128 -> 128 16x4 K-split two ways: 96 B/lane of scratch; 32 -> 32 32x8 two
        // blocks per CU: missed its occupancy target) are withdrawn
        case 11: return launch_ws<T, 128, 1, 8, 4, 128, 4, 2, 1>(p, st);
        case 12: return launch_ws<T, 128, 1, 8, 8, 64, 2, 2, 1>(p, st);
        case 13: return launch_ws<T, 128, 2, 16, 2, 128, 4, 2, 1>(p, st);
        case 14: return launch_ws<T, 128, 2, 8, 4, 128, 4, 2, 1>(p, st);
        case 15: return launch_ws<T, 128, 1, 16, 4, 64, 2, 2, 1>(p, st);
        // 256 input channels: dark5 / PAFPN / yolox_l head 3x3s (K split four ways)
        case 16: return launch_ws<T, 256, 1, 8, 4, 64, 2, 4, 1>(p, st);
        case 17: return launch_ws<T, 256, 1, 16, 2, 64, 2, 4, 1>(p, st);
        // 4-wave blocks held to 256 registers, two resident per CU: one block's
        // barriers / epilogue overlap the other's MFMAs
        case 18: return launch_ws<T, 32, 1, 16, 8, 32, 1, 1, 4, 2>(p, st);
        case 19: return launch_ws<T, 64, 1, 32, 2, 64, 2, 1, 2, 2>(p, st);
        case 20: return launch_ws<T, 128, 1, 16, 2, 64, 2, 2, 1, 2>(p, st);
        case 21: return launch_ws<T, 128, 1, 8, 4, 64, 2, 2, 1, 2>(p, st);
        case 22: return launch_ws<T, 128, 2, 16, 1, 64, 2, 2, 1, 2>(p, st);
        case 23: return launch_ws<T, 256, 1, 8, 2, 32, 1, 4, 1, 2>(p, st);
        case 24: return launch_ws<T, 64, 2, 16, 2, 64, 2, 1, 2, 2>(p, st);
        // one 4-wave block per CU with 512 registers: 128 channels x all of K per block, no
        // K split (no reduce barrier)
        case 25: return launch_ws<T, 128, 1, 16, 4, 128, 4, 1, 1>(p, st);
        case 26: return launch_ws<T, 128, 1, 16, 2, 128, 4, 1, 1>(p, st);
        case 27: return launch_ws<T, 128, 1, 8, 4, 128, 4, 1, 1>(p, st);
        // stride 2 from 256 channels (dark5 downsample 256 -> 512, PAFPN bu_conv1 256 -> 256)
        case 28: return launch_ws<T, 256, 2, 8, 2, 32, 1, 4, 1>(p, st);
        case 29: return launch_ws<T, 256, 2, 8, 2, 64, 2, 4, 1>(p, st);
        case 30: return launch_ws<T, 256, 2, 16, 1, 32, 1, 4, 1>(p, st);
        // fused Bottleneck (conv1 1x1 + conv2 3x3 + shortcut): ids 191-196
        case 31: return launch_ws<T, 32, 1, 16, 8, 32, 1, 1, 4, 1, true>(p, st);
        case 32: return launch_ws<T, 32, 1, 16, 16, 32, 1, 1, 8, 1, true>(p, st);
        case 33: return launch_ws<T, 64, 1, 16, 4, 64, 2, 1, 2, 1, true>(p, st);
        case 34: return launch_ws<T, 64, 1, 16, 8, 64, 2, 1, 2, 1, true>(p, st);
        case 35: return launch_ws<T, 128, 1, 16, 4, 128, 4, 1, 1, 1, true>(p, st);
        case 36: return launch_ws<T, 128, 1, 8, 4, 128, 4, 1, 1, 1, true>(p, st);
        // 1x1 post conv (ids 41-48 = tiles 221-228): dark2's Bottleneck 3x3 32 -> 32 + CspLayer.conv3
        // over [y | x_2] (64 -> 64); the 64 -> 64 3x3s of dark3's last Bottleneck / C3_p3 + conv3 over
        // [y | x_2] (128 -> 128); dark3[0] (3x3 s2 64 -> 128) + CspLayer conv1 | conv2 (128 -> 128)
        case 41: return launch_ws<T, 32, 1, 16, 8, 32, 1, 1, 4, 1, false, 64, 32>(p, st);
        case 42: return launch_ws<T, 32, 1, 16, 4, 32, 1, 1, 4, 2, false, 64, 32>(p, st);
        case 43: return launch_ws<T, 64, 1, 16, 4, 64, 2, 1, 2, 1, false, 128, 64>(p, st);
        case 44: return launch_ws<T, 64, 1, 8, 4, 64, 2, 2, 1, 2, false, 128, 64>(p, st);
        case 45: return launch_ws<T, 64, 2, 16, 2, 128, 4, 1, 1, 1, false, 128, 0>(p, st);
        case 46: return launch_ws<T, 64, 2, 16, 4, 128, 4, 1, 1, 1, false, 128, 0>(p, st);
        // K split over two waves: half the stationary weights per wave, so two blocks per CU
        // (64 -> 64) or eight waves per block (s2 64 -> 128) fit the post conv's weights too
        case 47: return launch_ws<T, 64, 1, 16, 2, 64, 2, 2, 1, 2, false, 128, 64>(p, st);
        case 48: return launch_ws<T, 64, 1, 16, 4, 64, 2, 2, 1, 1, false, 128, 64>(p, st);
        case 49: return launch_ws<T, 64, 2, 16, 2, 128, 4, 2, 1, 1, false, 128, 0>(p, st);
        case 50: return launch_ws<T, 64, 2, 8, 4, 128, 4, 2, 1, 1, false, 128, 0>(p, st);
        // head form (ids 51-53 = tiles 231-233): a level's cls_convs[k][1] | reg_convs[k][1] with
        // each group's preds + decode (yolo_head.py:149-251) in the same launch
        case 51: return launch_ws<T, 128, 1, 16, 4, 128, 4, 1, 1, 1, false, 0, 0, 5>(p, st);
        // (id 52, the eight-wave K-split head form, spilled once its post pieces rode the MFMA loop)
        case 53: return launch_ws<T, 128, 1, 16, 2, 128, 4, 1, 1, 1, false, 0, 0, 5>(p, st);
        // Bottleneck chain (YXH_CONV_POST_STORE): the 3x3 + shortcut output stored AND the next
        // Bottleneck's conv1 (1x1 C -> C) over it: dark3 (64 @80x80), dark4 (128 @40x40)
        // (one block of 4 waves per CU: the 2-block / 8-wave forms spill)
        case 52: return launch_ws<T, 64, 1, 16, 8, 64, 2, 1, 2, 1, false, 64, 0>(p, st);
        case 54: return launch_ws<T, 64, 1, 16, 4, 64, 2, 1, 2, 1, false, 64, 0>(p, st);
        case 55: return launch_ws<T, 128, 1, 8, 4, 128, 4, 1, 1, 1, false, 128, 0>(p, st);
        case 56: return launch_ws<T, 128, 1, 16, 2, 128, 4, 1, 1, 1, false, 128, 0>(p, st);
        // wide / odd input channels (ids 61-80 = tiles 261-280): yolox_x (80 / 160 / 320, widths x1.25)
        // and yolox_l (512) 3x3s.  Register budget per wave: <= 160 weight registers at two waves per SIMD,
        // <= 288 at one; LDS: two halo buffers of CIN / 8 + 2 16-byte slots per pixel (the big-CIN tiles
        // are one or two pixel rows high).  80 input channels run as K = 96 (zero chunks).  Withdrawn:
        // ids 70, 73, 75, 77, 78 (10- / 16-wave blocks: 168 / 128 registers per wave, they spilled) --
        // 640 input channels have no form that fits (K = 20 blocks: 180 weight registers at WK 4)
        case 61: return launch_ws<T, 96, 1, 16, 4, 80, 5, 1, 1, 1, false, 0, 0, 0, 80>(p, st);
        case 62: return launch_ws<T, 96, 1, 16, 4, 32, 2, 1, 2, 2, false, 0, 0, 0, 80>(p, st);
        case 63: return launch_ws<T, 96, 2, 16, 4, 80, 5, 1, 1, 1, false, 0, 0, 0, 80>(p, st);
        case 64: return launch_ws<T, 96, 2, 16, 4, 32, 2, 1, 2, 1, false, 0, 0, 0, 80>(p, st);
        case 65: return launch_ws<T, 160, 1, 16, 4, 64, 4, 1, 1>(p, st);
        case 66: return launch_ws<T, 160, 1, 16, 4, 32, 2, 1, 2>(p, st);
        case 67: return launch_ws<T, 160, 2, 16, 2, 64, 4, 1, 1>(p, st);
        case 68: return launch_ws<T, 160, 2, 16, 2, 32, 2, 1, 2>(p, st);
        case 69: return launch_ws<T, 320, 1, 8, 4, 32, 2, 2, 1>(p, st);
        case 71: return launch_ws<T, 320, 1, 16, 2, 32, 2, 2, 1>(p, st);
        case 72: return launch_ws<T, 320, 2, 16, 1, 32, 2, 2, 1>(p, st);
        case 74: return launch_ws<T, 512, 1, 8, 2, 32, 2, 4, 1>(p, st);
        case 76: return launch_ws<T, 512, 1, 16, 1, 32, 2, 4, 1>(p, st);
        case 79: return launch_ws<T, 160, 1, 16, 2, 64, 4, 1, 1>(p, st);
        case 80: return launch_ws<T, 96, 1, 8, 4, 32, 2, 1, 2, 2, false, 0, 0, 0, 80>(p, st);
        // fp32-gradient forms (ids 81-88 = tiles 281-288): the stride-1 3x3 data gradients of the training
        // step (yolox_x's 80 / 160 / 320-channel maps; yolox_s / yolox_l's 64 / 128 / 256)
        case 81: return launch_ws<T, 96, 1, 16, 4, 32, 2, 1, 2, 2, false, 0, 0, 0, 80, true>(p, st);
        case 82: return launch_ws<T, 160, 1, 16, 4, 64, 4, 1, 1, 1, false, 0, 0, 0, 160, true>(p, st);
        case 83: return launch_ws<T, 160, 1, 16, 4, 32, 2, 1, 2, 1, false, 0, 0, 0, 160, true>(p, st);
        case 84: return launch_ws<T, 320, 1, 8, 4, 32, 2, 2, 1, 1, false, 0, 0, 0, 320, true>(p, st);
        case 85: return launch_ws<T, 320, 1, 16, 2, 32, 2, 2, 1, 1, false, 0, 0, 0, 320, true>(p, st);
        case 86: return launch_ws<T, 64, 1, 16, 4, 64, 2, 1, 2, 2, false, 0, 0, 0, 64, true>(p, st);
        case 87: return launch_ws<T, 128, 1, 16, 4, 128, 4, 1, 1, 1, false, 0, 0, 0, 128, true>(p, st);
        case 88: return launch_ws<T, 256, 1, 8, 4, 64, 2, 4, 1, 1, false, 0, 0, 0, 256, true>(p, st);
        // the training step's stem conv (Focus 12 channels stored as 16 -> yolox_x's 80, 3x3 s1): K = 32 with
        // the upper 16-channel half zero (round 5; it ran on the register-staged conv_igemm at ~110 TFLOP/s)
        case 89: return launch_ws<T, 32, 1, 16, 4, 80, 5, 1, 1, 1, false, 0, 0, 0, 16>(p, st);
        default: set_error("conv_ws tile id %d", id); return YXH_EINVAL;
    }
}

int conv_ws_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st) {
    if (p.taps != 9 || p.kw != 3 || p.pad != 1 || p.nsrc != 1 || p.sup[0] || p.sw[0] != p.in_w) {
        set_error("conv_ws needs a 3x3 pad-1 conv over one plain source");
        return YXH_EUNSUPPORTED;
    }
    if ((long long)p.in_h * p.in_w * p.scs[0] * 2 >= (1LL << 31)) {
        set_error("conv_ws: image exceeds 31-bit byte offsets");
        return YXH_EUNSUPPORTED;
    }
    if (dtype == YXH_BF16) return ws_dispatch_t<bf16>(id, p, st);
    if (dtype == YXH_F16) return ws_dispatch_t<f16>(id, p, st);
    set_error("conv_ws is built for bf16/f16");
    return YXH_EUNSUPPORTED;
}

}  // namespace yxh
