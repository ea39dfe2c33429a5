// conv_r3: 3x3 conv (stride 1 or 2, pad 1) with a branch-free LDS-DMA loader
// (reference network_blocks.py:48-49 BaseConv with ksize 3: the 3x3 convs of
// darknet.py / yolo_pafpn.py / yolo_head.py).
//
// Same tiling as conv_rows (a block = TN output channels x a TY x TX pixel tile of one
// image; per K stage (channel block cb, kernel row ky) the three kx taps of the weights
// and the TY input rows the tile reads, HX = (TX-1)*S + 3 pixels wide, land in LDS and
// the kx taps read the row image shifted by kx), but the loader does no per-stage
// address work:
//  * every DMA is a buffer_load ... lds through a buffer descriptor (image / weights):
//    the per-lane byte offset is computed ONCE per block, the stage offset (cb, ky) is a
//    scalar soffset, and zero padding is the descriptor's range check -- a lane whose
//    source pixel is outside the image carries an out-of-range offset and the hardware
//    writes zeros (no select, no branch, no zero buffer);
//  * the ky loop is unrolled against a 3-slot ring (slot = ky), so the per-lane offset
//    for row ky is one of three precomputed registers;
//  * instructions are A (weights) or B (pixels) per wave-uniform index, never mixed;
//  * DMAs are issued from inline asm: hipcc's own global/buffer_load_lds makes it put
//    s_waitcnt vmcnt(0) in front of every later ds_read (it cannot tell the ring slots
//    apart), which would drain the ring each stage; counted vmcnt + raw s_barrier order
//    the reads instead.
// TN = 64 (4 waves along pixels) or 128 (2 x 2); CH 16-byte chunks (8 channels each
// for 16-bit types) per stage.
#include "conv_common.hpp"
#include "lds_dma.hpp"

namespace yxh {

namespace {

// Probe builds only (tools/r3_split.sh): 1 = no MFMA / LDS reads, 2 = no DMA
#ifndef YXH_R3_PROBE
#define YXH_R3_PROBE 0
#endif

}  // namespace

// NBUF = 3: the ring slot of stage (cb, ky) is ky, two stages in flight;
// NBUF = 2: slot (3 cb + ky) & 1, one stage in flight, 2/3 of the LDS (more blocks per CU).
// A stage is exactly its A + B bytes: its 1 KiB wave-loads are dealt round-robin over
// the waves, and a wave whose share runs out skips the instruction (its counted vmcnt
// waits use its own per-stage count).
// NW waves per block (4 or 8); MINW = waves per SIMD the register budget must allow
// (8-wave blocks: 4 = two blocks per CU).
template <typename T, int S, int TX, int TY, int CH, int TN, int NBUF, int NW, int MINW>
__global__ __launch_bounds__(64 * NW, MINW) void conv_r3(ConvParams p, int tiles_x, int tiles_y, int ntn) {
    static_assert(NBUF == 2 || NBUF == 3, "ring depth");
    static_assert(NW == 4 || NW == 8 || NW == 16, "waves per block");
    constexpr int WN = TN >= 64 ? TN / 64 : 1, WM = NW / WN;  // wave grid: WN along channels
    constexpr int WTN = TN / WN;                               // 64 (or TN = 32)
    constexpr int EPC = Chunk<T>::N;
    constexpr int ES = sizeof(T);
    constexpr int KS = CH / 4;  // 64-byte slabs (one MFMA K step) per stage
    constexpr int KST = CH * EPC;
    constexpr int TM = TX * TY, WTM = TM / WM;
    constexpr int FR = WTN / 16, FC = WTM / 16;
    constexpr int HX = (TX - 1) * S + 3;
    constexpr int A_SLOTS = 3 * TN * CH, B_SLOTS = TY * HX * CH;
    constexpr int A_LOADS = A_SLOTS / 64, B_LOADS = (B_SLOTS + 63) / 64;  // 1 KiB wave-loads
    constexpr int GA = (A_LOADS + NW - 1) / NW, GB = (B_LOADS + NW - 1) / NW;
    constexpr int G = GA + GB;  // DMA instructions per wave per stage (at most)
    constexpr int A_PART = A_LOADS % NW, B_PART = B_LOADS % NW;  // waves in a partial last group
    constexpr int A_BYTES = A_LOADS * 1024;
    constexpr int BUF = A_BYTES + B_LOADS * 1024;
    constexpr int PXG = 16 / CH;
    static_assert(A_SLOTS % 64 == 0, "weight slots: whole wave-loads");
    static_assert(TM % (16 * WM) == 0, "pixel tile must split into 16-pixel fragments per wave");
    static_assert(G <= 20, "vmcnt range");
    __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nblk = tiles_x * tiles_y * (p.M / p.ohw) * ntn;
    const int bid = dma::xcd_remap(blockIdx.x, nblk);
    const int nt = bid % ntn;
    int t = bid / ntn;
    const int tx_i = t % tiles_x;
    t /= tiles_x;
    const int ty_i = t % tiles_y;
    const int b = t / tiles_y;
    const int n0 = nt * TN, oy0 = ty_i * TY, ox0 = tx_i * TX;
    const int wr = wave / WM, wc = wave % WM;
    const int cin = p.cin, scs = p.scs[0], in_w = p.in_w, in_h = p.in_h;

    const dma::u32x4 wsrd = dma::srd(p.w, (uint32_t)((long long)p.cout * 9 * cin * ES));
    const dma::u32x4 xsrd = dma::srd((const T*)p.sptr[0] + (long long)b * p.sbs[0],
                              (uint32_t)((long long)in_h * in_w * scs * ES));

    // per-lane DMA offsets, fixed for the block's life
    uint32_t aoff[GA];
#pragma unroll
    for (int i = 0; i < GA; ++i) {
        const int s = 64 * (wave + NW * i) + lane;
        const int kx = s / (CH * TN), rem = s - kx * (CH * TN);
        const int c = rem / TN, rp = rem - c * TN;
        const int n = min(n0 + (rp ^ (2 * (c & 3) + (c >> 2))), p.cout - 1);
        aoff[i] = s < A_SLOTS ? (uint32_t)(((n * 9 + kx) * cin + c * EPC) * ES) : dma::kOob;
    }
    uint32_t boff[GB][3];  // per kernel row ky
#pragma unroll
    for (int i = 0; i < GB; ++i) {
        const int sb = 64 * (wave + NW * i) + lane;
        const int hp = sb / CH, cp = sb - hp * CH;
        const int c = cp ^ ((hp / PXG) & (CH - 1));
        const int ty = hp / HX, hx = hp - ty * HX;
        const int iy0 = (oy0 + ty) * S - 1, ix = ox0 * S - 1 + hx;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
            const int iy = iy0 + ky;
            const bool ok = sb < B_SLOTS && iy >= 0 && iy < in_h && ix >= 0 && ix < in_w;
            boff[i][ky] = ok ? (uint32_t)(((iy * in_w + ix) * scs + c * EPC) * ES) : dma::kOob;
        }
    }
    const uint32_t lds0 = dma::lds_addr(smem) + (uint32_t)wave * 1024;

    auto issue_to = [&](int cb, auto kyc, uint32_t slot) {
        constexpr int ky = decltype(kyc)::value;
        if constexpr (YXH_R3_PROBE == 2) return;
        const uint32_t base = lds0 + slot * BUF;
        const uint32_t soa = (uint32_t)((ky * 3 * cin + cb * KST) * ES), sob = (uint32_t)(cb * KST * ES);
#pragma unroll
        for (int i = 0; i < GA; ++i)
            if (A_PART == 0 || i + 1 < GA || wave < A_PART)
                dma::load16(wsrd, aoff[i], soa, base + i * NW * 1024);
#pragma unroll
        for (int i = 0; i < GB; ++i)
            if (B_PART == 0 || i + 1 < GB || wave < B_PART)
                dma::load16(xsrd, boff[i][ky], sob, base + A_BYTES + i * NW * 1024);
    };
    auto issue = [&](int cb, auto kyc) { issue_to(cb, kyc, (uint32_t)decltype(kyc)::value); };

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

    auto compute = [&](int slot) {
        if constexpr (YXH_R3_PROBE == 1) return;
        const char* A = smem + slot * BUF;
        const char* B = A + A_BYTES;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
#pragma unroll
            for (int sl = 0; sl < KS; ++sl) {
                const int chunk = sl * 4 + fq, swa = 2 * fq + sl;
                uint4 af[FR], bf[FC];
#pragma unroll
                for (int i = 0; i < FR; ++i) {
                    const int r = wr * WTN + i * 16 + frow;
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

    using K0 = std::integral_constant<int, 0>;
    using K1 = std::integral_constant<int, 1>;
    using K2 = std::integral_constant<int, 2>;
    const int ncb = p.ncb;
    // this wave's DMA instructions per stage, and "wait until one younger stage remains"
    const int cnt = G - (A_PART && wave >= A_PART ? 1 : 0) - (B_PART && wave >= B_PART ? 1 : 0);
    auto wait_younger = [&]() {
        if (cnt == G) dma::wait_vm<G>();
        else if (cnt == G - 1) dma::wait_vm<G - 1>();
        else dma::wait_vm<G - 2>();
    };
    if constexpr (NBUF == 3) {
        issue(0, K0{});
        issue(0, K1{});
        // stage (cb, ky): wait for it (one younger stage may fly), barrier, issue the stage
        // two ahead into the slot stage (cb, ky-1) just vacated, compute
        for (int cb = 0; cb < ncb; ++cb) {
            const bool more = cb + 1 < ncb;
            wait_younger();
            dma::barrier();
            issue(cb, K2{});
            compute(0);
            wait_younger();
            dma::barrier();
            if (more) issue(cb + 1, K0{});
            compute(1);
            if (more) wait_younger();
            else dma::wait_vm<0>();
            dma::barrier();
            if (more) issue(cb + 1, K1{});
            compute(2);
        }
    } else {
        // stage s = 3 cb + ky in slot s & 1: wait for it, barrier (every wave is done with
        // stage s - 1, whose slot the next stage takes), issue stage s + 1, compute
        issue_to(0, K0{}, 0u);
        for (int cb = 0; cb < ncb; ++cb) {
            const uint32_t s0 = (uint32_t)(3 * cb) & 1u;
            dma::wait_vm<0>();
            dma::barrier();
            issue_to(cb, K1{}, s0 ^ 1u);
            compute((int)s0);
            dma::wait_vm<0>();
            dma::barrier();
            issue_to(cb, K2{}, s0);
            compute((int)(s0 ^ 1u));
            dma::wait_vm<0>();
            dma::barrier();
            if (cb + 1 < ncb) issue_to(cb + 1, K0{}, s0 ^ 1u);
            compute((int)s0);
        }
    }
    dma::wait_vm<0>();
    dma::barrier();
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

// conv_r3h: the same conv with the pixel operand staged ONCE per channel block.
// conv_r3 stages, per (cb, ky), the TY input rows that kernel row ky reads: every input row
// is fetched three times.  Here a stage of channel block cb is the whole halo tile
// (HY = (TY-1)*S + 3 rows x HX pixels x 32 channels, one B slot of two, by cb parity) and
// the weights of ONE kernel row (3 taps x TN x 32 channels, A ring of three, slot ky):
//   stage (cb, 0): A(cb, 0) + B(cb);  stage (cb, 1): A(cb, 1);  stage (cb, 2): A(cb, 2)
// and kernel row ky reads B rows ty*S + ky.  Two stages stay in flight (the A ring of
// three); the DMA bytes per channel block drop from 3*TY*HX to HY*HX pixel chunks, which
// matters because the LDS-DMA path (~10 TB/s chip-wide, MI355X_MICROARCH.md ldsdma-fill)
// is what bounds conv_r3 (probe: DMA alone 117 us of a 145 us 80x80 128->256 launch).
__device__ __forceinline__ void r3_wait_dyn(int n) {
    switch (n) {
#define YXH_W(k) \
    case k: dma::wait_vm<k>(); break;
        YXH_W(1) YXH_W(2) YXH_W(3) YXH_W(4) YXH_W(5) YXH_W(6) YXH_W(7) YXH_W(8) YXH_W(9) YXH_W(10)
        YXH_W(11) YXH_W(12) YXH_W(13) YXH_W(14) YXH_W(15) YXH_W(16) YXH_W(17) YXH_W(18) YXH_W(19) YXH_W(20)
#undef YXH_W
        default: dma::wait_vm<0>(); break;
    }
}

template <typename T, int S, int TX, int TY, int TN, int NW, int MINW>
__global__ __launch_bounds__(64 * NW, MINW) void conv_r3h(ConvParams p, int tiles_x, int tiles_y, int ntn) {
    constexpr int CH = 4;  // 16-byte chunks (32 channels) per channel block
    constexpr int WN = TN >= 64 ? TN / 64 : 1, WM = NW / WN, WTN = TN / WN;
    constexpr int EPC = Chunk<T>::N;
    constexpr int ES = sizeof(T);
    constexpr int KST = CH * EPC;
    constexpr int TM = TX * TY, WTM = TM / WM;
    constexpr int FR = WTN / 16, FC = WTM / 16;
    constexpr int HX = (TX - 1) * S + 3, HY = (TY - 1) * S + 3;
    constexpr int A_SLOTS = 3 * TN * CH, B_SLOTS = HY * HX * CH;
    constexpr int A_LOADS = A_SLOTS / 64, B_LOADS = (B_SLOTS + 63) / 64;
    constexpr int GA = (A_LOADS + NW - 1) / NW, GB = (B_LOADS + NW - 1) / NW;
    constexpr int A_PART = A_LOADS % NW, B_PART = B_LOADS % NW;
    constexpr int ABUF = A_LOADS * 1024, BBUF = B_LOADS * 1024;
    constexpr int SMEM = 3 * ABUF + 2 * BBUF;
    static_assert(A_SLOTS % 64 == 0 && TM % (16 * WM) == 0 && GA + GB <= 20, "tile");
    static_assert(SMEM <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nblk = tiles_x * tiles_y * (p.M / p.ohw) * ntn;
    const int bid = dma::xcd_remap(blockIdx.x, nblk);
    const int nt = bid % ntn;
    int t = bid / ntn;
    const int tx_i = t % tiles_x;
    t /= tiles_x;
    const int ty_i = t % tiles_y;
    const int b = t / tiles_y;
    const int n0 = nt * TN, oy0 = ty_i * TY, ox0 = tx_i * TX;
    const int wr = wave / WM, wc = wave % WM;
    const int cin = p.cin, scs = p.scs[0], in_w = p.in_w, in_h = p.in_h;

    const dma::u32x4 wsrd = dma::srd(p.w, (uint32_t)((long long)p.cout * 9 * cin * ES));
    const dma::u32x4 xsrd = dma::srd((const T*)p.sptr[0] + (long long)b * p.sbs[0],
                              (uint32_t)((long long)in_h * in_w * scs * ES));
    uint32_t aoff[GA];
#pragma unroll
    for (int i = 0; i < GA; ++i) {
        const int s = 64 * (wave + NW * i) + lane;
        const int kx = s / (CH * TN), rem = s - kx * (CH * TN);
        const int c = rem / TN, rp = rem - c * TN;
        const int n = min(n0 + (rp ^ (2 * c)), p.cout - 1);
        aoff[i] = s < A_SLOTS ? (uint32_t)(((n * 9 + kx) * cin + c * EPC) * ES) : dma::kOob;
    }
    uint32_t boff[GB];
#pragma unroll
    for (int i = 0; i < GB; ++i) {
        const int sb = 64 * (wave + NW * i) + lane;
        const int hp = sb / CH, cp = sb - hp * CH;
        const int c = cp ^ ((hp >> 2) & 3);
        const int hy = hp / HX, hx = hp - hy * HX;
        const int iy = oy0 * S - 1 + hy, ix = ox0 * S - 1 + hx;
        const bool ok = sb < B_SLOTS && iy >= 0 && iy < in_h && ix >= 0 && ix < in_w;
        boff[i] = ok ? (uint32_t)(((iy * in_w + ix) * scs + c * EPC) * ES) : dma::kOob;
    }
    const uint32_t lds0 = dma::lds_addr(smem) + (uint32_t)wave * 1024;
    // this wave's share of a stage's wave-loads
    const int cnt_a = GA - (A_PART && wave >= A_PART ? 1 : 0);
    const int cnt_b = GB - (B_PART && wave >= B_PART ? 1 : 0);

    auto issue_a = [&](int cb, int ky) {
        if constexpr (YXH_R3_PROBE == 2) return;
        const uint32_t base = lds0 + (uint32_t)(ky * ABUF);
        const uint32_t soa = (uint32_t)((ky * 3 * cin + cb * KST) * ES);
#pragma unroll
        for (int i = 0; i < GA; ++i)
            if (A_PART == 0 || i + 1 < GA || wave < A_PART) dma::load16(wsrd, aoff[i], soa, base + i * NW * 1024);
    };
    auto issue_b = [&](int cb) {
        if constexpr (YXH_R3_PROBE == 2) return;
        const uint32_t base = lds0 + (uint32_t)(3 * ABUF + (cb & 1) * BBUF);
        const uint32_t sob = (uint32_t)(cb * KST * ES);
#pragma unroll
        for (int i = 0; i < GB; ++i)
            if (B_PART == 0 || i + 1 < GB || wave < B_PART) dma::load16(xsrd, boff[i], sob, base + i * NW * 1024);
    };

    f32x4 acc[FR][FC];
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float lbias[FR][4];
    load_lane_bias<TN, WN, WM>(p, n0, lbias);

    const int frow = lane & 15, fq = lane >> 4;
    int hp0[FC];  // halo-tile pixel of this lane's fragment column at (ky, kx) = (0, 0)
#pragma unroll
    for (int j = 0; j < FC; ++j) {
        const int pl = wc * WTM + j * 16 + frow;
        const int ty = pl / TX, tx = pl - ty * TX;
        hp0[j] = ty * S * HX + tx * S;
    }

    auto compute = [&](int cb, auto kyc) {
        if constexpr (YXH_R3_PROBE == 1) return;
        constexpr int ky = decltype(kyc)::value;
        const char* A = smem + ky * ABUF;
        const char* B = smem + 3 * ABUF + (cb & 1) * BBUF;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            uint4 af[FR], bf[FC];
#pragma unroll
            for (int i = 0; i < FR; ++i) {
                const int r = wr * WTN + i * 16 + frow;
                af[i] = *(const uint4*)(A + ((kx * CH + fq) * TN + (r ^ (2 * fq))) * 16);
            }
#pragma unroll
            for (int j = 0; j < FC; ++j) {
                const int hp = hp0[j] + ky * HX + kx;
                bf[j] = *(const uint4*)(B + (hp * CH + (fq ^ ((hp >> 2) & 3))) * 16);
            }
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int j = 0; j < FC; ++j) Mma<T>::run(acc[i][j], af[i], bf[j]);
        }
    };

    using K0 = std::integral_constant<int, 0>;
    using K1 = std::integral_constant<int, 1>;
    using K2 = std::integral_constant<int, 2>;
    const int ncb = p.ncb;
    issue_a(0, 0);
    issue_b(0);
    issue_a(0, 1);
    for (int cb = 0; cb < ncb; ++cb) {
        const bool more = cb + 1 < ncb;
        r3_wait_dyn(cnt_a);  // stage (cb, 0) landed; (cb, 1) may fly
        dma::barrier();
        issue_a(cb, 2);
        compute(cb, K0{});
        r3_wait_dyn(cnt_a);  // (cb, 1) landed; (cb, 2) may fly
        dma::barrier();
        if (more) {
            issue_a(cb + 1, 0);
            issue_b(cb + 1);
        }
        compute(cb, K1{});
        r3_wait_dyn(more ? cnt_a + cnt_b : 0);  // (cb, 2) landed; (cb + 1, 0) may fly
        dma::barrier();
        if (more) issue_a(cb + 1, 1);
        compute(cb, K2{});
    }
    dma::wait_vm<0>();
    dma::barrier();
    const int OH = p.out_h, OW = p.out_w, mb = b * p.ohw;
    conv_epilogue_map<T, TN, TM, WN, WM, SMEM>(
        p, acc, smem,
        [=](int pl) {
            const int ty = pl / TX, tx = pl - ty * TX;
            const int oy = oy0 + ty, ox = ox0 + tx;
            return (oy < OH && ox < OW) ? mb + oy * OW + ox : -1;
        },
        n0, lbias);
}

template <typename T, int S, int TX, int TY, int TN, int NW, int MINW = NW >= 8 ? 4 : 1>
static int launch_r3h(const ConvParams& p, hipStream_t st) {
    if (p.stride != S) {
        set_error("conv_r3h variant built for stride %d", S);
        return YXH_EUNSUPPORTED;
    }
    const int kst = 4 * Chunk<T>::N;
    if (p.cin % kst) {
        set_error("conv_r3h: cin %d not a multiple of the %d-channel stage", p.cin, kst);
        return YXH_EUNSUPPORTED;
    }
    ConvParams q = p;
    q.ncb = p.cin / kst;
    const int tiles_x = (p.out_w + TX - 1) / TX, tiles_y = (p.out_h + TY - 1) / TY;
    const int ntn = (p.cout + TN - 1) / TN;
    const long long nblk = (long long)tiles_x * tiles_y * (p.M / p.ohw) * ntn;
    if (nblk >= (1LL << 31)) {
        set_error("conv_r3h grid too large");
        return YXH_EINVAL;
    }
    hipLaunchKernelGGL((conv_r3h<T, S, TX, TY, TN, NW, MINW>), dim3((unsigned)nblk), dim3(64 * NW), 0, st, q, tiles_x,
                       tiles_y, ntn);
    YXH_CHECK_LAUNCH("conv_r3h launch");
    return YXH_OK;
}

template <typename T, int S, int TX, int TY, int CH, int TN, int NBUF = 3, int NW = 4, int MINW = NW >= 8 ? 4 : 1>
static int launch_r3(const ConvParams& p, hipStream_t st) {
    constexpr int HX = (TX - 1) * S + 3;
    constexpr int AL = 3 * TN * CH / 64, BL = (TY * HX * CH + 63) / 64;
    constexpr int G = (AL + NW - 1) / NW + (BL + NW - 1) / NW;
    constexpr int lds = NBUF * (AL + BL) * 1024;
    if constexpr (lds > 160 * 1024 || G > 20) {
        set_error("conv_r3 variant needs more than 160 KiB of LDS");
        return YXH_EUNSUPPORTED;
    } else {
        if (p.stride != S) {
            set_error("conv_r3 variant built for stride %d", S);
            return YXH_EUNSUPPORTED;
        }
        const int kst = CH * Chunk<T>::N;
        if (p.cin % kst) {
            set_error("conv_r3: cin %d not a multiple of the %d-channel stage", p.cin, kst);
            return YXH_EUNSUPPORTED;
        }
        ConvParams q = p;
        q.ncb = p.cin / kst;
        const int tiles_x = (p.out_w + TX - 1) / TX, tiles_y = (p.out_h + TY - 1) / TY;
        const int ntn = (p.cout + TN - 1) / TN;
        const long long nblk = (long long)tiles_x * tiles_y * (p.M / p.ohw) * ntn;
        if (nblk >= (1LL << 31)) {
            set_error("conv_r3 grid too large");
            return YXH_EINVAL;
        }
        hipLaunchKernelGGL((conv_r3<T, S, TX, TY, CH, TN, NBUF, NW, MINW>), dim3((unsigned)nblk), dim3(64 * NW), 0, st, q, tiles_x,
                           tiles_y, ntn);
        YXH_CHECK_LAUNCH("conv_r3 launch");
        return YXH_OK;
    }
}

template <typename T>
static int r3_dispatch_t(int id, const ConvParams& p, hipStream_t st) {
    // id -> (stride, TX, TY, CH, TN, ring slots, waves, min waves per SIMD)
    switch (id) {
        // 4 waves, three-slot ring: 63 KiB -> two blocks per CU
        case 1: return launch_r3<T, 1, 16, 8, 4, 64>(p, st);
        case 2: return launch_r3<T, 1, 32, 4, 4, 64>(p, st);
        case 3: return launch_r3<T, 2, 16, 4, 4, 64>(p, st);
        case 4: return launch_r3<T, 2, 8, 8, 4, 64>(p, st);
        // 4 waves, two-slot ring (one stage in flight): 42 KiB -> three blocks, 58-66 KiB -> two
        case 5: return launch_r3<T, 1, 16, 8, 4, 64, 2>(p, st);
        case 6: return launch_r3<T, 1, 32, 4, 4, 64, 2>(p, st);
        case 7: return launch_r3<T, 1, 32, 8, 4, 64, 2>(p, st);
        case 8: return launch_r3<T, 1, 16, 16, 4, 64, 2>(p, st);
        case 9: return launch_r3<T, 1, 16, 8, 4, 128, 2>(p, st);
        case 10: return launch_r3<T, 2, 16, 4, 4, 64, 2>(p, st);
        case 11: return launch_r3<T, 2, 8, 8, 4, 64, 2>(p, st);
        case 12: return launch_r3<T, 2, 16, 8, 4, 64, 2>(p, st);
        // 8-wave blocks, two-slot ring, two blocks per CU
        case 14: return launch_r3<T, 1, 32, 8, 4, 64, 2, 8>(p, st);
        case 16: return launch_r3<T, 1, 8, 8, 4, 128, 2, 8>(p, st);
        case 17: return launch_r3<T, 2, 8, 8, 4, 128, 2, 8>(p, st);
        case 18: return launch_r3<T, 2, 16, 8, 4, 64, 2, 8>(p, st);
        case 19: return launch_r3<T, 1, 16, 8, 4, 64, 2, 8>(p, st);
        case 20: return launch_r3<T, 2, 8, 16, 4, 64, 2, 8>(p, st);
        // 8 waves, three-slot ring (two stages in flight)
        case 21: return launch_r3<T, 1, 16, 8, 4, 64, 3, 8>(p, st);
        case 22: return launch_r3<T, 1, 32, 4, 4, 64, 3, 8>(p, st);
        // ids 13, 15, 23-25 and the 16-bit 29 spilled to scratch at their occupancy targets
        // (tools/kernel_resources.py): withdrawn (EINVAL)
        // one block per CU, wide tiles (small late layers)
        case 26: return launch_r3<T, 1, 20, 16, 4, 64>(p, st);
        case 27: return launch_r3<T, 2, 20, 8, 4, 128>(p, st);
        // 32 output channels per block (cout = 32 layers)
        case 28: return launch_r3<T, 1, 32, 8, 4, 32, 2, 8>(p, st);
        // conv_r3h: halo tile staged once per channel block -> (stride, TX, TY, TN, waves)
        case 30: return launch_r3h<T, 1, 32, 8, 64, 8>(p, st);
        case 31: return launch_r3h<T, 1, 16, 8, 64, 4>(p, st);
        case 32: return launch_r3h<T, 1, 32, 8, 32, 8>(p, st);
        case 33: return launch_r3h<T, 2, 8, 8, 64, 4>(p, st);
        case 34: return launch_r3h<T, 2, 16, 8, 64, 8, 2>(p, st);
        case 35: return launch_r3h<T, 2, 8, 16, 64, 8, 2>(p, st);
        case 36: return launch_r3h<T, 1, 16, 16, 128, 8, 2>(p, st);
        case 37: return launch_r3h<T, 1, 32, 16, 64, 16>(p, st);
        case 38: return launch_r3h<T, 1, 16, 8, 64, 8>(p, st);
        // 20-pixel-wide tiles for 20 x 20 outputs (yolox_l / yolox_x dark5 and PAFPN 512-channel 3x3s: the 32-wide
        // tiles compute 37.5 % padding there); stride 2: 17 x 41 halo + three 24 KiB weight slots = all 160 KiB
        case 39: return launch_r3h<T, 2, 20, 8, 128, 4>(p, st);
        case 40: return launch_r3h<T, 1, 20, 8, 128, 4>(p, st);
        default: set_error("conv_r3 tile id %d", id); return YXH_EINVAL;
    }
}

// fp32 (the training path at BASELINE configs[2]): the halo-tile kernel only; a stage is
// 16 channels (4 fp32 per 16-byte chunk) and each fragment pair is 4 x v_mfma_f32_16x16x4f32,
// so the kernel is MFMA-bound where its 16-bit form is DMA-bound.
static int r3h_dispatch_f32(int id, const ConvParams& p, hipStream_t st) {
    switch (id) {
        // 16 x 16 TN 64 8 waves: held to 128 VGPRs (two blocks per CU) it spilled 16 B/lane; one
        // block per CU, 256 VGPRs
        case 29: return launch_r3h<float, 1, 16, 16, 64, 8, 2>(p, st);
        case 30: return launch_r3h<float, 1, 32, 8, 64, 8>(p, st);
        case 31: return launch_r3h<float, 1, 16, 8, 64, 4>(p, st);
        case 32: return launch_r3h<float, 1, 32, 8, 32, 8>(p, st);
        case 33: return launch_r3h<float, 2, 8, 8, 64, 4>(p, st);
        case 38: return launch_r3h<float, 1, 16, 8, 64, 8>(p, st);
        case 39: return launch_r3h<float, 2, 20, 8, 128, 4>(p, st);
        case 40: return launch_r3h<float, 1, 20, 8, 128, 4>(p, st);
        default: set_error("conv_r3 tile id %d is built for bf16/f16 only", id); return YXH_EUNSUPPORTED;
    }
}

int conv_r3_dispatch(int dtype, int id, const ConvParams& p, hipStream_t st) {
    if (p.taps != 9 || p.kw != 3 || p.pad != 1 || p.nsrc != 1 || p.sup[0] || p.sw[0] != p.in_w) {
        set_error("conv_r3 needs a 3x3 pad-1 conv over one plain source");
        return YXH_EUNSUPPORTED;
    }
    const long long es = dtype == YXH_F32 ? 4 : 2;
    if ((long long)p.in_h * p.in_w * p.scs[0] * es >= (1LL << 31) || (long long)p.cout * 9 * p.cin * es >= (1LL << 31)) {
        set_error("conv_r3: image / weights exceed 31-bit byte offsets");
        return YXH_EUNSUPPORTED;
    }
    if (dtype == YXH_BF16) return r3_dispatch_t<bf16>(id, p, st);
    if (dtype == YXH_F16) return r3_dispatch_t<f16>(id, p, st);
    if (dtype == YXH_F32) return r3h_dispatch_f32(id, p, st);
    set_error("conv_r3: dtype %d", dtype);
    return YXH_EUNSUPPORTED;
}

}  // namespace yxh
