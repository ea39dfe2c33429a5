// Detection post-processing on gfx950: utils.postprocess (reference
// yolox/utils/boxes.py:31-75) with torchvision nms / batched_nms semantics.
//
//   pp_filter : one wave per 64 anchors; the [64 x (5+C)] fp32 tile is read
//               coalesced into LDS (odd row stride -> conflict-free row reads),
//               cxcywh->xyxy is written back in place (boxes.py:32-37), class max
//               (first index, :46), score >= conf (fp32, :48) and compaction by a
//               per-image atomic counter.  Slot order is arbitrary; everything
//               downstream is keyed by (score desc, anchor asc) so results are
//               deterministic.
//   pp_sort_chunk / pp_merge / pp_gather : score sort of each image's candidates by
//               64-bit keys: chunks of 16384 bitonic-sorted in LDS (one chunk covers a
//               640 input's 8400 anchors), then, only for larger candidate sets (1280
//               inputs: 33600 anchors), log2(n/16384) pairwise merge passes (rank in own
//               run + lower_bound in the partner run); sorted rows gathered, max
//               coordinate for the coordinate-offset branch.  No candidate cap.
//   pp_mask   : 64x64 tiles of the upper-triangular suppression matrix; lane t of a
//               wave owns sorted box i = 64*rb + t and emits one 64-bit word per column
//               block (the wave64 <-> 64-bit mask correspondence).
//   pp_reduce : one wave per image walks the sorted boxes, keeps the unsuppressed
//               ones and ORs their mask rows (greedy NMS), writing detections in keep
//               order.
//   The matrix is built and consumed in passes of R sorted rows (R from a fixed byte
//   budget, pp_rows_per_pass): pass p holds rows [p*R, (p+1)*R) against every column, its
//   reduce continues the removed set and keep count of pass p-1 (kept in the workspace).
//   Greedy NMS only ever reads the rows of boxes it has reached, so the result is that
//   of the whole matrix; the workspace no longer grows with the square of the anchor
//   count, and passes past an image's candidate count exit at once.
//
// Bit-exactness: IoU is evaluated with exactly torchvision's CPU fp32 operation
// sequence (areas=(x2-x1)*(y2-y1); inter=w*h; inter/((a_i+a_j)-inter) > (double)thr),
// so FP contraction is disabled for this file (and -ffp-contract=off at build).
#pragma clang fp contract(off)

#include <algorithm>

#include "yxh_common.hpp"

namespace yxh {

constexpr int kSortCap = 16384;      // keys sorted per block in LDS (128 KiB)
constexpr int kMaxAnchors = 1 << 19;  // pp_reduce keeps one removed-bit per candidate in LDS
constexpr int kRow = 8;  // x1 y1 x2 y2 obj conf cls score
// bytes of suppression words per pass (all images): 320 MiB holds every row of the bench's batch (32 x 8 400
// anchors: 285 MiB) in one pass -- at 256 MiB a second mask + reduce pass launched ~8 000 blocks that
// had nothing to do (the candidates of conf 0.5 fit the first 64-row blocks)
constexpr size_t kMaskBudget = 320ull << 20;
size_t g_mask_budget = kMaskBudget;  // yxh_set_nms_mask_budget (tests: force many passes)

struct PPWork {
    int* cnt;         // [B]
    float* maxc;      // [B]
    int* slot_of;     // [B][A]
    unsigned long long* key;  // [B][A]
    float* cand;      // [B][A][8]
    float* srt;       // [B][A][8] sorted
    unsigned long long* mask;     // [B][rows per pass][capw]
    unsigned long long* removed;  // [B][capw] greedy state carried across passes
    int cap, capw;
};

__device__ __forceinline__ unsigned int ordered(float f) {
    unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Filter (boxes.py:36-52): one block = 64 anchor rows staged in LDS; four lanes per row
// each take the argmax over a quarter of the classes (first maximum wins, as a serial
// strict '>' scan does), combined with two lane shuffles.
__global__ __launch_bounds__(256) void pp_filter(float* pred, int A, int C, float conf, PPWork w) {
    extern __shared__ __attribute__((aligned(16))) float tile[];  // [64][5+C]
    const int D = 5 + C;
    const int b = blockIdx.y, a0 = blockIdx.x * 64, tid = threadIdx.x;
    const int rows = min(64, A - a0);
    float* src = pred + ((long long)b * A + a0) * D;
    // the block's rows are one contiguous run: 16-byte loads when it is aligned (the bench's
    // [32, 8400, 85] rows: every block), 4-byte ones otherwise
    const int n = rows * D;
    if ((n & 3) == 0 && ((uintptr_t)src & 15) == 0) {
        for (int q = tid; q < (n >> 2); q += 256) ((float4*)tile)[q] = ((const float4*)src)[q];
    } else {
        for (int q = tid; q < n; q += 256) tile[q] = src[q];
    }
    __syncthreads();
    const int r = tid >> 2, part = tid & 3;
    const float* p = tile + min(r, rows - 1) * D;
    // the serial scan starts from class 0 and replaces on a strict '>': quarter 0 does
    // exactly that; later quarters start empty (bi == C) and so skip NaNs and never win
    // a tie against a lower class; only quarter 0 can hold a NaN (class 0 itself)
    const int per = (C + 3) / 4, c0 = part * per, c1 = min(C, c0 + per);
    float best = part == 0 ? p[5] : -INFINITY;
    int bi = part == 0 ? 0 : C;
    for (int c = part == 0 ? 1 : c0; c < c1; ++c) {
        const float v = p[5 + c];
        if (v > best) { best = v; bi = c; }
    }
#pragma unroll
    for (int off = 1; off < 4; off <<= 1) {
        const float ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(bi, off);
        bool take;
        if (oi >= C) take = false;
        else if (bi >= C) take = true;
        else if (best != best) take = false;  // ours: class 0 is NaN, the serial answer
        else if (ob != ob) take = true;       // theirs
        else take = ob > best || (ob == best && oi < bi);
        if (take) { best = ob; bi = oi; }
    }
    if (part == 0 && r < rows) {
        const float cx = p[0], cy = p[1], bw = p[2], bh = p[3];
        const float hw = bw / 2.0f, hh = bh / 2.0f;
        const float x1 = cx - hw, y1 = cy - hh, x2 = cx + hw, y2 = cy + hh;
        float* g = src + r * D;
        g[0] = x1; g[1] = y1; g[2] = x2; g[3] = y2;
        const float obj = p[4];
        const float sc = obj * best;
        if (sc >= conf) {
            const int a = a0 + r;
            const int slot = atomicAdd(&w.cnt[b], 1);
            w.slot_of[(long long)b * A + a] = slot;
            w.key[(long long)b * A + slot] =
                ((unsigned long long)(~ordered(sc)) << 32) | (unsigned int)a;
            float* o = w.cand + ((long long)b * A + slot) * kRow;
            *(float4*)o = make_float4(x1, y1, x2, y2);
            *(float4*)(o + 4) = make_float4(obj, best, (float)bi, sc);
        }
    }
}

// The filter fed by the forward's per-anchor records (yxh_head_desc.scores, ABI 18): one thread per
// anchor reads its 32-byte record {obj * max class, max class, class index, obj | cx, cy, w, h} --
// written by head_pred2 from the very fp32 values it put in the row, the class maximum with this
// file's first-maximum / NaN rules -- and only WRITES the row's xyxy box in place (boxes.py:32-37).
// Candidates are pp_filter's (sc >= conf, the same key and candidate row).
__global__ __launch_bounds__(256) void pp_filter_scored(float* pred, const float4* scores, int A, int C, float conf,
                                                        PPWork w) {
    const int b = blockIdx.y, a = blockIdx.x * 256 + threadIdx.x;
    if (a >= A) return;
    const int D = 5 + C;
    const long long ra = (long long)b * A + a;
    const float4 rec = scores[2 * ra], box = scores[2 * ra + 1];
    const float cx = box.x, cy = box.y, bw = box.z, bh = box.w;
    const float hw = bw / 2.0f, hh = bh / 2.0f;
    const float x1 = cx - hw, y1 = cy - hh, x2 = cx + hw, y2 = cy + hh;
    float* g = pred + ra * D;
    g[0] = x1; g[1] = y1; g[2] = x2; g[3] = y2;
    const float sc = rec.x;
    if (sc >= conf) {
        const int slot = atomicAdd(&w.cnt[b], 1);
        w.slot_of[ra] = slot;
        w.key[(long long)b * A + slot] = ((unsigned long long)(~ordered(sc)) << 32) | (unsigned int)a;
        float* o = w.cand + ((long long)b * A + slot) * kRow;
        *(float4*)o = make_float4(x1, y1, x2, y2);
        *(float4*)(o + 4) = make_float4(rec.w, rec.y, rec.z, sc);
    }
}

// counters of the filter (per image) and the caller's detection counts, zeroed in one launch
__global__ __launch_bounds__(256) void pp_init(int B, int* cnt, int* counts) {
    for (int q = threadIdx.x; q < B; q += 256) {
        cnt[q] = 0;
        counts[q] = 0;
    }
}

// Stage 1 of the score sort: chunk c of image b (keys [c*kSortCap, ...) of its n
// candidates) is bitonic-sorted in LDS and written back in place.  With A <= kSortCap
// there is one chunk and the sort is complete.
__global__ __launch_bounds__(1024) void pp_sort_chunk(int A, PPWork w) {
    __shared__ unsigned long long keys[kSortCap];
    const int b = blockIdx.y, tid = threadIdx.x;
    const int n = w.cnt[b];
    const int lo = blockIdx.x * kSortCap;
    if (lo >= n) return;
    const int m = min(kSortCap, n - lo);
    unsigned long long* g = w.key + (long long)b * A + lo;
    int np2 = 1;
    while (np2 < m) np2 <<= 1;
    for (int q = tid; q < np2; q += 1024) keys[q] = q < m ? g[q] : ~0ull;
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int q = tid; q < np2; q += 1024) {
                const int ixj = q ^ j;
                if (ixj > q) {
                    const unsigned long long x = keys[q], y = keys[ixj];
                    const bool asc = (q & k) == 0;
                    if ((x > y) == asc) {
                        keys[q] = y;
                        keys[ixj] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (int q = tid; q < m; q += 1024) g[q] = keys[q];
}

// Stage 2 (only when A > kSortCap): merge sorted runs of length L pairwise.  Keys are
// unique (the anchor index is in the low word), so an element's output position is
// its rank in its own run plus the number of smaller keys in the partner run.
__global__ __launch_bounds__(256) void pp_merge(int A, PPWork w, int L, const unsigned long long* src,
                                                unsigned long long* dst) {
    const int b = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    const int n = w.cnt[b];
    if (i >= n) return;
    const unsigned long long* s = src + (long long)b * A;
    unsigned long long* d = dst + (long long)b * A;
    const int run = i / L, start = run * L;
    const int ps = (run ^ 1) * L;
    const unsigned long long key = s[i];
    if (ps >= n) {
        d[i] = key;
        return;
    }
    int lo = ps, hi = min(ps + L, n);  // lower_bound of key in [ps, pe)
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[mid] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    d[min(start, ps) + (i - start) + (lo - ps)] = key;
}

// Stage 3: sorted candidate rows (by the final key order) and the max box coordinate
// for the coordinate-offset branch of batched_nms.
__global__ __launch_bounds__(1024) void pp_gather(int A, PPWork w, const unsigned long long* keys) {
    __shared__ float red[1024 / 64];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int n = w.cnt[b];
    float m = -INFINITY;
    for (int q = tid; q < n; q += 1024) {
        const float4 r = *(const float4*)(w.cand + ((long long)b * A + q) * kRow);
        m = fmaxf(m, fmaxf(fmaxf(r.x, r.y), fmaxf(r.z, r.w)));
    }
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    if ((tid & 63) == 0) red[tid >> 6] = m;
    __syncthreads();
    if (tid == 0) {
        float mm = red[0];
        for (int i = 1; i < 16; ++i) mm = fmaxf(mm, red[i]);
        w.maxc[b] = mm;
    }
    const unsigned long long* kb = keys + (long long)b * A;
    for (int q = tid; q < n; q += 1024) {
        const int a = (int)(kb[q] & 0xffffffffu);
        const int slot = w.slot_of[(long long)b * A + a];
        const float* s = w.cand + ((long long)b * A + slot) * kRow;
        float* d = w.srt + ((long long)b * A + q) * kRow;
        *(float4*)d = *(const float4*)s;
        *(float4*)(d + 4) = *(const float4*)(s + 4);
    }
}

struct Box {
    float x1, y1, x2, y2, area, cls;
};

__device__ __forceinline__ Box load_box(const float* r, int mode, float step) {
    Box bx;
    bx.x1 = r[0]; bx.y1 = r[1]; bx.x2 = r[2]; bx.y2 = r[3];
    bx.cls = r[6];
    if (mode == 1) {  // coordinate trick: boxes + idxs * (max + 1)
        const float off = bx.cls * step;
        bx.x1 = bx.x1 + off; bx.y1 = bx.y1 + off; bx.x2 = bx.x2 + off; bx.y2 = bx.y2 + off;
    }
    const float ww = bx.x2 - bx.x1;
    const float hh = bx.y2 - bx.y1;
    bx.area = ww * hh;
    return bx;
}

// torchvision nms_kernel.cpp inner loop, operation for operation.
__device__ __forceinline__ bool suppresses(const Box& i, const Box& j, double thr) {
    const float xx1 = i.x1 < j.x1 ? j.x1 : i.x1;
    const float yy1 = i.y1 < j.y1 ? j.y1 : i.y1;
    const float xx2 = j.x2 < i.x2 ? j.x2 : i.x2;
    const float yy2 = j.y2 < i.y2 ? j.y2 : i.y2;
    const float dw = xx2 - xx1, dh = yy2 - yy1;
    const float w = 0.0f < dw ? dw : 0.0f;
    const float h = 0.0f < dh ? dh : 0.0f;
    const float inter = w * h;
    const float den = (i.area + j.area) - inter;
    const float ovr = inter / den;
    return (double)ovr > thr;
}

__device__ __forceinline__ int image_mode(int n, int agnostic, long long vanilla_numel) {
    if (agnostic) return 0;
    return (4LL * n > vanilla_numel) ? 2 : 1;
}

// Suppression bitmask, one 64 x 64 (row block, column block) pair per work item: the four
// waves of a block each test 16 of the 64 columns for every row and the partial words meet
// in LDS (the tests of one row are independent, so the bits are those of a serial scan).
// This pass covers row blocks [rb0, rb1) (sorted rows [64*rb0, 64*rb1)) x column blocks >= rb.
__global__ __launch_bounds__(256) void pp_mask(int A, double thr, int agnostic, long long vanilla_numel,
                                               PPWork w, int rb0, int rb1) {
    __shared__ Box cols[64];
    __shared__ unsigned long long part[4][64];
    const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = w.cnt[b];
    const int nb = (n + 63) / 64;
    rb1 = min(rb1, nb);
    if (rb0 >= rb1) return;
    const int mode = image_mode(n, agnostic, vanilla_numel);
    const float step = w.maxc[b] + 1.0f;
    const int nr = nb - rb0;  // column blocks of the pass's first row block
    // row block rb0 + k holds nr - k pairs; S(k) = pairs of the first k row blocks
    auto S = [nr](long long k) { return k * nr - k * (k - 1) / 2; };
    const long long pairs = S(rb1 - rb0);
    const float* srt = w.srt + (long long)b * A * kRow;
    for (long long pi = blockIdx.x; pi < pairs; pi += gridDim.x) {
        const double q = 2.0 * nr + 1.0;
        int k = (int)((q - sqrt(q * q - 8.0 * (double)pi)) * 0.5);
        k = max(0, min(k, rb1 - rb0 - 1));
        while (k > 0 && S(k) > pi) --k;
        while (k + 1 < rb1 - rb0 && S(k + 1) <= pi) ++k;
        const int rb = rb0 + k;
        const int cb = rb + (int)(pi - S(k));
        __syncthreads();
        if (tid < 64 && cb * 64 + tid < n) cols[tid] = load_box(srt + (long long)(cb * 64 + tid) * kRow, mode, step);
        __syncthreads();
        const int i = rb * 64 + lane;
        unsigned long long bits = 0;
        if (i < n) {
            const Box bi = load_box(srt + (long long)i * kRow, mode, step);
            const int jn = min(64, n - cb * 64);
            for (int t = wv * 16; t < min(jn, wv * 16 + 16); ++t) {
                const int jj = cb * 64 + t;
                if (jj <= i) continue;
                const Box& bj = cols[t];
                if (mode == 2 && bj.cls != bi.cls) continue;
                if (suppresses(bi, bj, thr)) bits |= 1ull << t;
            }
        }
        part[wv][lane] = bits;
        __syncthreads();
        if (tid < 64 && i < n)
            w.mask[((long long)b * w.cap + (i - rb0 * 64)) * w.capw + cb] =
                part[0][lane] | part[1][lane] | part[2][lane] | part[3][lane];
    }
}

// Greedy NMS over the sorted boxes, one wave per image, 64 boxes per step: the
// removed-set words live in LDS; within a 64-box block the keep decisions are a
// register-only scan over the block's diagonal mask words (one coalesced load),
// then every kept lane ORs its own mask row into the later words (independent
// loads across lanes) -- no dependent global load per kept box.  One launch per pass
// (row blocks [rb0, rb1)): the removed set and the keep count continue from the
// previous pass through the workspace / ``counts``.
// last: the final pass, which also zeroes the image's filter counter for the workspace's next call
// (one wave: its load of the counter above precedes the store in program order), and an image
// without candidates gets its count here (yxh_postprocess_scored skips pp_init).
__global__ __launch_bounds__(64) void pp_reduce(int A, PPWork w, float* det, int* counts, int rb0, int rb1, int last) {
    extern __shared__ unsigned long long removed[];  // [capw]
    const int b = blockIdx.x, lane = threadIdx.x;
    const int n = w.cnt[b];
    const int nw = (n + 63) / 64;
    if (rb0 == 0 && n == 0 && lane == 0) counts[b] = 0;
    rb1 = min(rb1, nw);
    if (rb0 >= rb1) {
        if (last && lane == 0) w.cnt[b] = 0;
        return;
    }
    unsigned long long* gremoved = w.removed + (long long)b * w.capw;
    for (int q = lane; q < nw; q += 64) removed[q] = rb0 == 0 ? 0ull : gremoved[q];
    __syncthreads();
    const float* srt = w.srt + (long long)b * A * kRow;
    // pass-local mask rows: sorted row i is row i - 64*rb0 of this pass
    const unsigned long long* pass = w.mask + (long long)b * w.cap * w.capw;
    auto mword = [&](int row, int col) { return pass[(long long)(row - rb0 * 64) * w.capw + col]; };
    float* out = det + (long long)b * A * 7;
    int nk = rb0 == 0 ? 0 : counts[b];
    // the diagonal word of block blk + 1 is loaded while block blk is scanned
    unsigned long long diag_next = rb0 * 64 + lane < n ? mword(rb0 * 64 + lane, rb0) : 0ull;
    for (int blk = rb0; blk < rb1; ++blk) {
        const int row = blk * 64 + lane;
        const int cnt = min(64, n - blk * 64);
        const unsigned long long diag = diag_next;
        diag_next = (blk + 1 < rb1 && row + 64 < n) ? mword(row + 64, blk + 1) : 0ull;
        unsigned long long cur = removed[blk];
        unsigned long long kept = 0;
        for (int t = 0; t < cnt; ++t) {
            if (!((cur >> t) & 1ull)) {
                kept |= 1ull << t;
                const unsigned int lo = __builtin_amdgcn_readlane((unsigned int)diag, t);
                const unsigned int hi = __builtin_amdgcn_readlane((unsigned int)(diag >> 32), t);
                cur |= ((unsigned long long)hi << 32) | lo;
            }
        }
        const bool mine = (kept >> lane) & 1ull;
        if (mine) {
            const int pos = nk + __popcll(kept & ((1ull << lane) - 1ull));
            const float* s = srt + (long long)row * kRow;
            float* o = out + (long long)pos * 7;
#pragma unroll
            for (int c = 0; c < 7; ++c) o[c] = s[c];
            for (int q = blk + 1; q < nw; ++q) {
                const unsigned long long v = mword(row, q);
                if (v) atomicOr(&removed[q], v);
            }
        }
        nk += __popcll(kept);
        __syncthreads();
    }
    if (rb1 < nw)  // a later pass continues from here
        for (int q = lane; q < nw; q += 64) gremoved[q] = removed[q];
    if (lane == 0) {
        counts[b] = nk;
        if (last) w.cnt[b] = 0;
    }
}

// Sorted rows per mask pass: a multiple of 64, all rows at once when the budget allows.
int pp_rows_per_pass(int B, int A) {
    const size_t capw = ((size_t)A + 63) / 64;
    const size_t all = capw * 64;
    size_t r = g_mask_budget / ((size_t)B * capw * 8) / 64 * 64;
    if (r < 64) r = 64;
    return (int)(r < all ? r : all);
}

void pp_set_mask_budget(size_t bytes) { g_mask_budget = bytes ? bytes : kMaskBudget; }

size_t pp_workspace(int B, int A) {
    const size_t cap = (size_t)pp_rows_per_pass(B, A);
    const size_t capw = ((size_t)A + 63) / 64;
    size_t s = 0;
    auto add = [&](size_t bytes) { s += (bytes + 255) & ~(size_t)255; };
    add(sizeof(int) * B);
    add(sizeof(float) * B);
    add(sizeof(int) * (size_t)B * A);
    add(sizeof(unsigned long long) * (size_t)B * A);
    add(sizeof(float) * kRow * (size_t)B * A);
    add(sizeof(float) * kRow * (size_t)B * A);
    add(sizeof(unsigned long long) * (size_t)B * cap * capw);
    add(sizeof(unsigned long long) * (size_t)B * A);  // merge ping-pong keys
    add(sizeof(unsigned long long) * (size_t)B * capw);  // removed set between passes
    return s;
}

// rest: the stream of the passes after the filter (sort, gather, mask, reduce); nullptr = st.  With a
// separate rest stream, filter_done (required) is recorded on st after the filter and rest waits on it:
// a serving loop keeps the filter in order behind its forward and runs the NMS proper beside the next one.
int postprocess(float* pred, int B, int A, int C, float conf, double nms, int agnostic, long long vanilla_numel,
                float* det, int* counts, void* ws, size_t ws_bytes, hipStream_t st, hipEvent_t filter_done,
                hipStream_t rest, const float* scores) {
    YXH_CHECK_ARG(!rest || rest == st || filter_done, "a separate rest stream needs the filter_done event");
    YXH_CHECK_ARG(pred && det && counts, "null pointer");
    YXH_CHECK_ARG(B > 0 && A >= 0 && C > 0, "postprocess shape B=%d A=%d C=%d", B, A, C);
    YXH_CHECK_ARG(ws && ws_bytes >= pp_workspace(B, A), "workspace too small (%zu < %zu)", ws_bytes,
                  pp_workspace(B, A));
    const size_t lds = (size_t)64 * (5 + C) * sizeof(float);
    YXH_CHECK_ARG(lds <= 64 * 1024, "too many classes for the filter tile");
    PPWork w;
    char* p = (char*)ws;
    auto take = [&](size_t bytes) {
        void* r = p;
        p += (bytes + 255) & ~(size_t)255;
        return r;
    };
    YXH_CHECK_ARG(A <= kMaxAnchors, "postprocess supports at most %d anchors per image (got %d)", kMaxAnchors, A);
    w.cap = pp_rows_per_pass(B, A);
    w.capw = (A + 63) / 64;
    w.cnt = (int*)take(sizeof(int) * B);
    w.maxc = (float*)take(sizeof(float) * B);
    w.slot_of = (int*)take(sizeof(int) * (size_t)B * A);
    w.key = (unsigned long long*)take(sizeof(unsigned long long) * (size_t)B * A);
    w.cand = (float*)take(sizeof(float) * kRow * (size_t)B * A);
    w.srt = (float*)take(sizeof(float) * kRow * (size_t)B * A);
    w.mask = (unsigned long long*)take(sizeof(unsigned long long) * (size_t)B * w.cap * w.capw);
    unsigned long long* key2 = (unsigned long long*)take(sizeof(unsigned long long) * (size_t)B * A);
    w.removed = (unsigned long long*)take(sizeof(unsigned long long) * (size_t)B * w.capw);
    // the counters are zero on entry to the scored path: the final reduce pass of every call leaves
    // them so, and a fresh workspace is zero-filled (yxh_postprocess_scored's contract)
    if (!scores || A == 0) {
        hipLaunchKernelGGL(pp_init, dim3(1), dim3(256), 0, st, B, w.cnt, counts);
        YXH_CHECK_LAUNCH("pp_init");
    }
    int rc = YXH_OK;
    if (A > 0 && scores) {
        hipLaunchKernelGGL(pp_filter_scored, dim3((A + 255) / 256, B), dim3(256), 0, st, pred, (const float4*)scores, A, C,
                           conf, w);
        YXH_CHECK_LAUNCH("pp_filter_scored");
    } else if (A > 0) {
        hipLaunchKernelGGL(pp_filter, dim3((A + 63) / 64, B), dim3(256), lds, st, pred, A, C, conf, w);
        YXH_CHECK_LAUNCH("pp_filter");
    }
    if (filter_done) {  // pred is read and rewritten only by the filter
        rc = check_hip(hipEventRecord(filter_done, st), "record filter_done");
        if (rc) return rc;
    }
    if (rest && rest != st) {  // counts (pp_init) and the filter's workspace rows are rest's inputs
        rc = check_hip(hipStreamWaitEvent(rest, filter_done, 0), "rest stream wait");
        if (rc) return rc;
        st = rest;
    }
    if (A == 0) return YXH_OK;
    const int nch = (A + kSortCap - 1) / kSortCap;
    hipLaunchKernelGGL(pp_sort_chunk, dim3(nch, B), dim3(1024), 0, st, A, w);
    YXH_CHECK_LAUNCH("pp_sort_chunk");
    unsigned long long* cur = w.key;
    unsigned long long* nxt = key2;
    for (int L = kSortCap; L < A; L *= 2) {
        hipLaunchKernelGGL(pp_merge, dim3((A + 255) / 256, B), dim3(256), 0, st, A, w, L, cur, nxt);
        YXH_CHECK_LAUNCH("pp_merge");
        unsigned long long* t = cur;
        cur = nxt;
        nxt = t;
    }
    hipLaunchKernelGGL(pp_gather, dim3(B), dim3(1024), 0, st, A, w, (const unsigned long long*)cur);
    YXH_CHECK_LAUNCH("pp_gather");
    const int rbp = w.cap / 64;  // row blocks per pass
    for (int rb0 = 0; rb0 < w.capw; rb0 += rbp) {
        // worst-case pairs of this pass (n = A): rbp row blocks x up to capw - rb0 column blocks
        const long long worst = (long long)rbp * (w.capw - rb0);
        // blocks per image (pairs dealt round-robin): at conf 0.5 an image of the bench keeps ~1 000
        // candidates = ~150 64 x 64 pairs, so fewer blocks serialise them (64 per image measured
        // 49.7 vs 29.4 us per pass, profiles/r05/nms_r5n.txt)
        const int gx = (int)std::min<long long>(worst, std::max(128, 8192 / B));
        hipLaunchKernelGGL(pp_mask, dim3(gx, B), dim3(256), 0, st, A, nms, agnostic, vanilla_numel, w, rb0,
                           rb0 + rbp);
        YXH_CHECK_LAUNCH("pp_mask");
        hipLaunchKernelGGL(pp_reduce, dim3(B), dim3(64), (size_t)w.capw * 8, st, A, w, det, counts, rb0, rb0 + rbp,
                           rb0 + rbp >= w.capw ? 1 : 0);
        YXH_CHECK_LAUNCH("pp_reduce");
    }
    return YXH_OK;
}

}  // namespace yxh
