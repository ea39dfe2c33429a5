// SimOTA label assignment + YOLOX losses on gfx950 -- reference
// yolox/models/yolo_head.py:253-574 (get_losses, get_assignments,
// get_geometry_constraint, simota_matching), losses.py:13-51 (IouLoss).
//
// The reference runs a Python loop over images and, inside it, over ground truths
// with several host syncs per image.  Here the whole batch is six launches with no
// host sync:
//   sim_flags      : thread per anchor.  Centre-radius geometry (strict > 0 against
//                    +-1.5 strides) and, for anchors inside any GT's radius,
//                    S1 = sum_c -max(log(1 - p_c), -100) with p = sqrt(sig(cls)*sig(obj)).
//   sim_candidates : block per image: ordered compaction of the flagged anchors (the
//                    reference's anchor_filter order) with their S1.
//   sim_match      : block per (image, GT).  IoU + cost for every candidate
//                    (cls cost = S1 - term(1-p_k) + term(p_k): torch's clamped BCE of the
//                    one-hot target), dynamic_k = max(1, int(sum of the top-10 IoUs)),
//                    the dynamic_k smallest costs (ties -> lower candidate index).
//   sim_resolve    : per candidate.  Anchors matched by >1 GT keep the first argmin
//                    cost over all GTs; fg mask, matched GT, pred IoU, num_fg.
//   sim_loss       : per anchor partial sums (IoU^2 loss on fg, BCE-with-logits obj on
//                    all, cls on fg with target onehot * IoU, optional L1), reduced in a
//                    fixed order (deterministic), divided by max(sum num_fg, 1).
#pragma clang fp contract(off)  // IoU / cost formulas round like torch's separate ops

#include "yxh_common.hpp"

namespace yxh {

constexpr int kSimThreads = 256;

struct SimWork {
    int* ncand;       // [B]
    int* cand;        // [B][A] anchor index of candidate j
    float* s1;        // [B][A] class-cost base sum per candidate
    float* cost;      // [B][L][A]
    float* iou;       // [B][L][A]
    int* nmatch;      // [B][A] matches per candidate
    int* lastg;       // [B][A] a GT that matched it
    float* partial;   // [B][nblk][4]
    float* s1a;       // [B][A] class-cost base sum per anchor (flagged anchors only)
    uint8_t* flag;    // [B][A] anchor inside some GT's centre radius
};

struct SimGeom {
    int nlev;
    int lh[4], lw[4], stride[4], off[5];
};

__device__ __forceinline__ void anchor_geom(const SimGeom& g, int a, float& xs, float& ys, float& st) {
    int l = 0;
    while (l + 1 < g.nlev && a >= g.off[l + 1]) ++l;
    const int r = a - g.off[l];
    const int y = r / g.lw[l], x = r - y * g.lw[l];
    xs = (float)x;
    ys = (float)y;
    st = (float)g.stride[l];
}

// get_geometry_constraint (yolo_head.py:511-540), same fp32 operation order
__device__ __forceinline__ bool in_center(const float* gt, float xs, float ys, float st) {
    const float xc = (xs + 0.5f) * st, yc = (ys + 0.5f) * st;
    const float cd = st * 1.5f;
    const float gl = gt[0] - cd, gr = gt[0] + cd, gtp = gt[1] - cd, gb = gt[1] + cd;
    const float cl = xc - gl, ct = yc - gtp, cr = gr - xc, cb = gb - yc;
    return fminf(fminf(cl, ct), fminf(cr, cb)) > 0.0f;
}

__device__ __forceinline__ int num_labels(const float* lab, int L) {
    int n = 0;
    for (int i = 0; i < L; ++i) {
        const float* r = lab + 5 * i;
        const float s = (((r[0] + r[1]) + r[2]) + r[3]) + r[4];
        n += s > 0.0f;
    }
    return n;
}

__device__ __forceinline__ float clamped_log(float v) { return fmaxf(logf(v), -100.0f); }

__device__ __forceinline__ float sig(float x) { return 1.0f / (1.0f + expf(-x)); }

// bboxes_iou(xyxy=False) for one pair (utils/boxes.py:78-101 operation order)
__device__ __forceinline__ float iou_cxcywh(const float* a, const float* b) {
    const float tlx = fmaxf(a[0] - a[2] / 2, b[0] - b[2] / 2);
    const float tly = fmaxf(a[1] - a[3] / 2, b[1] - b[3] / 2);
    const float brx = fminf(a[0] + a[2] / 2, b[0] + b[2] / 2);
    const float bry = fminf(a[1] + a[3] / 2, b[1] + b[3] / 2);
    const float area_a = a[2] * a[3], area_b = b[2] * b[3];
    const float en = (tlx < brx && tly < bry) ? 1.0f : 0.0f;
    const float area_i = ((brx - tlx) * (bry - tly)) * en;
    return area_i / ((area_a + area_b) - area_i);
}

// One thread per anchor: the 80 class-logit reads of different anchors are independent,
// so thousands are in flight instead of one image's block walking them chunk by chunk.
// Per-step initialisation of the assignment outputs and the match counters (one launch;
// replaces five memset nodes, so a captured training step has only kernel nodes here).
__global__ __launch_bounds__(256) void sim_init(int BA, int B, int* nmatch, uint8_t* fg, int* matched, float* piou,
                                                int* num_fg) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < BA) {
        nmatch[i] = 0;
        fg[i] = 0;
        matched[i] = -1;
        piou[i] = 0.f;
    }
    if (i < B) num_fg[i] = 0;
}

__global__ __launch_bounds__(256) void sim_flags(const float* preds, const float* labels, int A, int C, int L,
                                                 SimGeom geo, SimWork w) {
    const int b = blockIdx.y, a = blockIdx.x * 256 + threadIdx.x;
    if (a >= A) return;
    const float* lab = labels + (long long)b * L * 5;
    const int G = num_labels(lab, L);
    bool in = false;
    if (G > 0) {
        float xs, ys, st;
        anchor_geom(geo, a, xs, ys, st);
        for (int g = 0; g < G && !in; ++g) in = in_center(lab + 5 * g + 1, xs, ys, st);
    }
    w.flag[(long long)b * A + a] = in ? 1 : 0;
    if (!in) return;
    const float* p = preds + ((long long)b * A + a) * (5 + C);
    const float so = sig(p[4]);
    float s1 = 0.0f;
    int c = 0;
    for (; c + 8 <= C; c += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[5 + c + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) s1 += -clamped_log(1.0f - sqrtf(sig(v[u]) * so));
    }
    for (; c < C; ++c) s1 += -clamped_log(1.0f - sqrtf(sig(p[5 + c]) * so));
    w.s1a[(long long)b * A + a] = s1;
}

__global__ __launch_bounds__(1024) void sim_candidates(int A, SimWork w) {
    __shared__ int wsum[16];
    __shared__ int base;
    const int b = blockIdx.x, tid = threadIdx.x;
    if (tid == 0) base = 0;
    __syncthreads();
    for (int a0 = 0; a0 < A; a0 += 1024) {
        const int a = a0 + tid;
        const bool in = a < A && w.flag[(long long)b * A + a];
        // ordered compaction: wave ballot + per-wave prefix
        const unsigned long long m = __ballot(in);
        const int lane = tid & 63, wv = tid >> 6;
        if (lane == 0) wsum[wv] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int i = 0; i < wv; ++i) off += wsum[i];
        const int pos = off + __popcll(m & ((1ull << lane) - 1ull));
        if (in) {
            w.cand[(long long)b * A + pos] = a;
            w.s1[(long long)b * A + pos] = w.s1a[(long long)b * A + a];
        }
        __syncthreads();
        if (tid == 0) {
            int t = 0;
            for (int i = 0; i < 16; ++i) t += wsum[i];
            base += t;
        }
        __syncthreads();
    }
    if (tid == 0) w.ncand[b] = base;
}

// block-wide (value, index) selection helpers
struct VI {
    float v;
    int i;
};

__device__ __forceinline__ bool better_max(VI a, VI b) { return a.v > b.v || (a.v == b.v && a.i < b.i); }
__device__ __forceinline__ bool better_min(VI a, VI b) { return a.v < b.v || (a.v == b.v && a.i < b.i); }

template <bool MAX>
__device__ VI block_select(VI x, VI* red) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int off = 32; off > 0; off >>= 1) {
        VI y;
        y.v = __shfl_xor(x.v, off);
        y.i = __shfl_xor(x.i, off);
        if (MAX ? better_max(y, x) : better_min(y, x)) x = y;
    }
    if (lane == 0) red[wv] = x;
    __syncthreads();
    VI r = red[0];
    for (int k = 1; k < kSimThreads / 64; ++k)
        if (MAX ? better_max(red[k], r) : better_min(red[k], r)) r = red[k];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(kSimThreads) void sim_match(const float* preds, const float* labels, int A, int C,
                                                          int L, SimGeom geo, SimWork w) {
    __shared__ VI red[kSimThreads / 64];
    __shared__ int selected[16];
    const int b = blockIdx.y, g = blockIdx.x, tid = threadIdx.x;
    const float* lab = labels + (long long)b * L * 5;
    const int G = num_labels(lab, L);
    if (g >= G) return;
    const int n = w.ncand[b];
    if (n == 0) return;
    const int D = 5 + C;
    const float* gt = lab + 5 * g;
    const int k = (int)gt[0];
    float* crow = w.cost + ((long long)b * L + g) * A;
    float* irow = w.iou + ((long long)b * L + g) * A;
    for (int j = tid; j < n; j += kSimThreads) {
        const int a = w.cand[(long long)b * A + j];
        const float* p = preds + ((long long)b * A + a) * D;
        float xs, ys, st;
        anchor_geom(geo, a, xs, ys, st);
        const float io = iou_cxcywh(gt + 1, p);
        const float pk = sqrtf(sig(p[5 + k]) * sig(p[4]));
        const float cls_cost = (w.s1[(long long)b * A + j] - (-clamped_log(1.0f - pk))) + (-clamped_log(pk));
        const float iou_cost = -logf(io + 1e-8f);
        const float geom = in_center(gt + 1, xs, ys, st) ? 0.0f : 1.0f;
        crow[j] = cls_cost + 3.0f * iou_cost + 1e6f * geom;
        irow[j] = io;
    }
    __syncthreads();
    // dynamic k: int(sum of the top-min(10, n) IoUs), at least 1
    const int ncand = min(10, n);
    float topsum = 0.0f;
    for (int r = 0; r < ncand; ++r) {
        VI best{-INFINITY, 0x7fffffff};
        for (int j = tid; j < n; j += kSimThreads) {
            bool used = false;
            for (int q = 0; q < r; ++q) used |= selected[q] == j;
            VI c{irow[j], j};
            if (!used && better_max(c, best)) best = c;
        }
        VI s = block_select<true>(best, red);
        if (tid == 0) selected[r] = s.i;
        topsum += s.v;
        __syncthreads();
    }
    const int dk = max(1, (int)topsum);
    for (int r = 0; r < dk && r < n; ++r) {
        VI best{INFINITY, 0x7fffffff};
        for (int j = tid; j < n; j += kSimThreads) {
            bool used = false;
            for (int q = 0; q < r; ++q) used |= selected[q] == j;
            VI c{crow[j], j};
            if (!used && better_min(c, best)) best = c;
        }
        VI s = block_select<false>(best, red);
        if (tid == 0) {
            selected[r] = s.i;
            atomicAdd(&w.nmatch[(long long)b * A + s.i], 1);
            w.lastg[(long long)b * A + s.i] = g;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void sim_resolve(const float* labels, int A, int L, SimWork w,
                                                    uint8_t* fg, int* matched, float* piou, int* num_fg) {
    const int b = blockIdx.y;
    const int j = blockIdx.x * 256 + threadIdx.x;
    const int n = w.ncand[b];
    if (j >= n) return;
    const int cnt = w.nmatch[(long long)b * A + j];
    if (cnt == 0) return;
    const int a = w.cand[(long long)b * A + j];
    int g = w.lastg[(long long)b * A + j];
    if (cnt > 1) {
        const int G = num_labels(labels + (long long)b * L * 5, L);
        float best = INFINITY;
        for (int q = 0; q < G; ++q) {
            const float c = w.cost[((long long)b * L + q) * A + j];
            if (c < best) {
                best = c;
                g = q;
            }
        }
    }
    fg[(long long)b * A + a] = 1;
    matched[(long long)b * A + a] = g;
    piou[(long long)b * A + a] = w.iou[((long long)b * L + g) * A + j];
    atomicAdd(&num_fg[b], 1);
}

__device__ __forceinline__ float bce_logits(float x, float t) {
    // torch binary_cross_entropy_with_logits (no weights), CPU formulation
    const float m = fmaxf(-x, 0.0f);
    return (1.0f - t) * x + m + logf(expf(-m) + expf(-x - m));
}

// partial[b][blk][4] = (iou, obj, cls, l1) sums over this block's anchors
__global__ __launch_bounds__(256) void sim_loss(const float* preds, const float* origin, const float* labels,
                                                 int A, int C, int L, SimGeom geo, const uint8_t* fg,
                                                 const int* matched, const float* piou, float* partial) {
    __shared__ float red[4][256];
    const int b = blockIdx.y, tid = threadIdx.x;
    const int a = blockIdx.x * 256 + tid;
    const int D = 5 + C;
    float li = 0.f, lo = 0.f, lc = 0.f, l1 = 0.f;
    if (a < A) {
        const float* p = preds + ((long long)b * A + a) * D;
        const bool f = fg[(long long)b * A + a];
        lo = bce_logits(p[4], f ? 1.0f : 0.0f);
        if (f) {
            const int g = matched[(long long)b * A + a];
            const float* gt = labels + ((long long)b * L + g) * 5;
            const float tlx = fmaxf(p[0] - p[2] / 2, gt[1] - gt[3] / 2);
            const float tly = fmaxf(p[1] - p[3] / 2, gt[2] - gt[4] / 2);
            const float brx = fminf(p[0] + p[2] / 2, gt[1] + gt[3] / 2);
            const float bry = fminf(p[1] + p[3] / 2, gt[2] + gt[4] / 2);
            const float area_p = p[2] * p[3], area_g = gt[3] * gt[4];
            const float en = (tlx < brx && tly < bry) ? 1.0f : 0.0f;
            const float area_i = ((brx - tlx) * (bry - tly)) * en;
            const float io = area_i / (((area_p + area_g) - area_i) + 1e-16f);
            li = 1.0f - io * io;
            const int k = (int)gt[0];
            const float t = piou[(long long)b * A + a];
            for (int c = 0; c < C; ++c) lc += bce_logits(p[5 + c], c == k ? t : 0.0f);
            if (origin) {
                float xs, ys, st;
                anchor_geom(geo, a, xs, ys, st);
                const float* o = origin + ((long long)b * A + a) * 4;
                const float t0 = gt[1] / st - xs, t1 = gt[2] / st - ys;
                const float t2 = logf(gt[3] / st + 1e-8f), t3 = logf(gt[4] / st + 1e-8f);
                l1 = fabsf(o[0] - t0) + fabsf(o[1] - t1) + fabsf(o[2] - t2) + fabsf(o[3] - t3);
            }
        }
    }
    red[0][tid] = li;
    red[1][tid] = lo;
    red[2][tid] = lc;
    red[3][tid] = l1;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s)
            for (int q = 0; q < 4; ++q) red[q][tid] += red[q][tid + s];
        __syncthreads();
    }
    if (tid < 4) partial[((long long)b * gridDim.x + blockIdx.x) * 4 + tid] = red[tid][0];
}

__global__ void sim_finalize(const float* partial, int nparts, const int* num_fg, const float* labels, int B, int L,
                             int use_l1, float* losses) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double s[4] = {0, 0, 0, 0};
    for (int i = 0; i < nparts; ++i)
        for (int q = 0; q < 4; ++q) s[q] += partial[4 * i + q];
    float nfg = 0.0f, ngt = 0.0f;
    for (int b = 0; b < B; ++b) {
        nfg += (float)num_fg[b];
        ngt += (float)num_labels(labels + (long long)b * L * 5, L);
    }
    const float d = fmaxf(nfg, 1.0f);
    const float li = (float)s[0] / d, lo = (float)s[1] / d, lc = (float)s[2] / d;
    const float l1 = use_l1 ? (float)s[3] / d : 0.0f;
    losses[0] = 5.0f * li + lo + lc + l1;  // total_loss
    losses[1] = 5.0f * li;                 // iou_loss (reg_weight * loss_iou)
    losses[2] = lo;                        // conf_loss
    losses[3] = lc;                        // cls_loss
    losses[4] = l1;                        // l1_loss
    losses[5] = d / fmaxf(ngt, 1.0f);      // num_fg / max(num_gts, 1)
}


// get_output_and_grid (yolo_head.py:213-231) on raw pred-conv outputs
__global__ __launch_bounds__(256) void head_decode_train(const float* raw, int B, int A, int D, SimGeom geo,
                                                        float* out) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)B * A * D) return;
    const int ch = (int)(idx % D);
    const int a = (int)((idx / D) % A);
    float v = raw[idx];
    if (ch < 4) {
        float xs, ys, st;
        anchor_geom(geo, a, xs, ys, st);
        v = ch < 2 ? (v + (ch == 0 ? xs : ys)) * st : expf(v) * st;
    }
    out[idx] = v;
}

__device__ __forceinline__ float tie_w(float a, float b, bool want_greater) {
    // torch.maximum / minimum backward: full gradient to the selected input, half on ties
    if (a == b) return 0.5f;
    return (want_greater ? a > b : a < b) ? 1.0f : 0.0f;
}

__device__ __forceinline__ float sgn(float v) { return v > 0.0f ? 1.0f : (v < 0.0f ? -1.0f : 0.0f); }

// d total_loss / d raw outputs (autograd of yolo_head.py:382-402 + losses.py:13-51 through
// the decode of :227-230); one thread per anchor.
template <typename T>
__global__ __launch_bounds__(256) void sim_loss_bwd(const float* preds, const float* raw, const float* labels, int B,
                                                    int A, int C, int L, SimGeom geo, const uint8_t* fg,
                                                    const int* matched, const float* piou, const int* num_fg,
                                                    const float* gtot, int use_l1, T* g_ro, T* g_cls) {
    const int b = blockIdx.y, a = blockIdx.x * 256 + threadIdx.x;
    if (a >= A) return;
    int nfg = 0;
    for (int q = 0; q < B; ++q) nfg += num_fg[q];
    const float gs = gtot[0] / fmaxf((float)nfg, 1.0f);
    const long long row = (long long)b * A + a;
    const int D = 5 + C;
    const float* p = preds + row * D;
    const float* r = raw + row * D;
    const bool f = fg[row];
    float gr[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    gr[4] = (sig(r[4]) - (f ? 1.0f : 0.0f)) * gs;
    T* gc = g_cls + row * C;
    if (!f) {
        for (int c = 0; c < C; ++c) gc[c] = from_f32<T>(0.0f);
    } else {
        const int g = matched[row];
        const float* gt = labels + ((long long)b * L + g) * 5;
        const int k = (int)gt[0];
        const float t = piou[row];
        for (int c = 0; c < C; ++c) gc[c] = from_f32<T>((sig(r[5 + c]) - (c == k ? t : 0.0f)) * gs);
        // IoU loss (reg_weight 5): L = 1 - iou^2
        const float px = p[0], py = p[1], pw = p[2], ph = p[3];
        const float atx = px - pw / 2, btx = gt[1] - gt[3] / 2, aty = py - ph / 2, bty = gt[2] - gt[4] / 2;
        const float abx = px + pw / 2, bbx = gt[1] + gt[3] / 2, aby = py + ph / 2, bby = gt[2] + gt[4] / 2;
        const float tlx = fmaxf(atx, btx), tly = fmaxf(aty, bty), brx = fminf(abx, bbx), bry = fminf(aby, bby);
        const float en = (tlx < brx && tly < bry) ? 1.0f : 0.0f;
        const float dxx = brx - tlx, dyy = bry - tly;
        const float ai = (dxx * dyy) * en;
        const float ap = pw * ph, ag = gt[3] * gt[4];
        const float u = ((ap + ag) - ai) + 1e-16f;
        const float io = ai / u;
        const float gi = 5.0f * gs * (-2.0f * io);
        const float gu = -gi * ai / (u * u);
        const float gai = gi / u - gu;
        const float gap = gu;
        const float gdx = gai * en * dyy, gdy = gai * en * dxx;
        const float gtlx = -gdx * tie_w(atx, btx, true), gbrx = gdx * tie_w(abx, bbx, false);
        const float gtly = -gdy * tie_w(aty, bty, true), gbry = gdy * tie_w(aby, bby, false);
        const float gpx = gtlx + gbrx, gpy = gtly + gbry;
        const float gpw = 0.5f * (gbrx - gtlx) + gap * ph;
        const float gph = 0.5f * (gbry - gtly) + gap * pw;
        float xs, ys, st;
        anchor_geom(geo, a, xs, ys, st);
        gr[0] = gpx * st;
        gr[1] = gpy * st;
        gr[2] = gpw * st * expf(r[2]);
        gr[3] = gph * st * expf(r[3]);
        if (use_l1) {
            const float t0 = gt[1] / st - xs, t1 = gt[2] / st - ys;
            const float t2 = logf(gt[3] / st + 1e-8f), t3 = logf(gt[4] / st + 1e-8f);
            gr[0] += sgn(r[0] - t0) * gs;
            gr[1] += sgn(r[1] - t1) * gs;
            gr[2] += sgn(r[2] - t2) * gs;
            gr[3] += sgn(r[3] - t3) * gs;
        }
    }
    T o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = from_f32<T>(gr[q]);
    T* go = g_ro + row * 8;
#pragma unroll
    for (int q = 0; q < 8; ++q) go[q] = o[q];
}

// ------------------------------------------------------------------ host
static size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

static SimGeom make_geom(const int* lhw, const int* strides, int nlev) {
    SimGeom geo{};
    geo.nlev = nlev;
    geo.off[0] = 0;
    for (int l = 0; l < nlev; ++l) {
        geo.lh[l] = lhw[2 * l];
        geo.lw[l] = lhw[2 * l + 1];
        geo.stride[l] = strides[l];
        geo.off[l + 1] = geo.off[l] + geo.lh[l] * geo.lw[l];
    }
    return geo;
}

size_t sim_workspace(int B, int A, int L) {
    const int nblk = (A + 255) / 256;
    return al(sizeof(int) * B) + al(sizeof(int) * (size_t)B * A) + al(sizeof(float) * (size_t)B * A) +
           2 * al(sizeof(float) * (size_t)B * L * A) + 2 * al(sizeof(int) * (size_t)B * A) +
           al(sizeof(float) * 4 * (size_t)B * nblk) + al(sizeof(float) * (size_t)B * A) + al((size_t)B * A);
}

int yolox_loss(const float* preds, const float* origin, const float* labels, int B, int A, int C, int L,
               const int* lhw, const int* strides, int nlev, uint8_t* fg, int* matched, float* piou, int* num_fg,
               float* losses, void* ws, size_t ws_bytes, hipStream_t st) {
    YXH_CHECK_ARG(preds && labels && fg && matched && piou && num_fg && losses && lhw && strides, "null pointer");
    YXH_CHECK_ARG(B > 0 && A > 0 && C > 0 && L > 0 && nlev > 0 && nlev <= 4, "shape B=%d A=%d C=%d L=%d", B, A, C, L);
    YXH_CHECK_ARG(ws && ws_bytes >= sim_workspace(B, A, L), "workspace too small");
    SimGeom geo = make_geom(lhw, strides, nlev);
    YXH_CHECK_ARG(geo.off[nlev] == A, "level sizes sum to %d, not A=%d", geo.off[nlev], A);
    char* p = (char*)ws;
    auto take = [&](size_t bytes) {
        void* r = p;
        p += al(bytes);
        return r;
    };
    const int nblk = (A + 255) / 256;
    SimWork w;
    w.ncand = (int*)take(sizeof(int) * B);
    w.cand = (int*)take(sizeof(int) * (size_t)B * A);
    w.s1 = (float*)take(sizeof(float) * (size_t)B * A);
    w.cost = (float*)take(sizeof(float) * (size_t)B * L * A);
    w.iou = (float*)take(sizeof(float) * (size_t)B * L * A);
    w.nmatch = (int*)take(sizeof(int) * (size_t)B * A);
    w.lastg = (int*)take(sizeof(int) * (size_t)B * A);
    w.partial = (float*)take(sizeof(float) * 4 * (size_t)B * nblk);
    w.s1a = (float*)take(sizeof(float) * (size_t)B * A);
    w.flag = (uint8_t*)take((size_t)B * A);
    YXH_CHECK_ARG((long long)B * A < (1LL << 31), "B*A too large");
    const int BA = B * A;
    hipLaunchKernelGGL(sim_init, dim3((BA + 255) / 256), dim3(256), 0, st, BA, B, w.nmatch, fg, matched, piou, num_fg);
    YXH_CHECK_LAUNCH("sim_init");
    hipLaunchKernelGGL(sim_flags, dim3((A + 255) / 256, B), dim3(256), 0, st, preds, labels, A, C, L, geo, w);
    YXH_CHECK_LAUNCH("sim_flags");
    hipLaunchKernelGGL(sim_candidates, dim3(B), dim3(1024), 0, st, A, w);
    YXH_CHECK_LAUNCH("sim_candidates");
    hipLaunchKernelGGL(sim_match, dim3(L, B), dim3(kSimThreads), 0, st, preds, labels, A, C, L, geo, w);
    YXH_CHECK_LAUNCH("sim_match");
    hipLaunchKernelGGL(sim_resolve, dim3((A + 255) / 256, B), dim3(256), 0, st, labels, A, L, w, fg, matched, piou,
                       num_fg);
    YXH_CHECK_LAUNCH("sim_resolve");
    hipLaunchKernelGGL(sim_loss, dim3(nblk, B), dim3(256), 0, st, preds, origin, labels, A, C, L, geo, fg, matched,
                       piou, w.partial);
    YXH_CHECK_LAUNCH("sim_loss");
    hipLaunchKernelGGL(sim_finalize, dim3(1), dim3(64), 0, st, w.partial, B * nblk, num_fg, labels, B, L,
                       origin ? 1 : 0, losses);
    YXH_CHECK_LAUNCH("sim_finalize");
    return YXH_OK;
}


int head_decode_train_launch(const float* raw, int B, int A, int C, const int* lhw, const int* strides, int nlev,
                             float* out, hipStream_t st) {
    YXH_CHECK_ARG(raw && out && lhw && strides, "null pointer");
    YXH_CHECK_ARG(B > 0 && A > 0 && C > 0 && nlev > 0 && nlev <= 4, "shape");
    SimGeom geo = make_geom(lhw, strides, nlev);
    YXH_CHECK_ARG(geo.off[nlev] == A, "level sizes sum to %d, not A=%d", geo.off[nlev], A);
    const long long total = (long long)B * A * (5 + C);
    hipLaunchKernelGGL(head_decode_train, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, raw, B, A, 5 + C,
                       geo, out);
    YXH_CHECK_LAUNCH("head_decode_train");
    return YXH_OK;
}

int yolox_loss_bwd(const float* preds, const float* raw, const float* labels, int B, int A, int C, int L,
                   const int* lhw, const int* strides, int nlev, const uint8_t* fg, const int* matched,
                   const float* piou, const int* num_fg, const float* gtot, int use_l1, int dt, void* g_ro,
                   void* g_cls, hipStream_t st) {
    YXH_CHECK_ARG(preds && raw && labels && fg && matched && piou && num_fg && gtot && g_ro && g_cls && lhw && strides,
                  "null pointer");
    YXH_CHECK_ARG(B > 0 && A > 0 && C > 0 && L > 0 && nlev > 0 && nlev <= 4, "shape");
    SimGeom geo = make_geom(lhw, strides, nlev);
    YXH_CHECK_ARG(geo.off[nlev] == A, "level sizes sum to %d, not A=%d", geo.off[nlev], A);
    dim3 grid((A + 255) / 256, B);
#define YXH_LB(T)                                                                                                    \
    hipLaunchKernelGGL(sim_loss_bwd<T>, grid, dim3(256), 0, st, preds, raw, labels, B, A, C, L, geo, fg, matched,  \
                       piou, num_fg, gtot, use_l1, (T*)g_ro, (T*)g_cls)
    if (dt == YXH_BF16) YXH_LB(bf16);
    else if (dt == YXH_F16) YXH_LB(f16);
    else if (dt == YXH_F32) YXH_LB(float);
    else {
        set_error("loss_bwd dtype %d", dt);
        return YXH_EINVAL;
    }
#undef YXH_LB
    YXH_CHECK_LAUNCH("sim_loss_bwd");
    return YXH_OK;
}

}  // namespace yxh
