/*
 * ORACLE -- test infrastructure only.  Never linked into, called by, or measured as
 * the product.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it.
 *
 * Plain-C restatement of the reference's post-processing on the CPU:
 *
 *   yolox/utils/boxes.py:31-75  postprocess(prediction, num_classes, conf_thre,
 *                                            nms_thre, class_agnostic)
 *     :32-37  cxcywh -> xyxy written back INTO prediction[..., :4]
 *     :46     class_conf, class_pred = max(cls, 1)   (first index of the max)
 *     :48     keep obj * class_conf >= conf_thre      (fp32 product, fp32 compare:
 *             torch casts the Python scalar to the tensor dtype)
 *     :50     det = [x1, y1, x2, y2, obj, class_conf, (float)class_pred]
 *     :56-67  torchvision.ops.nms / batched_nms(det[:, :4], obj*cls, cls_idx, nms_thre)
 *
 * torchvision is a third-party dependency absent from /root/reference (pinned at
 * torchvision 0.17.2, reference poetry.lock:2084-2085; not vendored).  Its published
 * algorithm is restated:
 *   nms (csrc/ops/cpu/nms_kernel.cpp): order = stable sort of scores, descending;
 *     areas = (x2-x1)*(y2-y1) (no +1); greedy over order: keep i, suppress j when
 *     inter / (area_i + area_j - inter) > iou_threshold, the fp32 IoU compared
 *     against the DOUBLE threshold.
 *   batched_nms (ops/boxes.py): if boxes.numel() > 4000 on CPU -> per-class vanilla
 *     nms, union, re-sort by score descending; else the coordinate trick:
 *     offsets = idx * (boxes.max() + 1), nms(boxes + offsets[:, None]).
 *     The trick changes the IoU's float rounding, so both branches are restated.
 *     The vanilla branch's final re-sort uses torch's (non-stable) CPU sort; ties in
 *     score are resolved here by ascending index (documented in DESIGN.md).
 *
 * Built with -ffp-contract=off and no fast-math so every fp32 operation rounds like
 * torch's element-wise CPU kernels.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    float score;
    int64_t idx;
} scored_t;

static int cmp_desc_stable(const void* a, const void* b) {
    const scored_t* x = (const scored_t*)a;
    const scored_t* y = (const scored_t*)b;
    if (x->score > y->score) return -1;
    if (x->score < y->score) return 1;
    return (x->idx < y->idx) ? -1 : (x->idx > y->idx);
}

static void sort_desc(const float* scores, int64_t n, int64_t* order) {
    scored_t* tmp = (scored_t*)malloc(sizeof(scored_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        tmp[i].score = scores[i];
        tmp[i].idx = i;
    }
    qsort(tmp, (size_t)n, sizeof(scored_t), cmp_desc_stable);
    for (int64_t i = 0; i < n; ++i) order[i] = tmp[i].idx;
    free(tmp);
}

/* torchvision nms_kernel_impl<float>.  boxes [n,4] xyxy.  Returns #kept; keep[] in
 * descending-score order. */
int64_t oracle_nms(const float* boxes, const float* scores, int64_t n, double iou_threshold,
                   int64_t* keep) {
    if (n <= 0) return 0;
    float* areas = (float*)malloc(sizeof(float) * (size_t)n);
    int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    unsigned char* suppressed = (unsigned char*)calloc((size_t)n, 1);
    for (int64_t i = 0; i < n; ++i) {
        float w = boxes[4 * i + 2] - boxes[4 * i + 0];
        float h = boxes[4 * i + 3] - boxes[4 * i + 1];
        areas[i] = w * h;
    }
    sort_desc(scores, n, order);
    int64_t nk = 0;
    for (int64_t oi = 0; oi < n; ++oi) {
        int64_t i = order[oi];
        if (suppressed[i]) continue;
        keep[nk++] = i;
        float ix1 = boxes[4 * i + 0], iy1 = boxes[4 * i + 1];
        float ix2 = boxes[4 * i + 2], iy2 = boxes[4 * i + 3];
        float iarea = areas[i];
        for (int64_t oj = oi + 1; oj < n; ++oj) {
            int64_t j = order[oj];
            if (suppressed[j]) continue;
            float xx1 = ix1 > boxes[4 * j + 0] ? ix1 : boxes[4 * j + 0];
            float yy1 = iy1 > boxes[4 * j + 1] ? iy1 : boxes[4 * j + 1];
            float xx2 = ix2 < boxes[4 * j + 2] ? ix2 : boxes[4 * j + 2];
            float yy2 = iy2 < boxes[4 * j + 3] ? iy2 : boxes[4 * j + 3];
            float w = xx2 - xx1;
            float h = yy2 - yy1;
            if (!(w > 0.0f)) w = 0.0f; /* std::max(0, w): 0 when w <= 0 */
            if (!(h > 0.0f)) h = 0.0f;
            float inter = w * h;
            float denom = (iarea + areas[j]) - inter;
            float ovr = inter / denom;
            if ((double)ovr > iou_threshold) suppressed[j] = 1;
        }
    }
    free(areas);
    free(order);
    free(suppressed);
    return nk;
}

/* torchvision batched_nms with the CPU branch rule (numel > vanilla_numel_limit ->
 * per-class vanilla; otherwise coordinate trick).  idxs are the float class ids the
 * reference passes (det[:, 6]). */
int64_t oracle_batched_nms(const float* boxes, const float* scores, const float* idxs, int64_t n,
                           double iou_threshold, int64_t vanilla_numel_limit, int64_t* keep) {
    if (n <= 0) return 0;
    if (4 * n > vanilla_numel_limit) {
        unsigned char* keep_mask = (unsigned char*)calloc((size_t)n, 1);
        unsigned char* done = (unsigned char*)calloc((size_t)n, 1);
        float* sb = (float*)malloc(sizeof(float) * 4 * (size_t)n);
        float* ss = (float*)malloc(sizeof(float) * (size_t)n);
        int64_t* map = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
        int64_t* k = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
        for (int64_t s = 0; s < n; ++s) {
            if (done[s]) continue;
            float cls = idxs[s];
            int64_t m = 0;
            for (int64_t i = s; i < n; ++i) {
                if (idxs[i] == cls) {
                    done[i] = 1;
                    memcpy(sb + 4 * m, boxes + 4 * i, 4 * sizeof(float));
                    ss[m] = scores[i];
                    map[m++] = i;
                }
            }
            int64_t nk = oracle_nms(sb, ss, m, iou_threshold, k);
            for (int64_t t = 0; t < nk; ++t) keep_mask[map[k[t]]] = 1;
        }
        int64_t nk = 0;
        for (int64_t i = 0; i < n; ++i)
            if (keep_mask[i]) map[nk++] = i;
        for (int64_t t = 0; t < nk; ++t) ss[t] = scores[map[t]];
        sort_desc(ss, nk, k);
        for (int64_t t = 0; t < nk; ++t) keep[t] = map[k[t]];
        free(keep_mask); free(done); free(sb); free(ss); free(map); free(k);
        return nk;
    }
    float maxc = boxes[0];
    for (int64_t i = 1; i < 4 * n; ++i)
        if (boxes[i] > maxc) maxc = boxes[i];
    float step = maxc + 1.0f;
    float* shifted = (float*)malloc(sizeof(float) * 4 * (size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        float off = idxs[i] * step;
        for (int c = 0; c < 4; ++c) shifted[4 * i + c] = boxes[4 * i + c] + off;
    }
    int64_t nk = oracle_nms(shifted, scores, n, iou_threshold, keep);
    free(shifted);
    return nk;
}

/* boxes.py:32-37: cxcywh -> xyxy written back into pred[..., :4] (rows of D). */
void oracle_xyxy_inplace(float* pred, int64_t rows, int64_t D) {
    for (int64_t r = 0; r < rows; ++r) {
        float* p = pred + r * D;
        float cx = p[0], cy = p[1], w = p[2], h = p[3];
        float hw = w / 2.0f, hh = h / 2.0f;
        p[0] = cx - hw;
        p[1] = cy - hh;
        p[2] = cx + hw;
        p[3] = cy + hh;
    }
}

/* boxes.py:46-51 for one image whose rows are already xyxy: det rows
 * [x1,y1,x2,y2,obj,class_conf,class_pred] of the candidates, in anchor order. */
int64_t oracle_filter(const float* pred, int64_t A, int64_t C, float conf_thre, float* det) {
    const int64_t D = 5 + C;
    int64_t n = 0;
    for (int64_t a = 0; a < A; ++a) {
        const float* p = pred + a * D;
        float best = p[5];
        int64_t bi = 0;
        for (int64_t c = 1; c < C; ++c)
            if (p[5 + c] > best) { best = p[5 + c]; bi = c; }
        float sc = p[4] * best;
        if (!(sc >= conf_thre)) continue;
        float* d = det + 7 * n;
        d[0] = p[0]; d[1] = p[1]; d[2] = p[2]; d[3] = p[3];
        d[4] = p[4]; d[5] = best; d[6] = (float)bi;
        ++n;
    }
    return n;
}

/* utils.postprocess restated.  pred [B, A, 5+C] fp32 is modified in place (xyxy),
 * like the reference.  out_rows has room for B*A rows of 7 floats; rows for image b
 * start at out_rows + 7*A*b.  counts[b] = #detections (0 -> the reference's None). */
int oracle_postprocess(float* pred, int64_t B, int64_t A, int64_t C, float conf_thre,
                       double nms_thre, int class_agnostic, int64_t vanilla_numel_limit,
                       float* out_rows, int64_t* counts) {
    const int64_t D = 5 + C;
    const size_t cap = (size_t)(A > 0 ? A : 1);
    oracle_xyxy_inplace(pred, B * A, D);
    float* det = (float*)malloc(sizeof(float) * 7 * cap);
    float* boxes = (float*)malloc(sizeof(float) * 4 * cap);
    float* scores = (float*)malloc(sizeof(float) * cap);
    float* idxs = (float*)malloc(sizeof(float) * cap);
    int64_t* keep = (int64_t*)malloc(sizeof(int64_t) * cap);
    for (int64_t b = 0; b < B; ++b) {
        int64_t n = oracle_filter(pred + b * A * D, A, C, conf_thre, det);
        for (int64_t i = 0; i < n; ++i) {
            memcpy(boxes + 4 * i, det + 7 * i, 4 * sizeof(float));
            scores[i] = det[7 * i + 4] * det[7 * i + 5];
            idxs[i] = det[7 * i + 6];
        }
        int64_t nk;
        if (class_agnostic)
            nk = oracle_nms(boxes, scores, n, nms_thre, keep);
        else
            nk = oracle_batched_nms(boxes, scores, idxs, n, nms_thre, vanilla_numel_limit, keep);
        for (int64_t t = 0; t < nk; ++t)
            memcpy(out_rows + 7 * (A * b + t), det + 7 * keep[t], 7 * sizeof(float));
        counts[b] = nk;
    }
    free(det); free(boxes); free(scores); free(idxs); free(keep);
    return 0;
}
