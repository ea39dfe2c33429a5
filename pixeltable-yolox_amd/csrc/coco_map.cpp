// COCO box-mAP engine (host C++): the evaluation the reference runs for its mAP numbers
// -- CocoEvaluator.evaluate_prediction (yolox/evaluators/coco_evaluator.py:253-315) ->
// CocoEvalOpt (yolox/layers/fast_coco_eval_api.py:24-149): pycocotools' computeIoU
// (bbox), the C++ EvaluateImages (yolox/layers/cocoeval/cocoeval.cpp:140-197) and
// Accumulate (:370-500).
//
// Layout: every (image, category) cell p = image * K + category owns the ground truths
// gts[gt_off[p], gt_off[p+1]) and detections dts[dt_off[p], dt_off[p+1]) (any order).
// One call does the whole evaluation:
//   1. per cell, detections are ordered by score (descending, stable) and cut to the
//      largest max-detections setting; box IoU of each kept detection with each ground
//      truth (bbIou: crowd ground truths use the detection's area as the union);
//   2. per (cell, area range): ground truths whose area is outside the range (or flagged
//      ignore) go last (stable); for each IoU threshold every detection, best score
//      first, takes the unmatched ground truth (crowds may be reused) with the highest
//      IoU >= min(thr, 1 - 1e-10), preferring regular over ignored ground truths;
//      unmatched detections outside the area range are ignored;
//   3. per (category, area range, max-dets): the first max-dets detections of every
//      image, ordered by score (stable, image-major ties), give cumulative TP / FP,
//      recall = TP / #valid GT, precision made monotone from the right and sampled at
//      each recall threshold (first recall >= threshold).
// Outputs are the arrays CocoEvalOpt.accumulate stores: precision / scores
// [T][R][K][A][M], recall [T][K][A][M], -1 where a setting has no valid ground truth.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>

#include "yoloxhip.h"

namespace yxh {
void set_error(const char* fmt, ...);
}

namespace {

struct Cell {  // one (image, category) after step 1
    std::vector<int32_t> det;  // score-ordered kept detection indices into dts
    std::vector<double> iou;   // [det.size()][G]
};

// pycocotools maskApi.c bbIou, bbox (x, y, w, h)
double box_iou(const yxh_coco_instance& d, const yxh_coco_instance& g) {
    const double w = std::min(d.box[0] + d.box[2], g.box[0] + g.box[2]) - std::max(d.box[0], g.box[0]);
    if (w <= 0) return 0.0;
    const double h = std::min(d.box[1] + d.box[3], g.box[1] + g.box[3]) - std::max(d.box[1], g.box[1]);
    if (h <= 0) return 0.0;
    const double inter = w * h;
    const double da = d.box[2] * d.box[3];
    const double uni = g.is_crowd ? da : da + g.box[2] * g.box[3] - inter;
    return inter / uni;
}

// Per (cell, area range, threshold) matching results, in score order.
struct Matches {
    std::vector<int64_t> match;        // [T][D] id of the matched ground truth, 0 = none
    std::vector<uint8_t> ignored;      // [T][D]
    std::vector<double> score;         // [D]
    int valid_gt = 0;
};

void match_cell(const yxh_coco_instance* gts, int G, const yxh_coco_instance* dts, const Cell& cell,
                const double* arng, const double* thr, int T, Matches& out) {
    const int D = (int)cell.det.size();
    // ground truths: regular first, then ignored (stable)
    std::vector<int32_t> order(G);
    std::vector<uint8_t> gign(G);
    for (int g = 0; g < G; ++g) gign[g] = gts[g].ignore || gts[g].area < arng[0] || gts[g].area > arng[1];
    int pos = 0;
    for (int pass = 0; pass < 2; ++pass)
        for (int g = 0; g < G; ++g)
            if (gign[g] == pass) order[pos++] = g;
    out.valid_gt = 0;
    for (int g = 0; g < G; ++g) out.valid_gt += !gign[g];
    out.match.assign((size_t)T * D, 0);
    out.ignored.assign((size_t)T * D, 0);
    out.score.resize(D);
    for (int d = 0; d < D; ++d) out.score[d] = dts[cell.det[d]].score;
    std::vector<int64_t> taken(G);  // id of the detection holding each ground truth, 0 = free
    for (int t = 0; t < T; ++t) {
        std::fill(taken.begin(), taken.end(), 0);
        const double floor_iou = std::min(thr[t], 1.0 - 1e-10);
        for (int d = 0; d < D; ++d) {
            const double* row = cell.iou.data() + (size_t)d * G;
            double best = floor_iou;
            int m = -1;  // position in `order`
            for (int k = 0; k < G; ++k) {
                const int g = order[k];
                if (taken[g] && !gts[g].is_crowd) continue;
                if (m >= 0 && !gign[order[m]] && gign[g]) break;  // only ignored ones remain
                if (row[g] >= best) {
                    best = row[g];
                    m = k;
                }
            }
            const yxh_coco_instance& det = dts[cell.det[d]];
            bool ign = false;
            int64_t id = 0;
            if (m >= 0) {
                const int g = order[m];
                taken[g] = det.id;
                ign = gign[g];
                id = gts[g].id;
            }
            // unmatched (or matched to ground truth id 0) detections outside the range
            if (id == 0 && (det.area < arng[0] || det.area > arng[1])) ign = true;
            out.match[(size_t)t * D + d] = id;
            out.ignored[(size_t)t * D + d] = ign;
        }
    }
}

}  // namespace

extern "C" int yxh_coco_eval(const yxh_coco_params* p, const yxh_coco_instance* gts, const int64_t* gt_off,
                             const yxh_coco_instance* dts, const int64_t* dt_off, double* precision, double* recall,
                             double* scores) {
    if (!p || !gt_off || !dt_off || !precision || !recall || !scores || p->num_images < 0 ||
        p->num_categories <= 0 || p->num_area_ranges <= 0 || p->num_iou_thresholds <= 0 ||
        p->num_recall_thresholds <= 0 || p->num_max_dets <= 0 || !p->area_ranges || !p->iou_thresholds ||
        !p->recall_thresholds || !p->max_dets) {
        yxh::set_error("coco_eval: bad parameters");
        return YXH_EINVAL;
    }
    const int I = p->num_images, K = p->num_categories, A = p->num_area_ranges, T = p->num_iou_thresholds;
    const int R = p->num_recall_thresholds, M = p->num_max_dets;
    int maxdet = 0;
    for (int m = 0; m < M; ++m) maxdet = std::max(maxdet, p->max_dets[m]);
    // step 1: score order, cut, IoU
    std::vector<Cell> cells((size_t)I * K);
    for (size_t c = 0; c < cells.size(); ++c) {
        const int64_t d0 = dt_off[c], d1 = dt_off[c + 1], g0 = gt_off[c], g1 = gt_off[c + 1];
        if (d1 < d0 || g1 < g0 || (d1 > d0 && !dts) || (g1 > g0 && !gts)) {
            yxh::set_error("coco_eval: bad instance offsets at cell %zu", c);
            return YXH_EINVAL;
        }
        Cell& cell = cells[c];
        cell.det.resize(d1 - d0);
        std::iota(cell.det.begin(), cell.det.end(), (int32_t)d0);
        std::stable_sort(cell.det.begin(), cell.det.end(),
                         [dts](int32_t a, int32_t b) { return dts[a].score > dts[b].score; });
        if ((int)cell.det.size() > maxdet) cell.det.resize(maxdet);
        const int G = (int)(g1 - g0);
        cell.iou.resize(cell.det.size() * (size_t)G);
        for (size_t d = 0; d < cell.det.size(); ++d)
            for (int g = 0; g < G; ++g) cell.iou[d * G + g] = box_iou(dts[cell.det[d]], gts[g0 + g]);
    }
    const size_t nprec = (size_t)T * R * K * A * M, nrec = (size_t)T * K * A * M;
    std::fill(precision, precision + nprec, -1.0);
    std::fill(scores, scores + nprec, -1.0);
    std::fill(recall, recall + nrec, -1.0);
    std::vector<Matches> mt(I);
    struct Ref { double score; int img, d; };
    std::vector<Ref> list;
    std::vector<double> prec, rec;
    for (int k = 0; k < K; ++k) {
        for (int a = 0; a < A; ++a) {
            // step 2 for every image of this (category, area range)
            for (int i = 0; i < I; ++i) {
                const size_t c = (size_t)i * K + k;
                match_cell(gts ? gts + gt_off[c] : nullptr, (int)(gt_off[c + 1] - gt_off[c]), dts, cells[c],
                           p->area_ranges + 2 * a, p->iou_thresholds, T, mt[i]);
            }
            int valid = 0;
            for (int i = 0; i < I; ++i) valid += mt[i].valid_gt;
            for (int m = 0; m < M; ++m) {
                if (valid == 0) continue;
                // step 3
                list.clear();
                for (int i = 0; i < I; ++i)
                    for (int d = 0; d < (int)mt[i].score.size() && d < p->max_dets[m]; ++d)
                        list.push_back({mt[i].score[d], i, d});
                std::stable_sort(list.begin(), list.end(), [](const Ref& x, const Ref& y) { return x.score > y.score; });
                for (int t = 0; t < T; ++t) {
                    long long tp = 0, fp = 0;
                    prec.clear();
                    rec.clear();
                    for (const Ref& r : list) {
                        const Matches& q = mt[r.img];
                        const size_t j = (size_t)t * q.score.size() + r.d;
                        if (!q.ignored[j]) {  // ignored: neither TP nor FP, the curve repeats
                            tp += q.match[j] > 0;
                            fp += q.match[j] == 0;
                        }
                        rec.push_back((double)tp / valid);
                        prec.push_back(tp + fp > 0 ? (double)tp / (double)(tp + fp) : 0.0);
                    }
                    const size_t ri = (((size_t)t * K + k) * A + a) * M + m;
                    recall[ri] = rec.empty() ? 0.0 : rec.back();
                    for (size_t n = prec.size(); n-- > 1;)
                        if (prec[n] > prec[n - 1]) prec[n - 1] = prec[n];
                    for (int rr = 0; rr < R; ++rr) {
                        const size_t at = std::lower_bound(rec.begin(), rec.end(), p->recall_thresholds[rr]) - rec.begin();
                        const size_t o = ((((size_t)t * R + rr) * K + k) * A + a) * M + m;
                        if (at < prec.size()) {
                            precision[o] = prec[at];
                            scores[o] = list[at].score;
                        } else {
                            precision[o] = 0.0;
                            scores[o] = 0.0;
                        }
                    }
                }
            }
        }
    }
    return YXH_OK;
}

extern "C" int yxh_coco_iou(const yxh_coco_instance* dts, int32_t nd, const yxh_coco_instance* gts, int32_t ng,
                            double* iou) {
    if (nd < 0 || ng < 0 || (nd && !dts) || (ng && !gts) || (nd && ng && !iou)) {
        yxh::set_error("coco_iou: bad arguments");
        return YXH_EINVAL;
    }
    for (int d = 0; d < nd; ++d)
        for (int g = 0; g < ng; ++g) iou[(size_t)d * ng + g] = box_iou(dts[d], gts[g]);
    return YXH_OK;
}
