// C-ABI surface of libyoloxhip: argument checking, error channel, the op-list
// executor and hipGraph capture/replay of a whole forward pass.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <vector>

#include "yxh_common.hpp"

namespace yxh {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return YXH_OK;
    set_error("%s: %s", what, hipGetErrorString(e));
    return YXH_EHIP;
}

int device_cus() {
    // queried once per process, on the first launch's device: every conv launch asks, and a
    // hipGetDevice per launch cost the eager training step (~1 600 launches, host-bound) 1.5-3 ms
    // of host issue (profiles/r06).  One process drives one GPU model (one process per GPU).
    static std::atomic<int> cache{0};
    int n = cache.load(std::memory_order_relaxed);
    if (n == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        cache.store(n, std::memory_order_relaxed);
    }
    return n;
}

int conv2d(const yxh_conv_desc* d, hipStream_t st);
int focus_pack_launch(const void* img, int layout, int idt, int B, int H, int W, void* dst, int odt,
                      hipStream_t st);
int spp_launch(void* buf, int dt, int B, int H, int W, int C, int cs, long long bs, hipStream_t st);
int pack_frag_launch(const void* w, int cout, int taps, int cin, int dt, void* out, hipStream_t st);
int fold_launch(const float* w, const float* cb, const float* g, const float* beta, const float* mean,
                const float* var, float eps, int cout, int cin_g, int kh, int kw, int cin_pad, int dt, void* wo,
                float* bo, hipStream_t st);
int stem_launch(const yxh_stem_desc* d, hipStream_t st);
int stem_pack_launch(const float* w, const float* g, const float* beta, const float* mean, const float* var,
                     float eps, int cout, int dt, void* wo, float* bo, hipStream_t st);
size_t pp_workspace(int B, int A);
void pp_set_mask_budget(size_t bytes);
size_t sim_workspace(int B, int A, int L);
int yolox_loss(const float* preds, const float* origin, const float* labels, int B, int A, int C, int L,
               const int* lhw, const int* strides, int nlev, uint8_t* fg, int* matched, float* piou, int* num_fg,
               float* losses, void* ws, size_t ws_bytes, hipStream_t st);
int letterbox_batch_launch(const uint8_t* pool, const yxh_lb_image* images, int B, int th, int tw, int fmt,
                           void* dst, hipStream_t st);
size_t reduce_workspace(int C);
int bn_stats(int dt, int B, const yxh_src* y, const float* gamma, const float* beta, float* rmean, float* rvar,
             float eps, float momentum, float* stats, void* ws, size_t ws_bytes, hipStream_t st);
int bn_act_fwd_launch(int dt, int B, const yxh_src* y, const float* stats, int act, const yxh_src* res,
                      const yxh_src* out, hipStream_t st);
int bn_act_bwd_launch(int dt, int B, const yxh_src* y, const yxh_src* dout, const float* stats, const float* gamma,
                      int act, float* dgamma, float* dbeta, void* dx, void* ws, size_t ws_bytes, hipStream_t st);
int channel_sum_launch(int dt, int B, const yxh_src* x, float* out, void* ws, size_t ws_bytes, hipStream_t st);
int conv_wgrad_launch(const yxh_wgrad_desc* d, hipStream_t st);
int pack_dgrad_launch(const float* w, int cout, int cin, int kh, int kw, int c_begin, int c_count, int cout_pad, int dt,
                      void* out, hipStream_t st);
int spp_bwd_launch(int dt, int B, const yxh_src* cat, int c, const float* dcat, float* dx, hipStream_t st);
int pack_batch_launch(const yxh_pack_job* jobs, int njobs, int total_blocks, int dt, hipStream_t st);
int upsample_bwd_launch(const float* g, int B, int h, int w, int C, float* dst, hipStream_t st);
size_t dw_wgrad_workspace_bytes(long long pixels, int channels, int k);
int dw_wgrad_launch(int dt, int B, const yxh_src* x, const yxh_src* dy, int C, int k, int stride, int pad, int out_h,
                    int out_w, float* dw, void* ws, size_t ws_bytes, hipStream_t st);
int dw_dgrad_launch(int dt, int B, const yxh_src* dy, const void* w, int C, int k, int stride, int pad, int in_h,
                    int in_w, float* dx, int dxcs, long long dxbs, int accumulate, hipStream_t st);
int resize_bilinear_launch(int dt, int B, int C, int ih, int iw, const void* src, int oh, int ow, void* dst,
                           hipStream_t st);
int head_decode_train_launch(const float* raw, int B, int A, int C, const int* lhw, const int* strides, int nlev,
                             float* out, hipStream_t st);
int yolox_loss_bwd(const float* preds, const float* raw, const float* labels, int B, int A, int C, int L,
                   const int* lhw, const int* strides, int nlev, const uint8_t* fg, const int* matched,
                   const float* piou, const int* num_fg, const float* gtot, int use_l1, int dt, void* g_ro,
                   void* g_cls, hipStream_t st);
int postprocess(float* pred, int B, int A, int C, float conf, double nms, int agnostic, long long vanilla_numel,
                float* det, int* counts, void* ws, size_t ws_bytes, hipStream_t st, hipEvent_t filter_done,
                hipStream_t rest, const float* scores = nullptr);
int head_pred_launch(const yxh_head_desc* d, hipStream_t st);
int stem_s2_launch(const yxh_stem2_desc* d, hipStream_t st);
int augment_batch_launch(const uint8_t* pool, const yxh_aug_image* images, int B, int H, int W, uint8_t* mosaic_ws,
                         float* out, hipStream_t st);

static int run_op(const yxh_op& op, hipStream_t st) {
    switch (op.kind) {
        case YXH_OP_CONV:
            return conv2d(&op.u.conv, st);
        case YXH_OP_FOCUS: {
            const yxh_focus_desc& f = op.u.focus;
            return focus_pack_launch(f.img, f.layout, f.img_dtype, f.batch, f.h, f.w, f.dst, f.dst_dtype, st);
        }
        case YXH_OP_STEM:
            return stem_launch(&op.u.stem, st);
        case YXH_OP_HEAD:
            return head_pred_launch(&op.u.head, st);
        case YXH_OP_STEM2:
            return stem_s2_launch(&op.u.stem2, st);
        case YXH_OP_SPP: {
            const yxh_spp_desc& s = op.u.spp;
            return spp_launch(s.buf, s.dtype, s.batch, s.h, s.w, s.c, s.cstride, s.bstride, st);
        }
        default:
            set_error("unknown op kind %d", op.kind);
            return YXH_EINVAL;
    }
}

}  // namespace yxh

using namespace yxh;

extern "C" {

int yxh_abi_version(void) { return YXH_ABI_VERSION; }
const char* yxh_last_error(void) { return g_err; }
size_t yxh_sizeof_op(void) { return sizeof(yxh_op); }
size_t yxh_sizeof_conv_desc(void) { return sizeof(yxh_conv_desc); }

int yxh_conv2d(const yxh_conv_desc* d, void* stream) { return conv2d(d, (hipStream_t)stream); }

int yxh_head_pred(const yxh_head_desc* d, void* stream) { return head_pred_launch(d, (hipStream_t)stream); }

int yxh_focus_pack(const void* img, int32_t layout, int32_t img_dtype, int32_t batch, int32_t h, int32_t w,
                   void* dst, int32_t dst_dtype, void* stream) {
    return focus_pack_launch(img, layout, img_dtype, batch, h, w, dst, dst_dtype, (hipStream_t)stream);
}

int yxh_stem_conv(const yxh_stem_desc* d, void* stream) { return stem_launch(d, (hipStream_t)stream); }

int yxh_stem_s2(const yxh_stem2_desc* d, void* stream) { return stem_s2_launch(d, (hipStream_t)stream); }

int yxh_stem_pack(const float* conv_w, const float* bn_gamma, const float* bn_beta, const float* bn_mean,
                  const float* bn_var, float eps, int32_t cout, int32_t dtype, void* w_out, float* b_out,
                  void* stream) {
    return stem_pack_launch(conv_w, bn_gamma, bn_beta, bn_mean, bn_var, eps, cout, dtype, w_out, b_out,
                            (hipStream_t)stream);
}

int yxh_spp_maxpool(void* buf, int32_t dtype, int32_t batch, int32_t h, int32_t w, int32_t c, int32_t cstride,
                    int64_t bstride, void* stream) {
    return spp_launch(buf, dtype, batch, h, w, c, cstride, bstride, (hipStream_t)stream);
}

int yxh_pack_frag(const void* w, int32_t cout, int32_t taps, int32_t cin, int32_t dtype, void* out, void* stream) {
    return pack_frag_launch(w, cout, taps, cin, dtype, out, (hipStream_t)stream);
}

int yxh_fold_bn_pack(const float* conv_w, const float* conv_bias, const float* bn_gamma, const float* bn_beta,
                     const float* bn_mean, const float* bn_var, float eps, int32_t cout, int32_t cin_g, int32_t kh,
                     int32_t kw, int32_t cin_pad, int32_t dtype, void* w_out, float* b_out, void* stream) {
    return fold_launch(conv_w, conv_bias, bn_gamma, bn_beta, bn_mean, bn_var, eps, cout, cin_g, kh, kw, cin_pad,
                       dtype, w_out, b_out, (hipStream_t)stream);
}

int yxh_letterbox_batch(const uint8_t* pool, const yxh_lb_image* images, int32_t batch, int32_t dst_h,
                        int32_t dst_w, int32_t out_format, void* dst, void* stream) {
    return letterbox_batch_launch(pool, images, batch, dst_h, dst_w, out_format, dst, (hipStream_t)stream);
}

int yxh_augment_batch(const uint8_t* pool, const yxh_aug_image* images, int32_t batch, int32_t h, int32_t w,
                      uint8_t* mosaic_ws, float* out, void* stream) {
    return augment_batch_launch(pool, images, batch, h, w, mosaic_ws, out, (hipStream_t)stream);
}

size_t yxh_sizeof_aug_image(void) { return sizeof(yxh_aug_image); }

size_t yxh_postprocess_workspace_bytes(int32_t batch, int32_t anchors) { return pp_workspace(batch, anchors); }

void yxh_set_nms_mask_budget(size_t bytes) { pp_set_mask_budget(bytes); }

int yxh_postprocess(float* pred, int32_t batch, int32_t anchors, int32_t num_classes, float conf_thre,
                    double nms_thre, int32_t class_agnostic, int64_t vanilla_numel, float* det, int32_t* counts,
                    void* workspace, size_t workspace_bytes, void* stream) {
    return postprocess(pred, batch, anchors, num_classes, conf_thre, nms_thre, class_agnostic, vanilla_numel, det,
                       counts, workspace, workspace_bytes, (hipStream_t)stream, nullptr, nullptr);
}

int yxh_postprocess_ev(float* pred, int32_t batch, int32_t anchors, int32_t num_classes, float conf_thre,
                       double nms_thre, int32_t class_agnostic, int64_t vanilla_numel, float* det, int32_t* counts,
                       void* workspace, size_t workspace_bytes, void* filter_done, void* stream) {
    return postprocess(pred, batch, anchors, num_classes, conf_thre, nms_thre, class_agnostic, vanilla_numel, det,
                       counts, workspace, workspace_bytes, (hipStream_t)stream, (hipEvent_t)filter_done, nullptr);
}

int yxh_postprocess_split(float* pred, int32_t batch, int32_t anchors, int32_t num_classes, float conf_thre,
                          double nms_thre, int32_t class_agnostic, int64_t vanilla_numel, float* det, int32_t* counts,
                          void* workspace, size_t workspace_bytes, void* filter_done, void* filter_stream,
                          void* rest_stream) {
    YXH_CHECK_ARG(filter_done, "yxh_postprocess_split: null filter_done event");
    return postprocess(pred, batch, anchors, num_classes, conf_thre, nms_thre, class_agnostic, vanilla_numel, det,
                       counts, workspace, workspace_bytes, (hipStream_t)filter_stream, (hipEvent_t)filter_done,
                       (hipStream_t)rest_stream);
}

int yxh_postprocess_scored(float* pred, const float* scores, int32_t batch, int32_t anchors, int32_t num_classes,
                           float conf_thre, double nms_thre, int32_t class_agnostic, int64_t vanilla_numel, float* det,
                           int32_t* counts, void* workspace, size_t workspace_bytes, void* filter_done,
                           void* filter_stream, void* rest_stream) {
    YXH_CHECK_ARG(scores && ((uintptr_t)scores % 16) == 0, "yxh_postprocess_scored: 16-byte aligned score records");
    return postprocess(pred, batch, anchors, num_classes, conf_thre, nms_thre, class_agnostic, vanilla_numel, det,
                       counts, workspace, workspace_bytes, (hipStream_t)filter_stream, (hipEvent_t)filter_done,
                       (hipStream_t)rest_stream, scores);
}

size_t yxh_yolox_loss_workspace_bytes(int32_t batch, int32_t anchors, int32_t max_labels) {
    return sim_workspace(batch, anchors, max_labels);
}

int yxh_yolox_loss(const float* preds, const float* origin, const float* labels, int32_t batch, int32_t anchors,
                   int32_t num_classes, int32_t max_labels, const int32_t* level_hw, const int32_t* strides,
                   int32_t nlevels, uint8_t* fg_mask, int32_t* matched_gt, float* pred_iou, int32_t* num_fg,
                   float* losses, void* workspace, size_t workspace_bytes, void* stream) {
    return yolox_loss(preds, origin, labels, batch, anchors, num_classes, max_labels, level_hw, strides, nlevels,
                      fg_mask, matched_gt, pred_iou, num_fg, losses, workspace, workspace_bytes, (hipStream_t)stream);
}

size_t yxh_reduce_workspace_bytes(int32_t channels) { return reduce_workspace(channels); }

int yxh_bn_stats(int32_t dtype, int32_t batch, const yxh_src* y, const float* gamma, const float* beta,
                 float* running_mean, float* running_var, float eps, float momentum, float* stats, void* workspace,
                 size_t workspace_bytes, void* stream) {
    return bn_stats(dtype, batch, y, gamma, beta, running_mean, running_var, eps, momentum, stats, workspace,
                    workspace_bytes, (hipStream_t)stream);
}

int yxh_bn_act_fwd(int32_t dtype, int32_t batch, const yxh_src* y, const float* stats, int32_t act,
                   const yxh_src* residual, const yxh_src* out, void* stream) {
    return bn_act_fwd_launch(dtype, batch, y, stats, act, residual, out, (hipStream_t)stream);
}

int yxh_bn_act_bwd(int32_t dtype, int32_t batch, const yxh_src* y, const yxh_src* dout, const float* stats,
                   const float* gamma, int32_t act, float* dgamma, float* dbeta, void* dx, void* workspace,
                   size_t workspace_bytes, void* stream) {
    return bn_act_bwd_launch(dtype, batch, y, dout, stats, gamma, act, dgamma, dbeta, dx, workspace, workspace_bytes,
                             (hipStream_t)stream);
}

int yxh_channel_sum(int32_t dtype, int32_t batch, const yxh_src* x, float* out, void* workspace,
                    size_t workspace_bytes, void* stream) {
    return channel_sum_launch(dtype, batch, x, out, workspace, workspace_bytes, (hipStream_t)stream);
}

int yxh_conv_wgrad(const yxh_wgrad_desc* d, void* stream) { return conv_wgrad_launch(d, (hipStream_t)stream); }

int yxh_pack_dgrad_weight(const float* w, int32_t cout, int32_t cin, int32_t kh, int32_t kw, int32_t c_begin,
                          int32_t c_count, int32_t cout_pad, int32_t dtype, void* out, void* stream) {
    return pack_dgrad_launch(w, cout, cin, kh, kw, c_begin, c_count, cout_pad, dtype, out, (hipStream_t)stream);
}

int yxh_pack_weights_batch(const yxh_pack_job* jobs, int32_t njobs, int32_t total_blocks, int32_t dtype,
                           void* stream) {
    return pack_batch_launch(jobs, njobs, total_blocks, dtype, (hipStream_t)stream);
}

int yxh_spp_bwd(int32_t dtype, int32_t batch, const yxh_src* cat, int32_t c, const float* dcat, float* dx,
                void* stream) {
    return spp_bwd_launch(dtype, batch, cat, c, dcat, dx, (hipStream_t)stream);
}

int yxh_upsample_bwd(const float* g, int32_t batch, int32_t h, int32_t w, int32_t c, float* dst, void* stream) {
    return upsample_bwd_launch(g, batch, h, w, c, dst, (hipStream_t)stream);
}

size_t yxh_dw_wgrad_workspace_bytes(int32_t batch, int32_t out_h, int32_t out_w, int32_t channels, int32_t k) {
    return dw_wgrad_workspace_bytes((long long)batch * out_h * out_w, channels, k);
}

int yxh_dw_wgrad(int32_t dtype, int32_t batch, const yxh_src* x, const yxh_src* dy, int32_t channels, int32_t k,
                 int32_t stride, int32_t pad, int32_t out_h, int32_t out_w, float* dw, void* workspace,
                 size_t workspace_bytes, void* stream) {
    return dw_wgrad_launch(dtype, batch, x, dy, channels, k, stride, pad, out_h, out_w, dw, workspace, workspace_bytes,
                           (hipStream_t)stream);
}

int yxh_dw_dgrad(int32_t dtype, int32_t batch, const yxh_src* dy, const void* w, int32_t channels, int32_t k,
                 int32_t stride, int32_t pad, int32_t in_h, int32_t in_w, float* dx, int32_t dx_cstride,
                 int64_t dx_bstride, int32_t accumulate, void* stream) {
    return dw_dgrad_launch(dtype, batch, dy, w, channels, k, stride, pad, in_h, in_w, dx, dx_cstride, dx_bstride,
                           accumulate, (hipStream_t)stream);
}

int yxh_resize_bilinear(int32_t dtype, int32_t batch, int32_t channels, int32_t in_h, int32_t in_w, const void* src,
                        int32_t out_h, int32_t out_w, void* dst, void* stream) {
    return resize_bilinear_launch(dtype, batch, channels, in_h, in_w, src, out_h, out_w, dst, (hipStream_t)stream);
}

int yxh_head_decode_train(const float* raw, int32_t batch, int32_t anchors, int32_t num_classes,
                          const int32_t* level_hw, const int32_t* strides, int32_t nlevels, float* out, void* stream) {
    return head_decode_train_launch(raw, batch, anchors, num_classes, level_hw, strides, nlevels, out,
                                    (hipStream_t)stream);
}

int yxh_yolox_loss_bwd(const float* preds, const float* raw, const float* labels, int32_t batch, int32_t anchors,
                       int32_t num_classes, int32_t max_labels, const int32_t* level_hw, const int32_t* strides,
                       int32_t nlevels, const uint8_t* fg_mask, const int32_t* matched_gt, const float* pred_iou,
                       const int32_t* num_fg, const float* grad_total, int32_t use_l1, int32_t dtype, void* g_regobj,
                       void* g_cls, void* stream) {
    return yolox_loss_bwd(preds, raw, labels, batch, anchors, num_classes, max_labels, level_hw, strides, nlevels,
                          fg_mask, matched_gt, pred_iou, num_fg, grad_total, use_l1, dtype, g_regobj, g_cls,
                          (hipStream_t)stream);
}

int yxh_run_ops(const yxh_op* ops, int32_t n, void* stream) {
    YXH_CHECK_ARG(ops || n == 0, "null op list");
    for (int i = 0; i < n; ++i) {
        int rc = run_op(ops[i], (hipStream_t)stream);
        if (rc) {
            char tmp[512];
            snprintf(tmp, sizeof(tmp), "op %d: %s", i, g_err);
            set_error("%s", tmp);
            return rc;
        }
    }
    return YXH_OK;
}

int yxh_graph_create(const yxh_op* ops, int32_t n, void* stream, void** graph_exec) {
    YXH_CHECK_ARG(graph_exec, "null graph_exec");
    (void)stream;
    hipStream_t cap;
    int rc = check_hip(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking), "capture stream");
    if (rc) return rc;
    rc = check_hip(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal), "begin capture");
    if (rc) {
        (void)hipStreamDestroy(cap);
        return rc;
    }
    int orc = yxh_run_ops(ops, n, cap);
    hipGraph_t g = nullptr;
    rc = check_hip(hipStreamEndCapture(cap, &g), "end capture");
    (void)hipStreamDestroy(cap);
    if (orc) {
        if (g) (void)hipGraphDestroy(g);
        return orc;
    }
    if (rc) return rc;
    hipGraphExec_t ge = nullptr;
    rc = check_hip(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0), "instantiate");
    (void)hipGraphDestroy(g);
    if (rc) return rc;
    *graph_exec = (void*)ge;
    return YXH_OK;
}

// One graph node per op, wired by the op list's own dependency edges: each op is captured
// ALONE on one stream into a small graph (a conv is one kernel, post-processing several)
// and added to the parent as a child-graph node whose predecessors are the nodes of the ops
// it depends on.  No multi-stream capture is involved (yxh_graph_create_lanes with more
// than four capture streams ended in a segfault inside the lane join / hipStreamEndCapture
// after every op had been captured), and the parent holds exactly the dataflow DAG: every
// pair of independent ops -- the head levels, or batch chunks with arenas of their own --
// may run concurrently, with no lane assignment by the caller.
int yxh_graph_create_dag(const yxh_op* ops, int32_t n, const int32_t* dep_off, const int32_t* deps, void* stream,
                         void** graph_exec) {
    YXH_CHECK_ARG(graph_exec && (ops || n == 0) && dep_off, "null argument");
    YXH_CHECK_ARG(dep_off[0] == 0, "dep_off[0] must be 0");
    for (int i = 0; i < n; ++i) {
        YXH_CHECK_ARG(dep_off[i + 1] >= dep_off[i], "dep_off not monotone at %d", i);
        for (int k = dep_off[i]; k < dep_off[i + 1]; ++k)
            YXH_CHECK_ARG(deps && deps[k] >= 0 && deps[k] < i, "op %d dependency %d", i, deps ? deps[k] : -1);
    }
    (void)stream;
    hipStream_t cap = nullptr;
    hipGraph_t parent = nullptr;
    int rc = check_hip(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking), "capture stream");
    if (!rc) rc = check_hip(hipGraphCreate(&parent, 0), "graph create");
    std::vector<hipGraphNode_t> node(n, nullptr);
    std::vector<hipGraphNode_t> pred;
    int orc = YXH_OK;
    for (int i = 0; i < n && !rc && !orc; ++i) {
        rc = check_hip(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal), "begin capture");
        if (rc) break;
        orc = run_op(ops[i], cap);
        hipGraph_t g = nullptr;
        const int erc = check_hip(hipStreamEndCapture(cap, &g), "end capture");
        if (orc) {
            char tmp[512];
            snprintf(tmp, sizeof(tmp), "op %d: %s", i, g_err);
            set_error("%s", tmp);
        } else {
            rc = erc;
        }
        if (!rc && !orc) {
            pred.clear();
            for (int k = dep_off[i]; k < dep_off[i + 1]; ++k) {
                hipGraphNode_t d = node[deps[k]];
                bool dup = false;
                for (auto q : pred) dup |= q == d;
                if (!dup) pred.push_back(d);
            }
            rc = check_hip(hipGraphAddChildGraphNode(&node[i], parent, pred.empty() ? nullptr : pred.data(),
                                                     pred.size(), g),
                           "add op node");
        }
        if (g) (void)hipGraphDestroy(g);
    }
    hipGraphExec_t ge = nullptr;
    if (!rc && !orc) rc = check_hip(hipGraphInstantiate(&ge, parent, nullptr, nullptr, 0), "instantiate");
    if (parent) (void)hipGraphDestroy(parent);
    if (cap) (void)hipStreamDestroy(cap);
    if (orc) return orc;
    if (rc) return rc;
    *graph_exec = (void*)ge;
    return YXH_OK;
}

int yxh_graph_create_lanes(const yxh_op* ops, int32_t n, const int32_t* lanes, const int32_t* dep_off,
                           const int32_t* deps, int32_t nlanes, void* stream, void** graph_exec) {
    // Cap = the most capture streams a GPU test replays (tests/test_gpu_model.py: 8 chunk lanes,
    // bit-exact).  Round 2 saw a segfault in the join / hipStreamEndCapture with 7 streams (head
    // levels plus three reg lanes, chunked plan), never reproduced since (4-12 streams of plain
    // kernels, profiles/r04/lanes_probe.txt; the 8-lane plan).  Reading this function for what that
    // op list could have had that the probes did not (round 6): a lane with NO op.  Such a lane's
    // stream joined the capture only through the fork, whose event is recorded right after
    // BeginCapture, before any node exists (an empty dependency set); at the join its event record
    // and the origin's wait then carry that empty set -- the one capture path no passing run
    // exercised.  Lanes without ops now never join the capture (no stream, no fork wait, no join);
    // tests/test_gpu_model.py captures a plan with two empty lanes.  The cap stays at 8.
    constexpr int kMaxLanes = 8;
    YXH_CHECK_ARG(graph_exec && (ops || n == 0) && lanes && dep_off, "null argument");
    YXH_CHECK_ARG(nlanes >= 1 && nlanes <= kMaxLanes, "nlanes %d", nlanes);
    YXH_CHECK_ARG(dep_off[0] == 0, "dep_off[0] must be 0");
    for (int i = 0; i < n; ++i) {
        YXH_CHECK_ARG(lanes[i] >= 0 && lanes[i] < nlanes, "op %d lane %d", i, lanes[i]);
        YXH_CHECK_ARG(dep_off[i + 1] >= dep_off[i], "dep_off not monotone at %d", i);
        for (int k = dep_off[i]; k < dep_off[i + 1]; ++k)
            YXH_CHECK_ARG(deps && deps[k] >= 0 && deps[k] < i, "op %d dependency %d", i, deps ? deps[k] : -1);
    }
    (void)stream;
    hipStream_t st[kMaxLanes] = {};
    bool used[kMaxLanes] = {};
    used[0] = true;  // the origin stream carries the capture
    for (int i = 0; i < n; ++i) used[lanes[i]] = true;
    hipEvent_t fork = nullptr;
    std::vector<hipEvent_t> ev(n, nullptr), join(nlanes, nullptr);
    int rc = YXH_OK, orc = YXH_OK;
    bool capturing = false;
    hipGraph_t g = nullptr;
    for (int l = 0; l < nlanes && !rc; ++l)
        if (used[l]) rc = check_hip(hipStreamCreateWithFlags(&st[l], hipStreamNonBlocking), "lane stream");
    if (!rc) rc = check_hip(hipEventCreateWithFlags(&fork, hipEventDisableTiming), "event");
    for (int i = 0; i < n && !rc; ++i) rc = check_hip(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming), "event");
    for (int l = 0; l < nlanes && !rc; ++l)
        rc = check_hip(hipEventCreateWithFlags(&join[l], hipEventDisableTiming), "event");
    const bool dbg = getenv("YXH_DEBUG_LANES") != nullptr;
#define LDBG(...) do { if (dbg) { fprintf(stderr, __VA_ARGS__); fflush(stderr); } } while (0)
    LDBG("lanes: n=%d nlanes=%d rc=%d\n", n, nlanes, rc);
    if (!rc) {
        rc = check_hip(hipStreamBeginCapture(st[0], hipStreamCaptureModeThreadLocal), "begin capture");
        capturing = !rc;
    }
    LDBG("lanes: capture begun rc=%d\n", rc);
    if (!rc) rc = check_hip(hipEventRecord(fork, st[0]), "fork");
    for (int l = 1; l < nlanes && !rc; ++l)
        if (used[l]) rc = check_hip(hipStreamWaitEvent(st[l], fork, 0), "fork wait");
    for (int i = 0; i < n && !rc && !orc; ++i) {
        hipStream_t s = st[lanes[i]];
        for (int k = dep_off[i]; k < dep_off[i + 1] && !rc; ++k)
            if (lanes[deps[k]] != lanes[i]) rc = check_hip(hipStreamWaitEvent(s, ev[deps[k]], 0), "dependency wait");
        if (rc) break;
        LDBG("lanes: op %d kind %d lane %d deps %d\n", i, ops[i].kind, lanes[i], dep_off[i + 1] - dep_off[i]);
        orc = run_op(ops[i], s);
        if (orc) {
            char tmp[512];
            snprintf(tmp, sizeof(tmp), "op %d: %s", i, g_err);
            set_error("%s", tmp);
        } else {
            rc = check_hip(hipEventRecord(ev[i], s), "op event");
        }
    }
    LDBG("lanes: ops done rc=%d orc=%d\n", rc, orc);
    if (capturing) {  // join every lane (also after an error, so the capture ends cleanly)
        for (int l = 1; l < nlanes; ++l) {
            if (!used[l]) continue;
            (void)hipEventRecord(join[l], st[l]);
            (void)hipStreamWaitEvent(st[0], join[l], 0);
        }
        const int erc = check_hip(hipStreamEndCapture(st[0], &g), "end capture");
        if (!rc) rc = erc;
    }
    LDBG("lanes: capture ended rc=%d\n", rc);
    hipGraphExec_t ge = nullptr;
    if (!rc && !orc) rc = check_hip(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0), "instantiate");
    LDBG("lanes: instantiated rc=%d\n", rc);
#undef LDBG
    if (g) (void)hipGraphDestroy(g);
    for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
    for (auto e : join)
        if (e) (void)hipEventDestroy(e);
    if (fork) (void)hipEventDestroy(fork);
    for (int l = 0; l < nlanes; ++l)
        if (st[l]) (void)hipStreamDestroy(st[l]);
    if (orc) return orc;
    if (rc) return rc;
    *graph_exec = (void*)ge;
    return YXH_OK;
}

int yxh_graph_launch(void* graph_exec, void* stream) {
    YXH_CHECK_ARG(graph_exec, "null graph");
    return check_hip(hipGraphLaunch((hipGraphExec_t)graph_exec, (hipStream_t)stream), "graph launch");
}

int yxh_graph_destroy(void* graph_exec) {
    if (!graph_exec) return YXH_OK;
    return check_hip(hipGraphExecDestroy((hipGraphExec_t)graph_exec), "graph destroy");
}

}  // extern "C"
