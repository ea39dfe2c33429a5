/*
 * yoloxhip.h -- C ABI of libyoloxhip.so, the MI355X (gfx950) hot path of YOLOX.
 *
 * The reference (pixeltable-yolox) is pure Python over PyTorch/torchvision; it has
 * no FFI of its own.  Each entry point below replaces the library kernels the
 * reference reaches through torch.nn / torchvision at the cited call sites, and is
 * bound by the package's Python layer (yolox_amd/_native.py, ctypes) exactly as a
 * maintainer would bind it from the reference.
 *
 * Conventions
 *  - Plain pointers and sizes only; every buffer (including workspace) is allocated
 *    by the caller in device memory.  Functions never allocate, free or synchronise,
 *    so every call is legal inside hipStreamBeginCapture.
 *  - `stream` is a hipStream_t passed as void*; work is enqueued asynchronously.
 *  - Return 0 on success, a negative YXH_E* code otherwise; yxh_last_error() gives
 *    a thread-local message.
 *  - Activations are NHWC with explicit pixel stride (`cstride`, elements between
 *    consecutive pixels) and image stride (`bstride`), so channel slices of a wider
 *    buffer (torch.cat outputs) and nearest-x2 upsampled reads (nn.Upsample) are
 *    addressed in place -- no concat or upsample tensor is ever materialised.
 */
#ifndef YOLOXHIP_H
#define YOLOXHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YXH_ABI_VERSION 18

enum yxh_status {
    YXH_OK = 0,
    YXH_EINVAL = -1,       /* bad shape / pointer / alignment            */
    YXH_EHIP = -2,         /* HIP runtime error                          */
    YXH_EUNSUPPORTED = -3  /* valid request this build does not implement */
};

enum yxh_dtype { YXH_F32 = 0, YXH_BF16 = 1, YXH_F16 = 2, YXH_U8 = 3 };

enum yxh_act {
    YXH_ACT_NONE = 0,
    YXH_ACT_SILU = 1,         /* network_blocks.py:15-24                                  */
    YXH_ACT_RELU = 2,
    YXH_ACT_LRELU = 3,        /* LeakyReLU(0.1)                                            */
    YXH_ACT_DECODE = 4,       /* eval head: ch 0-1 (v+grid)*s, 2-3 exp(v)*s, 4.. sigmoid
                                 (yolo_head.py:185-187, 233-251)                            */
    YXH_ACT_DECODE_TRAIN = 5, /* train head: ch 0-1, 2-3 decoded, 4.. raw logits
                                 (yolo_head.py:213-231)                                     */
    YXH_ACT_DECODE_RAW = 6    /* ABI 16, eval head with decode_in_inference = False: ch 0-3 raw,
                                 4.. sigmoid (yolo_head.py:185-187, 208-211)                */
};

/* One input operand of a convolution: `channels` channels starting at `ptr`. */
typedef struct {
    const void* ptr;  /* element pointer to channel 0 of this slice                         */
    int32_t channels; /* channels taken from this source                                    */
    int32_t cstride;  /* elements between consecutive pixels                                */
    int64_t bstride;  /* elements between consecutive images                                */
    int32_t h, w;     /* stored spatial size                                                */
    int32_t upsample; /* 0: pixel (y,x); 1: nearest x2, reads (y>>1, x>>1) (yolo_pafpn.py:32);
                         2: zero-inserting x2 dilation, (y,x) even -> (y>>1, x>>1), odd -> 0
                            (the input of a stride-2 conv's data gradient; register-staged
                            conv kernel only)                                               */
    int32_t reserved;
} yxh_src;

/*
 * yxh_conv2d: Conv2d (+ folded BatchNorm) + activation (+ residual), implicit GEMM on
 * MFMA.  Replaces BaseConv.forward (network_blocks.py:48-49, conv/bn/act), the
 * Bottleneck residual add (:97-99), torch.cat before CspLayer.conv3 / PAFPN CSPs
 * (network_blocks.py:182, yolo_pafpn.py:98-112) via 2 sources, nn.Upsample via
 * src.upsample, the head's 1x1 preds + cat + sigmoid + decode (yolo_head.py:149-251)
 * via YXH_ACT_DECODE*, and DWConv's depthwise conv (network_blocks.py:55-74) via
 * groups == cin.
 *
 * weight: [cout][kh][kw][cin/groups] in `dtype`, BatchNorm already folded
 *         (yxh_fold_bn_pack).  bias: fp32 [cout].
 * residual (optional): same dtype as dst, added AFTER the activation.
 * dst: `dst_dtype` (dtype or F32); for DECODE acts the pixel (b, y, x) of a level is
 *      row b*dst_bstride + (y*out_w + x)*dst_cstride of the [B, A, 5+C] output.
 */
typedef struct {
    int32_t dtype;      /* YXH_F32 / YXH_BF16 / YXH_F16: inputs, weights, MFMA operands */
    int32_t batch;
    int32_t in_h, in_w; /* logical input size (after upsampling)                        */
    int32_t out_h, out_w;
    int32_t cin, cout, kh, kw, stride, pad;
    int32_t groups;     /* 1, or cin for depthwise                                       */
    int32_t nsrc;       /* 1 or 2; src[0].channels + src[1].channels == cin             */
    yxh_src src[2];
    const void* weight;
    const float* bias;
    const void* residual;
    int32_t res_cstride;
    int32_t dst_dtype;
    int64_t res_bstride;
    void* dst;
    int32_t dst_cstride;
    int32_t act;
    int64_t dst_bstride;
    float decode_stride; /* level stride for DECODE acts                                */
    int32_t decode_coff; /* position of output channel 0 in the 5+C row (0 or 5)       */
    int32_t tile;        /* 0: heuristic; else 2*id + (slabs-1): id 1-9 explicit tile
                            (TN x TM) of the register-staged kernel, id 17-25 the same
                            tiles on the LDS-DMA kernel, id 33-51 the row-tiled 3x3
                            kernel, id 65-70 the persistent streaming 1x1 kernel;
                            for the weight-stationary 1x1 ids 201-210 / 241-258 the low
                            bit instead selects the 16-byte-store epilogue (round 6; a
                            tile without it refuses the odd code); chosen by the
                            planner's on-device autotune                                 */
    int32_t flags;       /* YXH_CONV_ACCUMULATE: f32 dst += result (gradient accumulation) */
    int32_t grid_cap;    /* 0, or the CUs the persistent tiles (conv_ws / conv_ws1 / conv_pwf) may occupy: a
                            graph lane running beside another lane's work leaves it the rest of the chip */
    /* Fused Bottleneck (network_blocks.py:77-99): when pre_weight is set, the source is the
     * Bottleneck input x and the 3x3 conv reads t = act(pre_weight . x + pre_bias) (its
     * conv1, a 1x1 cin -> cin, BatchNorm folded), computed per pixel tile on the halo in LDS
     * and never written to memory.  3x3 s1 16-bit convs on the conv_ws fused tiles only;
     * dst must not alias the source (tile halos are read while other tiles write). */
    const void* pre_weight; /* [cin][cin] in dtype                                          */
    const float* pre_bias;  /* fp32 [cin]                                                    */
    /* Optional: `weight` in the MFMA fragment-major layout of yxh_pack_frag (16-bit, cout % 16
     * == 0, cin % 32 == 0).  The weight-stationary tiles (conv_ws / conv_ws1) then load their
     * stationary weights as whole 1 KiB wave reads (every lane one 16-byte piece of one
     * 128-byte line) instead of sixteen 64-byte row pieces per read; other tiles ignore it. */
    const void* weight_frag;
    /* ABI 15, optional 1x1 post conv (network_blocks.py:180-183 CspLayer.conv3 over the concat
     * [x_1 | x_2] after its last Bottleneck; :176-178 conv1 | conv2 after a stage's stride-2
     * conv).  When post_weight is set the conv's output (activation and residual applied,
     * rounded to dtype) is NOT stored to dst; a block keeps its output tile in LDS and writes
     *   post_dst <- SiLU(post_weight . [tile | post_src] + post_bias)
     * post_weight [post_cout][cout + post_src.channels] in dtype (the concat order), post_src
     * an optional second operand read at the conv's output pixels (channels 0: none).
     * conv_ws post tiles only (16-bit 3x3 whose block owns all cout channels). */
    const void* post_weight;
    const float* post_bias;
    yxh_src post_src;
    void* post_dst;
    int32_t post_cout;
    int32_t post_dst_cstride;
    int64_t post_dst_bstride;
    /* Head form (with YXH_CONV_GROUPS2: a level's cls_convs[k][1] | reg_convs[k][1]): group 0's
     * tile feeds the class preds (post_weight [post_cout = C][cout/2], 65-80 classes), group 1's
     * the reg | obj preds (post_weight2 [post_cout2 = 5][cout/2]); both write the level's fp32
     * [B, A, 5 + C] rows (post_dst = the level's first row, post_dst_cstride = 5 + C) decoded as
     * yxh_head_pred does (yolo_head.py:149-251): ch 0-1 (v + grid) * post_stride, 2-3
     * exp(v) * post_stride, 4.. sigmoid. */
    const void* post_weight2;
    const float* post_bias2;
    int32_t post_cout2;
    float post_stride;
} yxh_conv_desc;

#define YXH_CONV_ACCUMULATE 1
/* Two groups over one source of 2*cin channels: output channels [0, cout/2) read source channels
 * [0, cin), [cout/2, cout) read [cin, 2*cin) -- a head level's cls_convs[k][1] | reg_convs[k][1]
 * over its stacked [cls | reg] features (yolo_head.py:160-161) as ONE launch; conv_ws tiles,
 * 16-bit, 3x3 s1 only. */
#define YXH_CONV_GROUPS2 2
/* With post_weight (not the head form): ALSO store the conv's output tile to dst (the Bottleneck
 * chain of a CspLayer, network_blocks.py:95-99 / 160-183: Bottleneck i's 3x3 + shortcut output is
 * Bottleneck i+1's input and shortcut, and the post conv is Bottleneck i+1's conv1 over it). */
#define YXH_CONV_POST_STORE 4

int yxh_conv2d(const yxh_conv_desc* d, void* stream);

/*
 * yxh_focus_pack: Focus space-to-depth (network_blocks.py:193-208, channel order
 * TL, BL, TR, BR) of the network input into NHWC `dst_dtype` with 16 channels
 * (12 used, 4 zero), consumed by the stem conv.  Accepts the reference's layout
 * (float32 NCHW, processor.py:30-37) or NHWC uint8/bf16/f16/f32 images.
 */
enum yxh_layout { YXH_NCHW = 0, YXH_NHWC = 1 };
int yxh_focus_pack(const void* img, int32_t layout, int32_t img_dtype, int32_t batch, int32_t h,
                   int32_t w, void* dst, int32_t dst_dtype, void* stream);

/*
 * yxh_stem_conv: Focus + stem BaseConv fused (network_blocks.py:186-208,
 * darknet.py:112): the 3x3 conv on the 12 space-to-depth channels evaluated as the
 * equivalent 6x6 stride-2 pad-2 conv straight from the image (NCHW float32 or NHWC
 * uint8/bf16/f16/f32), BN folded, activation, NHWC output [B, h/2, w/2, cout].
 * weight/bias come from yxh_stem_pack ([round16(cout)][6][32] of `dtype`).
 */
typedef struct {
    const void* img;
    int32_t layout, img_dtype, batch, h, w;
    int32_t dtype, cout, act;
    const void* weight;
    const float* bias;
    void* dst;
    int32_t dst_cstride;
    int32_t reserved;
    int64_t dst_bstride;
} yxh_stem_desc;

/*
 * yxh_stem_s2: the Focus stem AND the first stride-2 3x3 conv (darknet.py:112-123 stem +
 * dark2[0], both BaseConv with BN folded) in one launch, from a uint8 / bf16 / f16 NHWC
 * image: the C1-channel stem map (H/2 x W/2) lives only in LDS, per 16 x 8 output tile.
 *   w1 [c1][3][3][12] (`dtype`; yxh_fold_bn_pack with cin_pad 12: k = ky*36 + kx*12 +
 *       q*3 + c over Focus channels q*3 + c, q = TL, BL, TR, BR), b1 [c1] fp32
 *   w2 [c2][3][3][c1] (`dtype`), b2 [c2] fp32
 *   dst [B][H/4][W/4] rows of dst_cstride elements (`dtype`), channels [0, c2)
 * bf16/f16 compute, c1 = 32 / c2 = 64 (yolox_s), h and w multiples of 4.
 */
typedef struct {
    const void* img;
    int32_t layout, img_dtype, batch, h, w;
    int32_t dtype, c1, c2, act;
    const void* w1;
    const float* b1;
    const void* w2;
    const float* b2;
    void* dst;
    int32_t dst_cstride;
    int32_t reserved;
    int64_t dst_bstride;
    /* ABI 15, optional CSP form (w3 != NULL): dark2's CspLayer conv1 | conv2 and its first
     * Bottleneck conv1 (network_blocks.py:176-178, 95-96) in the same launch.  The stride-2 map
     * is then NOT stored (dst unused):
     *   dst3 <- SiLU(w3 . map + b3), w3 [c2][c2] (conv1 rows then conv2 rows), whole 16-byte
     *           aligned rows of dst3_cstride elements;
     *   dst4 <- SiLU(w4 . dst3[:, :c2/2] + b4), w4 [c2/2][c2/2] (optional: w4 NULL skips it). */
    const void* w3;
    const float* b3;
    void* dst3;
    int32_t dst3_cstride;
    int32_t reserved3;
    int64_t dst3_bstride;
    const void* w4;
    const float* b4;
    void* dst4;
    int32_t dst4_cstride;
    int32_t reserved4;
    int64_t dst4_bstride;
} yxh_stem2_desc;
int yxh_stem_s2(const yxh_stem2_desc* d, void* stream);
int yxh_stem_conv(const yxh_stem_desc* d, void* stream);
int yxh_stem_pack(const float* conv_w, const float* bn_gamma, const float* bn_beta, const float* bn_mean,
                  const float* bn_var, float eps, int32_t cout, int32_t dtype, void* w_out, float* b_out,
                  void* stream);

/*
 * yxh_spp_maxpool: SPPBottleneck pools (network_blocks.py:129-141): reads channels
 * [0, c) of an NHWC buffer and writes max_pool(k, stride 1, pad k/2) for k = 5, 9,
 * 13 into channels [c, 2c), [2c, 3c), [3c, 4c) of the same buffer.
 */
int yxh_spp_maxpool(void* buf, int32_t dtype, int32_t batch, int32_t h, int32_t w, int32_t c,
                    int32_t cstride, int64_t bstride, void* stream);

/*
 * yxh_fold_bn_pack: BN folding (utils/model_utils.py:33-75) + repack of an
 * nn.Conv2d weight [cout][cin_g][kh][kw] fp32 to [cout][kh][kw][cin_pad] `dtype`
 * (zeros in [cin_g, cin_pad), e.g. the 12 Focus channels in the 16-channel layout of
 * yxh_focus_pack).  bn_* may be NULL (plain conv: scale 1, shift 0); conv_bias may be
 * NULL.
 */
int yxh_fold_bn_pack(const float* conv_w, const float* conv_bias, const float* bn_gamma,
                     const float* bn_beta, const float* bn_mean, const float* bn_var, float eps,
                     int32_t cout, int32_t cin_g, int32_t kh, int32_t kw, int32_t cin_pad,
                     int32_t dtype, void* w_out, float* b_out, void* stream);

/*
 * yxh_letterbox_batch: preproc / ValTransform (data_augment.py:140-156) for a whole
 * batch, replacing YoloxProcessor.__images_to_tensor's per-image loop + torch.stack
 * (processor.py:30-37).  `pool`: device bytes holding every source image (uint8 HWC
 * RGB, as np.array(PIL image) gives it); `images` (device): per image the byte offset
 * of its pixels in `pool` and its size.  Each image is resized by r = min(dst_h/h,
 * dst_w/w) (cv2 INTER_LINEAR restated; r == 1 is an exact copy) into the top-left of a
 * dst_h x dst_w canvas filled with 114.  out_format: YXH_LB_F32_NCHW -> float32
 * [B][3][dst_h][dst_w] (the reference's tensor), YXH_LB_U8_NHWC / YXH_LB_BF16_NHWC ->
 * [B][dst_h][dst_w][3] (read directly by yxh_stem_conv / yxh_focus_pack).  dst_w must be
 * a multiple of 4 and dst 16-byte aligned.  Images whose resized size is empty come
 * out as a plain 114 canvas (the Python layer rejects them first).
 */
typedef struct {
    int64_t src_offset;  /* bytes into pool */
    int32_t src_h, src_w;
} yxh_lb_image;
enum yxh_lb_format { YXH_LB_F32_NCHW = 0, YXH_LB_U8_NHWC = 1, YXH_LB_BF16_NHWC = 2 };
int yxh_letterbox_batch(const uint8_t* pool, const yxh_lb_image* images, int32_t batch, int32_t dst_h,
                        int32_t dst_w, int32_t out_format, void* dst, void* stream);

/*
 * yxh_augment_batch: the training-time sample pipeline for a whole batch on device, replacing
 * MosaicDetection.__getitem__ + mixup (datasets/mosaicdetection.py:76-232) and TrainTransform's
 * image half (data_augment.py:19-30 augment_hsv, :112-138 random_affine / _mirror, :140-156
 * preproc, :159-208) that the reference runs per image in DataLoader workers.  `pool`: device
 * bytes holding the dataset's pull_item images (uint8 HWC BGR, cv2.imread order); `images`
 * (device, one per sample): the parameters the host drew in the reference's random order and
 * the geometry derived from them (yolox_amd/data/mosaic.py packs them).  Output `out`: float32
 * [B][3][h][w] (TrainTransform's tensor); `mosaic_ws`: >= B*h*w*3 bytes of scratch (the warped
 * mosaic).  Labels stay on the host (numpy, as the reference computes them).  cv2's resize /
 * warpAffine / 8-bit HSV conversions are restated in fixed point (csrc/augment.hip).
 */
typedef struct {
    int32_t mosaic;   /* 1: mosaic + affine (+ mixup); 0: TrainTransform's letterbox of source 0 */
    int32_t mix;      /* mixup applied */
    int32_t flip;     /* _mirror applied */
    int32_t do_hsv;   /* augment_hsv applied */
    int32_t hsv[3];   /* augment_hsv's int16 gains (hue, saturation, value) */
    int32_t cp_flip;  /* mixup's FLIP */
    int64_t src_off[4];                      /* pool byte offset of each mosaic source */
    int32_t src_h[4], src_w[4];              /* source size */
    int32_t rh[4], rw[4];                    /* resized size: int(h0 * scale), int(w0 * scale) */
    double rsx[4], rsy[4];                   /* cv2 scale_x / scale_y = src / resized */
    int32_t lx1[4], ly1[4], lx2[4], ly2[4];  /* placement in the 2h x 2w canvas */
    int32_t sx1[4], sy1[4];                  /* crop origin inside the resized source */
    double minv[6];                          /* cv2.invertAffineTransform(M): output -> canvas */
    int64_t cp_off;                          /* mixup source (pool offset and size) */
    int32_t cp_h, cp_w, cp_rh, cp_rw;        /* ... and its letterbox size inside h x w */
    double cp_sx, cp_sy;
    int32_t jit_h, jit_w;                    /* jitter-resized letterbox canvas size */
    double jit_sx, jit_sy;
    int32_t x_off, y_off;                    /* crop offsets into the zero-padded copy */
} yxh_aug_image;
int yxh_augment_batch(const uint8_t* pool, const yxh_aug_image* images, int32_t batch, int32_t h, int32_t w,
                      uint8_t* mosaic_ws, float* out, void* stream);
size_t yxh_sizeof_aug_image(void);

/*
 * yxh_postprocess: utils.postprocess (utils/boxes.py:31-75) with torchvision
 * nms / batched_nms semantics (CPU branch rule: boxes.numel() > vanilla_numel ->
 * per-class NMS, else coordinate-offset NMS) on device.
 *   pred      [B, A, 5+C] fp32, converted to xyxy IN PLACE (boxes.py:32-37)
 *   det       [B, A, 7] fp32 out: rows [x1,y1,x2,y2,obj,cls_conf,cls_idx] in keep order
 *   counts    [B] int32 out: detections per image (0 == the reference's None)
 *   workspace >= yxh_postprocess_workspace_bytes(B, A)
 * Any candidate count (anchors <= 2^19 per image).  The u64 suppression matrix is built
 * and consumed in passes of R sorted rows x ceil(A/64) words per image, R chosen so one
 * pass holds at most the mask budget (320 MiB over the batch), so the workspace grows
 * linearly in A for large inputs instead of quadratically.
 */
size_t yxh_postprocess_workspace_bytes(int32_t batch, int32_t anchors);
/* Process-wide mask budget in bytes (0 = the 320 MiB default).  Changes the workspace size
 * and the pass count of later calls; tests use a tiny budget to force many passes. */
void yxh_set_nms_mask_budget(size_t bytes);
int yxh_postprocess(float* pred, int32_t batch, int32_t anchors, int32_t num_classes,
                    float conf_thre, double nms_thre, int32_t class_agnostic,
                    int64_t vanilla_numel, float* det, int32_t* counts, void* workspace,
                    size_t workspace_bytes, void* stream);
/* The same, recording `filter_done` (a hipEvent_t, may be NULL) on `stream` as soon as the
 * filter pass has read `pred` and written its xyxy columns: every later pass reads only the
 * workspace, so a producer may overwrite `pred` once that event has fired (a serving loop
 * runs the next batch's forward beside this batch's NMS). */
int yxh_postprocess_ev(float* pred, int32_t batch, int32_t anchors, int32_t num_classes,
                       float conf_thre, double nms_thre, int32_t class_agnostic,
                       int64_t vanilla_numel, float* det, int32_t* counts, void* workspace,
                       size_t workspace_bytes, void* filter_done, void* stream);
/* The same, split over two streams (ABI 17): the count reset and the filter pass on `filter_stream`,
 * `filter_done` (required) recorded there, then `rest_stream` waits on it and runs the sort, gather,
 * mask and reduce passes.  A serving loop passes its forward's stream as `filter_stream`: the next
 * batch's forward follows the filter in stream order while the NMS proper runs beside it.  det /
 * counts / workspace are complete once `rest_stream` reaches them, so the caller must not hand the
 * same workspace to the next batch's filter before then: the Python layer alternates two workspaces
 * (yolox_amd/utils/boxes.py), so a filter waits only on the NMS of the batch two before it. */
int yxh_postprocess_split(float* pred, int32_t batch, int32_t anchors, int32_t num_classes,
                          float conf_thre, double nms_thre, int32_t class_agnostic,
                          int64_t vanilla_numel, float* det, int32_t* counts, void* workspace,
                          size_t workspace_bytes, void* filter_done, void* filter_stream,
                          void* rest_stream);
/* The same passes with the filter fed by the forward's per-anchor score records (ABI 18;
 * yxh_head_desc.scores of the forward that wrote `pred`): one thread per anchor reads its 32-byte
 * record and only writes the row's box as xyxy in place (boxes.py:32-37) -- 32 B read per anchor
 * instead of 340 at 80 classes.  Identical results to yxh_postprocess (the records hold the
 * filter's own fp32 values).  filter_done / rest_stream as yxh_postprocess_ev / _split (either may be
 * NULL; rest_stream needs filter_done).  Workspace contract: this entry point does not reset the
 * per-image candidate counters (no pp_init launch in front of the filter): it expects them zero,
 * which every yxh_postprocess* call leaves them (the final reduce pass zeroes them) and a
 * zero-filled workspace is on its first use. */
int yxh_postprocess_scored(float* pred, const float* scores, int32_t batch, int32_t anchors,
                           int32_t num_classes, float conf_thre, double nms_thre, int32_t class_agnostic,
                           int64_t vanilla_numel, float* det, int32_t* counts, void* workspace,
                           size_t workspace_bytes, void* filter_done, void* filter_stream, void* rest_stream);

/*
 * yxh_yolox_loss: YoloxHead.get_losses (yolo_head.py:253-411) with SimOTA assignment
 * (get_assignments :420-509, get_geometry_constraint :511-540, simota_matching
 * :542-574) and IouLoss (losses.py:13-51) for the whole batch, no host sync.
 *   preds   [B, A, 5+C] fp32 train-mode head output: decoded cx,cy,w,h, raw obj/cls logits
 *   origin  [B, A, 4] raw reg outputs for the L1 loss, or NULL (use_l1 = False)
 *   labels  [B, L, 5] (cls, cx, cy, w, h), zero rows after the GTs
 *   level_hw [nlev][2], strides [nlev]: anchor grid (anchors level-major, row-major)
 *   out: fg_mask [B, A] u8, matched_gt [B, A] int32 (-1 = background), pred_iou [B, A],
 *        num_fg [B] int32, losses[6] = total, 5*iou, obj, cls, l1, num_fg/max(num_gts,1)
 */
size_t yxh_yolox_loss_workspace_bytes(int32_t batch, int32_t anchors, int32_t max_labels);
int yxh_yolox_loss(const float* preds, const float* origin, const float* labels, int32_t batch,
                   int32_t anchors, int32_t num_classes, int32_t max_labels, const int32_t* level_hw,
                   const int32_t* strides, int32_t nlevels, uint8_t* fg_mask, int32_t* matched_gt,
                   float* pred_iou, int32_t* num_fg, float* losses, void* workspace,
                   size_t workspace_bytes, void* stream);

/* ============================================================== training
 * The backward pass of YoloxModule (train mode): BaseConv = conv -> BatchNorm2d (batch
 * statistics) -> act, and its gradients.  Data gradients of convolutions run on
 * yxh_conv2d with yxh_pack_dgrad_weight's transposed, flipped weights (stride 2: the
 * gradient source with upsample == 2) and YXH_CONV_ACCUMULATE into fp32 gradient
 * buffers.  Views (yxh_src) give channel slices of wider buffers; `batch` images of
 * h x w pixels each.  Activation gradients are fp32; activations are `dtype`.
 */

/* Workspace for the per-channel reductions below (channels C). */
size_t yxh_reduce_workspace_bytes(int32_t channels);

/*
 * yxh_bn_stats: BatchNorm2d.forward in training mode (network_blocks.py:44-49,
 * eps / momentum config.py:162-166) over the raw conv output y: per-channel mean and
 * biased variance, stats[4][C] = mean, invstd, gamma*invstd, beta - mean*gamma*invstd;
 * running_mean / running_var (may both be NULL) updated with `momentum` and the
 * unbiased variance, as torch does.
 */
int yxh_bn_stats(int32_t dtype, int32_t batch, const yxh_src* y, const float* gamma, const float* beta,
                 float* running_mean, float* running_var, float eps, float momentum, float* stats,
                 void* workspace, size_t workspace_bytes, void* stream);

/* out = act(y * scale + shift) (+ residual, network_blocks.py:97-99). */
int yxh_bn_act_fwd(int32_t dtype, int32_t batch, const yxh_src* y, const float* stats, int32_t act,
                   const yxh_src* residual, const yxh_src* out, void* stream);

/*
 * Backward of act(BN(y)): dout fp32 view -> dgamma, dbeta (fp32 [C]) and the conv
 * output gradient dx (`dtype`, dense [batch*h*w][C]).
 */
int yxh_bn_act_bwd(int32_t dtype, int32_t batch, const yxh_src* y, const yxh_src* dout, const float* stats,
                   const float* gamma, int32_t act, float* dgamma, float* dbeta, void* dx, void* workspace,
                   size_t workspace_bytes, void* stream);

/* out[c] = sum over pixels of x[c] (bias gradients of the head's pred convs). */
int yxh_channel_sum(int32_t dtype, int32_t batch, const yxh_src* x, float* out, void* workspace,
                    size_t workspace_bytes, void* stream);

/*
 * yxh_conv_wgrad: weight gradient of Conv2d (autograd of network_blocks.py:48 and the
 * head's preds, yolo_head.py:149-160) on MFMA: dw[cout][cin_store][kh][kw] (torch layout,
 * fp32) += sum over output pixels of dy[cout] * x[cin](tap).  dw must be zeroed by the
 * caller (split-K over pixel ranges with fp32 atomics).  src: the forward's input views
 * (1-2 sources, nearest-x2 allowed); dy.channels >= cout, padded to 16-byte chunks.
 */
typedef struct {
    int32_t dtype, batch, in_h, in_w, out_h, out_w, cin, cout, kh, kw, stride, pad;
    int32_t nsrc, cin_store; /* cin_store <= cin: dw's input-channel extent (Focus: 12 of 16) */
    yxh_src src[2];
    yxh_src dy;
    float* dw;
    int32_t tile, reserved;  /* tile 0: by shape; 17-20 (fp32, any kernel / stride): k-major MFMA operands,
                                one tap per block, 64x64, 128x128,
                                128x64, 64x128; 1-4: 64x64, 128x128, 32x64, 16x64 (cout x cin,
                                register-transposed loader); 5-10 (bf16/f16): LDS-DMA +
                                ds_read_b64_tr_b16, 128x128 (3 / 2 buffers), 64x64 (3 / 2),
                                128x64, 64x128 */
    /* fp32 tiles 17-20: optional scratch for per-split partial gradients; with it the splits are
     * summed by a second launch in a fixed order (deterministic, no atomics) */
    float* workspace;
    int64_t workspace_bytes;
} yxh_wgrad_desc;
int yxh_conv_wgrad(const yxh_wgrad_desc* d, void* stream);

/*
 * yxh_pack_dgrad_weight: [cout][cin][kh][kw] fp32 -> [c_count][kh][kw][cout_pad] `dtype`
 * with flipped taps for input channels [c_begin, c_begin + c_count): the weights of the
 * data-gradient conv (zeros in [cout, cout_pad)).
 */
int yxh_pack_dgrad_weight(const float* w, int32_t cout, int32_t cin, int32_t kh, int32_t kw, int32_t c_begin,
                          int32_t c_count, int32_t cout_pad, int32_t dtype, void* out, void* stream);

/*
 * yxh_pack_frag: packed conv weights [cout][taps][cin] (16-bit) -> the MFMA fragment-major
 * layout the weight-stationary conv tiles read: 1 KiB blocks (16 output channels x 32 input
 * channels of one tap), block (nf, tap, kb) at ((nf * taps + tap) * cin/32 + kb) KiB, lane
 * l = 16 * q + r of a 16x16x32 MFMA operand at byte 16 * l of its block holding channel
 * 16 nf + r, inputs 32 kb + 8 q .. + 8.  cout % 16 == 0, cin % 32 == 0.
 */
int yxh_pack_frag(const void* w, int32_t cout, int32_t taps, int32_t cin, int32_t dtype, void* out, void* stream);

/*
 * yxh_pack_weights_batch: every weight repack of one training step in ONE launch (the
 * optimizer rewrites conv.weight each step, core/trainer.py:109-115, so the packed
 * forward / data-gradient layouts are rebuilt before the next forward).  jobs: a DEVICE
 * array of njobs descriptors, ordered by block0 (the job's first block of 256 elements;
 * block0 + ceil(elements / 256) is the next job's block0, total_blocks after the last).
 *   kind YXH_PACK_FWD  : yxh_fold_bn_pack without BN: [cout][kh][kw][pad] (pad = cin_pad >=
 *                        cin, zeros beyond cin) + bias_out[cout] = conv bias or 0 (bias_out
 *                        may be NULL)
 *   kind YXH_PACK_DGRAD: yxh_pack_dgrad_weight for input channels [c_begin, c_begin +
 *                        c_count): [c_count][kh][kw][pad] (pad = cout_pad), taps flipped
 * Results are bit-identical to the per-conv entry points.
 */
#define YXH_PACK_FWD 0
#define YXH_PACK_DGRAD 1
typedef struct {
    const float* w;    /* [cout][cin][kh][kw] fp32 */
    const float* cb;   /* conv bias [cout] or NULL (FWD) */
    void* out;         /* packed weights, `dtype` */
    float* bias_out;   /* FWD: [cout] or NULL */
    int32_t kind, cout, cin, kh, kw, pad, c_begin, c_count;
    int32_t block0, reserved;
} yxh_pack_job;
int yxh_pack_weights_batch(const yxh_pack_job* jobs, int32_t njobs, int32_t total_blocks, int32_t dtype,
                           void* stream);

/*
 * yxh_spp_bwd: SPPBottleneck concat + max_pool2d(5, 9, 13) backward
 * (network_blocks.py:137-141): cat holds x in channels [0, c); dcat fp32 dense
 * [batch*h*w][4c]; dx fp32 dense [batch*h*w][c] = dcat[:, :c] + pooled-argmax gradients.
 */
int yxh_spp_bwd(int32_t dtype, int32_t batch, const yxh_src* cat, int32_t c, const float* dcat, float* dx,
                void* stream);

/* nn.Upsample(nearest, x2) backward: dst[B,h,w,C] += 2x2 sums of g[B,2h,2w,C] (fp32). */
int yxh_upsample_bwd(const float* g, int32_t batch, int32_t h, int32_t w, int32_t c, float* dst, void* stream);

/*
 * ABI 16, depthwise conv gradients (DWConv.dconv of yolox_nano, network_blocks.py:55-74: Conv2d with
 * groups = channels, 3x3, stride 1 or 2, pad 1; the autograd of F.conv2d(groups=C) in the train step).
 * yxh_dw_wgrad: dw[c][ky][kx] (fp32, torch's [C][1][3][3]) = sum over the batch's output pixels of
 *   dy[c] * x[c](tap), WRITTEN (not accumulated); x: the forward's input view, dy: a view at the
 *   output size.  Per-block partials in `workspace` (yxh_dw_wgrad_workspace_bytes), summed by a
 *   second launch in a fixed order: deterministic.
 * yxh_dw_dgrad: dx[b][iy][ix][c] (fp32 view, 16-byte aligned dy rows) = (accumulate ? dx : 0) +
 *   sum over taps of dy[b][oy][ox][c] * w[c][tap], iy = oy * stride - pad + ky; w: the forward's
 *   packed weights [C][3][3] in `dtype` (yxh_fold_bn_pack with cin_pad 1).
 */
size_t yxh_dw_wgrad_workspace_bytes(int32_t batch, int32_t out_h, int32_t out_w, int32_t channels, int32_t k);
int yxh_dw_wgrad(int32_t dtype, int32_t batch, const yxh_src* x, const yxh_src* dy, int32_t channels, int32_t k,
                 int32_t stride, int32_t pad, int32_t out_h, int32_t out_w, float* dw, void* workspace,
                 size_t workspace_bytes, void* stream);
int yxh_dw_dgrad(int32_t dtype, int32_t batch, const yxh_src* dy, const void* w, int32_t channels, int32_t k,
                 int32_t stride, int32_t pad, int32_t in_h, int32_t in_w, float* dx, int32_t dx_cstride,
                 int64_t dx_bstride, int32_t accumulate, void* stream);

/*
 * ABI 16, yxh_resize_bilinear: YoloxConfig.preprocess's multiscale resize (config.py:296-305),
 * F.interpolate(x, size=(out_h, out_w), mode="bilinear", align_corners=False) of a dense NCHW
 * batch [batch][channels][in_h][in_w] in `dtype` (f32 / bf16 / f16) into [batch][channels][out_h]
 * [out_w]: ATen's bilinear arithmetic term for term in fp32 (scale = in / out, source index
 * clamped at 0, the +1 neighbour clamped at the border), one rounding to `dtype`.
 */
int yxh_resize_bilinear(int32_t dtype, int32_t batch, int32_t channels, int32_t in_h, int32_t in_w, const void* src,
                        int32_t out_h, int32_t out_w, void* dst, void* stream);

/*
 * yxh_head_decode_train: YoloxHead.get_output_and_grid (yolo_head.py:213-231) on the
 * raw pred-conv outputs raw[B, A, 5+C] (fp32): out = raw with ch 0-1 -> (v + grid) *
 * stride and ch 2-3 -> exp(v) * stride.
 */
int yxh_head_decode_train(const float* raw, int32_t batch, int32_t anchors, int32_t num_classes,
                          const int32_t* level_hw, const int32_t* strides, int32_t nlevels, float* out,
                          void* stream);

/*
 * yxh_yolox_loss_bwd: gradient of losses[0] (total_loss of yxh_yolox_loss) w.r.t. the raw
 * pred-conv outputs, given the assignment that call produced (autograd of
 * yolo_head.py:382-402, losses.py:13-51, through the decode of :227-230).
 * grad_total: device fp32 scalar dL/d(total_loss) (e.g. 1 or the loss scale).
 * out (`dtype`): g_regobj [B*A][8] (ch 0-3 reg, 4 obj, 5-7 zero), g_cls [B*A][C].
 */
int yxh_yolox_loss_bwd(const float* preds, const float* raw, const float* labels, int32_t batch,
                       int32_t anchors, int32_t num_classes, int32_t max_labels, const int32_t* level_hw,
                       const int32_t* strides, int32_t nlevels, const uint8_t* fg_mask,
                       const int32_t* matched_gt, const float* pred_iou, const int32_t* num_fg,
                       const float* grad_total, int32_t use_l1, int32_t dtype, void* g_regobj, void* g_cls,
                       void* stream);

/*
 * Plan execution.  A forward pass is a fixed list of ops (built once per model and
 * input shape by the Python planner) executed back-to-back on one stream, or
 * captured once into a hipGraph and replayed (the MI355X replacement for the
 * reference's eager per-module dispatch).
 */
enum yxh_op_kind { YXH_OP_CONV = 0, YXH_OP_FOCUS = 1, YXH_OP_SPP = 2, YXH_OP_STEM = 3, YXH_OP_HEAD = 4,
                   YXH_OP_STEM2 = 5 };
typedef struct {
    const void* img;
    int32_t layout, img_dtype, batch, h, w, dst_dtype;
    void* dst;
} yxh_focus_desc;
typedef struct {
    void* buf;
    int32_t dtype, batch, h, w, c, cstride;
    int64_t bstride;
} yxh_spp_desc;
/* One head level's reg_preds + obj_preds + cls_preds (1x1, with bias) + cat + sigmoid +
 * decode (yolo_head.py:149-160, 185-187, 205-207, 233-251) in one launch: rows
 * [a_off, a_off + h*w) of every image of the fp32 [B, A, 5+C] output (out_bstride =
 * A*(5+C)).  w_reg [5][cin] (reg 4 + obj 1) / w_cls [C][cin] in `dtype`, fp32 biases.
 * train = 1: obj/cls stay logits (get_output_and_grid, :213-231); train = 2 (ABI 16): the
 * eval rows without the box decode (decode_in_inference = False, :208-211): reg raw, obj/cls
 * sigmoid.
 * scores (ABI 18, NULL = none; eval decode rows (train = 0) of the 64 / 128 / 256-channel 16-bit levels
 * only): per anchor 8 floats {obj * max class, max class, its index, obj, cx, cy, w, h} -- the fp32
 * values utils.postprocess's filter computes from the row (boxes.py:46-48: first maximum, obj *
 * conf) and the row's box, from the same registers -- at [image][a_off + pixel], image stride
 * out_bstride / (5 + C) anchors.  yxh_postprocess_scored reads these 32 bytes instead of the row. */
typedef struct {
    int32_t dtype, batch, h, w, cin, num_classes;
    yxh_src reg, cls;
    const void* w_reg;
    const float* b_reg;
    const void* w_cls;
    const float* b_cls;
    float* out;
    int64_t out_bstride;
    int32_t a_off;
    float stride;
    int32_t train;
    int32_t reserved;
    float* scores;
} yxh_head_desc;
int yxh_head_pred(const yxh_head_desc* d, void* stream);

typedef struct {
    int32_t kind;
    int32_t reserved;
    union {
        yxh_conv_desc conv;
        yxh_focus_desc focus;
        yxh_spp_desc spp;
        yxh_stem_desc stem;
        yxh_head_desc head;
        yxh_stem2_desc stem2;
    } u;
} yxh_op;

int yxh_run_ops(const yxh_op* ops, int32_t n, void* stream);
int yxh_graph_create(const yxh_op* ops, int32_t n, void* stream, void** graph_exec);
/* yxh_graph_create_lanes: capture the op list with independent branches on separate
 * streams ("lanes"): op i runs on lane lanes[i] after every op listed in
 * deps[dep_off[i] .. dep_off[i+1]) (indices < i); cross-lane dependencies become graph
 * edges, same-lane order is stream order.  Lane 0 forks the others at the start and
 * joins them at the end.  Used to overlap the three head levels with each other and
 * with the PAFPN bottom-up path (yolo_head.py:140-211 runs the levels independently).
 * At most 8 lanes (EINVAL above: the most a GPU test replays; round 2's 7-stream crash is
 * unexplained, runtime.cpp -- past 8 use yxh_graph_create_dag). */
int yxh_graph_create_lanes(const yxh_op* ops, int32_t n, const int32_t* lanes, const int32_t* dep_off,
                           const int32_t* deps, int32_t nlanes, void* stream, void** graph_exec);
/* yxh_graph_create_dag: the op list as its dataflow DAG -- op i is one graph node (the
 * op captured alone) whose predecessors are the ops deps[dep_off[i] .. dep_off[i+1])
 * (indices < i).  No lanes: every independent pair of ops may run concurrently (head
 * levels, batch chunks planned on arenas of their own). */
int yxh_graph_create_dag(const yxh_op* ops, int32_t n, const int32_t* dep_off, const int32_t* deps,
                         void* stream, void** graph_exec);
int yxh_graph_launch(void* graph_exec, void* stream);
int yxh_graph_destroy(void* graph_exec);

/* ---------------------------------------------------------------- optimizer step
 * yxh_sgd_ema_step: one fused pass = torch.optim.SGD.step (momentum, nesterov, per-group
 * weight decay, dampening 0) + ModelEMA.update, replacing the reference's
 * `scaler.step(optimizer)` + `ema_model.update(model)` (core/trainer.py:124-127,
 * config.py:307-333, utils/ema.py:46-58).  segs: device array of segments (one per
 * parameter, plus EMA-only segments with param == NULL for floating buffers); chunks:
 * device int32 pairs {segment, chunk index} covering every segment in chunks of
 * yxh_opt_chunk_elems() elements.  All arrays fp32.  first_step: momentum buffers are
 * initialised to the (decayed) gradient, as torch does when a parameter has no
 * momentum_buffer yet. */
typedef struct yxh_opt_seg {
    float* param;       /* updated in place; NULL: EMA-only segment */
    const float* grad;  /* param's gradient (unscaled in place when amp_scale is set) */
    float* buf;         /* momentum buffer */
    float* ema;         /* EMA copy (NULL: none) */
    const float* src;   /* EMA source of an EMA-only segment */
    int64_t n;          /* elements */
    float weight_decay;
    int32_t group;      /* index into yxh_opt_hparams.lr */
} yxh_opt_seg;

typedef struct yxh_opt_hparams {
    float lr[4];        /* per parameter group */
    float momentum;
    float ema_d;        /* ModelEMA decay d for this update */
    float ema_omd;      /* 1 - d (rounded from double like torch's alpha) */
    int32_t nesterov;
    int32_t first_step;
    int32_t do_ema;
    int32_t reserved;
    const float* amp_scale;      /* GradScaler scale (device fp32) or NULL: gradients are
                                    unscaled in place by float(1/double(scale)) first */
    const float* amp_found_inf;  /* device flag from yxh_amp_found_inf: != 0 skips the SGD
                                    update (the EMA update still runs, as trainer.py:126-127) */
} yxh_opt_hparams;

int yxh_opt_chunk_elems(void);
int yxh_sgd_ema_step(const yxh_opt_seg* segs, const int32_t* chunks, int32_t nchunks,
                     const yxh_opt_hparams* hp, void* stream);

/* GradScaler on the device (torch.amp.GradScaler step/update, core/trainer.py:111-114),
 * no host sync: yxh_amp_found_inf sets *found_inf = 1 if any parameter segment's gradient
 * is non-finite (else 0); yxh_amp_update_scale is torch._amp_update_scale_ (scale *=
 * backoff on inf, else *= growth every growth_interval clean steps). */
int yxh_amp_found_inf(const yxh_opt_seg* segs, const int32_t* chunks, int32_t nchunks, float* found_inf,
                      void* stream);
int yxh_amp_update_scale(float* scale, int32_t* growth_tracker, const float* found_inf, double growth_factor,
                         double backoff_factor, int32_t growth_interval, void* stream);

/* ---------------------------------------------------------------- box mAP (host)
 * yxh_coco_eval: COCO bbox evaluation as the reference's CocoEvalOpt runs it
 * (yolox/layers/fast_coco_eval_api.py:24-149): pycocotools computeIoU (bbox, crowd-aware),
 * the C++ EvaluateImages (yolox/layers/cocoeval/cocoeval.cpp:140-197) and Accumulate
 * (:370-500) in one host call.  Cells p = image * num_categories + category hold ground
 * truths gts[gt_off[p], gt_off[p+1]) and detections dts[dt_off[p], dt_off[p+1]) in any
 * order (detection ids nonzero, as loadRes assigns 1..N).  Outputs (caller-allocated,
 * fp64, -1 where a setting has no valid ground truth): precision and scores
 * [T][R][K][A][M], recall [T][K][A][M] -- CocoEvalOpt.eval's arrays.  Host memory; no
 * device work.  yxh_coco_iou: the [nd][ng] IoU matrix alone. */
typedef struct {
    int64_t id;
    double score;     /* detections */
    double area;      /* the annotation's area (detections: w * h) */
    double box[4];    /* x, y, w, h */
    int32_t is_crowd;
    int32_t ignore;   /* ground truths: pycocotools' ignore (= iscrowd unless set) */
} yxh_coco_instance;
typedef struct {
    int32_t num_images, num_categories, num_area_ranges, num_iou_thresholds, num_recall_thresholds, num_max_dets;
    const double* area_ranges;        /* [A][2] */
    const double* iou_thresholds;     /* [T] */
    const double* recall_thresholds;  /* [R] */
    const int32_t* max_dets;          /* [M] */
} yxh_coco_params;
int yxh_coco_eval(const yxh_coco_params* params, const yxh_coco_instance* gts, const int64_t* gt_off,
                  const yxh_coco_instance* dts, const int64_t* dt_off, double* precision, double* recall,
                  double* scores);
int yxh_coco_iou(const yxh_coco_instance* dts, int32_t nd, const yxh_coco_instance* gts, int32_t ng, double* iou);

int yxh_abi_version(void);
const char* yxh_last_error(void);
size_t yxh_sizeof_op(void);        /* ABI self-check for bindings */
size_t yxh_sizeof_conv_desc(void);

#ifdef __cplusplus
}
#endif
#endif /* YOLOXHIP_H */
