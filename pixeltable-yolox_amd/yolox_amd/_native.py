"""ctypes binding of libyoloxhip.so (include/yoloxhip.h).

The HIP library is the only compute path of this package: there is no CPU or
PyTorch fallback.  If the library is missing or fails to load, every op raises.
torch is imported first so that the library binds to the HIP runtime torch already
loaded (both carry SONAME libamdhip64.so.7), which makes torch's stream handles and
device pointers valid here.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (must precede loading the HIP library)

LIB_PATH = os.environ.get(
    "YOLOX_AMD_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libyoloxhip.so"))

ABI_VERSION = 18

# enums (yoloxhip.h)
OK, EINVAL, EHIP, EUNSUPPORTED = 0, -1, -2, -3
F32, BF16, F16, U8 = 0, 1, 2, 3
ACT_NONE, ACT_SILU, ACT_RELU, ACT_LRELU, ACT_DECODE, ACT_DECODE_TRAIN, ACT_DECODE_RAW = range(7)
NCHW, NHWC = 0, 1
OP_CONV, OP_FOCUS, OP_SPP, OP_STEM, OP_HEAD, OP_STEM2 = 0, 1, 2, 3, 4, 5
LB_F32_NCHW, LB_U8_NHWC, LB_BF16_NHWC = 0, 1, 2

TORCH_DTYPE = {F32: torch.float32, BF16: torch.bfloat16, F16: torch.float16, U8: torch.uint8}
DTYPE_CODE = {v: k for k, v in TORCH_DTYPE.items()}
ACT_CODE = {"silu": ACT_SILU, "relu": ACT_RELU, "lrelu": ACT_LRELU, None: ACT_NONE, "none": ACT_NONE}


class Src(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("channels", C.c_int32), ("cstride", C.c_int32),
                ("bstride", C.c_int64), ("h", C.c_int32), ("w", C.c_int32),
                ("upsample", C.c_int32), ("reserved", C.c_int32)]


class ConvDesc(C.Structure):
    _fields_ = [("dtype", C.c_int32), ("batch", C.c_int32), ("in_h", C.c_int32), ("in_w", C.c_int32),
                ("out_h", C.c_int32), ("out_w", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32),
                ("kh", C.c_int32), ("kw", C.c_int32), ("stride", C.c_int32), ("pad", C.c_int32),
                ("groups", C.c_int32), ("nsrc", C.c_int32), ("src", Src * 2), ("weight", C.c_void_p),
                ("bias", C.c_void_p), ("residual", C.c_void_p), ("res_cstride", C.c_int32),
                ("dst_dtype", C.c_int32), ("res_bstride", C.c_int64), ("dst", C.c_void_p),
                ("dst_cstride", C.c_int32), ("act", C.c_int32), ("dst_bstride", C.c_int64),
                ("decode_stride", C.c_float), ("decode_coff", C.c_int32), ("tile", C.c_int32),
                ("flags", C.c_int32), ("grid_cap", C.c_int32), ("pre_weight", C.c_void_p), ("pre_bias", C.c_void_p),
                ("weight_frag", C.c_void_p), ("post_weight", C.c_void_p), ("post_bias", C.c_void_p),
                ("post_src", Src), ("post_dst", C.c_void_p), ("post_cout", C.c_int32),
                ("post_dst_cstride", C.c_int32), ("post_dst_bstride", C.c_int64), ("post_weight2", C.c_void_p),
                ("post_bias2", C.c_void_p), ("post_cout2", C.c_int32), ("post_stride", C.c_float)]


CONV_ACCUMULATE = 1
CONV_GROUPS2 = 2
CONV_POST_STORE = 4


class OptSeg(C.Structure):
    _fields_ = [("param", C.c_void_p), ("grad", C.c_void_p), ("buf", C.c_void_p), ("ema", C.c_void_p),
                ("src", C.c_void_p), ("n", C.c_int64), ("weight_decay", C.c_float), ("group", C.c_int32)]


class OptHparams(C.Structure):
    _fields_ = [("lr", C.c_float * 4), ("momentum", C.c_float), ("ema_d", C.c_float), ("ema_omd", C.c_float),
                ("nesterov", C.c_int32), ("first_step", C.c_int32), ("do_ema", C.c_int32), ("reserved", C.c_int32),
                ("amp_scale", C.c_void_p), ("amp_found_inf", C.c_void_p)]


class CocoInstance(C.Structure):
    _fields_ = [("id", C.c_int64), ("score", C.c_double), ("area", C.c_double), ("box", C.c_double * 4),
                ("is_crowd", C.c_int32), ("ignore", C.c_int32)]


class CocoParams(C.Structure):
    _fields_ = [("num_images", C.c_int32), ("num_categories", C.c_int32), ("num_area_ranges", C.c_int32),
                ("num_iou_thresholds", C.c_int32), ("num_recall_thresholds", C.c_int32),
                ("num_max_dets", C.c_int32), ("area_ranges", C.c_void_p), ("iou_thresholds", C.c_void_p),
                ("recall_thresholds", C.c_void_p), ("max_dets", C.c_void_p)]


class WgradDesc(C.Structure):
    _fields_ = [("dtype", C.c_int32), ("batch", C.c_int32), ("in_h", C.c_int32), ("in_w", C.c_int32),
                ("out_h", C.c_int32), ("out_w", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32),
                ("kh", C.c_int32), ("kw", C.c_int32), ("stride", C.c_int32), ("pad", C.c_int32),
                ("nsrc", C.c_int32), ("cin_store", C.c_int32), ("src", Src * 2), ("dy", Src),
                ("dw", C.c_void_p), ("tile", C.c_int32), ("reserved", C.c_int32), ("workspace", C.c_void_p),
                ("workspace_bytes", C.c_int64)]


class FocusDesc(C.Structure):
    _fields_ = [("img", C.c_void_p), ("layout", C.c_int32), ("img_dtype", C.c_int32), ("batch", C.c_int32),
                ("h", C.c_int32), ("w", C.c_int32), ("dst_dtype", C.c_int32), ("dst", C.c_void_p)]


class SppDesc(C.Structure):
    _fields_ = [("buf", C.c_void_p), ("dtype", C.c_int32), ("batch", C.c_int32), ("h", C.c_int32),
                ("w", C.c_int32), ("c", C.c_int32), ("cstride", C.c_int32), ("bstride", C.c_int64)]


class StemDesc(C.Structure):
    _fields_ = [("img", C.c_void_p), ("layout", C.c_int32), ("img_dtype", C.c_int32), ("batch", C.c_int32),
                ("h", C.c_int32), ("w", C.c_int32), ("dtype", C.c_int32), ("cout", C.c_int32), ("act", C.c_int32),
                ("weight", C.c_void_p), ("bias", C.c_void_p), ("dst", C.c_void_p), ("dst_cstride", C.c_int32),
                ("reserved", C.c_int32), ("dst_bstride", C.c_int64)]


class Stem2Desc(C.Structure):
    _fields_ = [("img", C.c_void_p), ("layout", C.c_int32), ("img_dtype", C.c_int32), ("batch", C.c_int32),
                ("h", C.c_int32), ("w", C.c_int32), ("dtype", C.c_int32), ("c1", C.c_int32), ("c2", C.c_int32),
                ("act", C.c_int32), ("w1", C.c_void_p), ("b1", C.c_void_p), ("w2", C.c_void_p), ("b2", C.c_void_p),
                ("dst", C.c_void_p), ("dst_cstride", C.c_int32), ("reserved", C.c_int32), ("dst_bstride", C.c_int64),
                ("w3", C.c_void_p), ("b3", C.c_void_p), ("dst3", C.c_void_p), ("dst3_cstride", C.c_int32),
                ("reserved3", C.c_int32), ("dst3_bstride", C.c_int64), ("w4", C.c_void_p), ("b4", C.c_void_p),
                ("dst4", C.c_void_p), ("dst4_cstride", C.c_int32), ("reserved4", C.c_int32),
                ("dst4_bstride", C.c_int64)]


class AugImage(C.Structure):
    """yxh_aug_image (include/yoloxhip.h): one training sample's drawn augmentation."""
    _fields_ = [("mosaic", C.c_int32), ("mix", C.c_int32), ("flip", C.c_int32), ("do_hsv", C.c_int32),
                ("hsv", C.c_int32 * 3), ("cp_flip", C.c_int32), ("src_off", C.c_int64 * 4),
                ("src_h", C.c_int32 * 4), ("src_w", C.c_int32 * 4), ("rh", C.c_int32 * 4), ("rw", C.c_int32 * 4),
                ("rsx", C.c_double * 4), ("rsy", C.c_double * 4), ("lx1", C.c_int32 * 4), ("ly1", C.c_int32 * 4),
                ("lx2", C.c_int32 * 4), ("ly2", C.c_int32 * 4), ("sx1", C.c_int32 * 4), ("sy1", C.c_int32 * 4),
                ("minv", C.c_double * 6), ("cp_off", C.c_int64), ("cp_h", C.c_int32), ("cp_w", C.c_int32),
                ("cp_rh", C.c_int32), ("cp_rw", C.c_int32), ("cp_sx", C.c_double), ("cp_sy", C.c_double),
                ("jit_h", C.c_int32), ("jit_w", C.c_int32), ("jit_sx", C.c_double), ("jit_sy", C.c_double),
                ("x_off", C.c_int32), ("y_off", C.c_int32)]


class HeadDesc(C.Structure):
    _fields_ = [("dtype", C.c_int32), ("batch", C.c_int32), ("h", C.c_int32), ("w", C.c_int32), ("cin", C.c_int32),
                ("num_classes", C.c_int32), ("reg", Src), ("cls", Src), ("w_reg", C.c_void_p), ("b_reg", C.c_void_p),
                ("w_cls", C.c_void_p), ("b_cls", C.c_void_p), ("out", C.c_void_p), ("out_bstride", C.c_int64),
                ("a_off", C.c_int32), ("stride", C.c_float), ("train", C.c_int32), ("reserved", C.c_int32),
                ("scores", C.c_void_p)]


class PackJob(C.Structure):
    """yxh_pack_job (include/yoloxhip.h): one repack of yxh_pack_weights_batch."""
    _fields_ = [("w", C.c_void_p), ("cb", C.c_void_p), ("out", C.c_void_p), ("bias_out", C.c_void_p),
                ("kind", C.c_int32), ("cout", C.c_int32), ("cin", C.c_int32), ("kh", C.c_int32), ("kw", C.c_int32),
                ("pad", C.c_int32), ("c_begin", C.c_int32), ("c_count", C.c_int32), ("block0", C.c_int32),
                ("reserved", C.c_int32)]


PACK_FWD, PACK_DGRAD = 0, 1


class _OpU(C.Union):
    _fields_ = [("conv", ConvDesc), ("focus", FocusDesc), ("spp", SppDesc), ("stem", StemDesc), ("head", HeadDesc),
                ("stem2", Stem2Desc)]


class Op(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_int32), ("u", _OpU)]


_lib = None
_lock = threading.Lock()


class NativeError(RuntimeError):
    pass


def lib():
    """Load (once) and return the HIP library; raise loudly if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"libyoloxhip.so not found at {LIB_PATH}; build it with "
                "`make -C pixeltable-yolox_amd` (or __graft_entry__.build()). "
                "yolox_amd has no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        vp, i32, i64, f32, f64, sz = C.c_void_p, C.c_int32, C.c_int64, C.c_float, C.c_double, C.c_size_t
        sig = {
            "yxh_abi_version": ([], C.c_int),
            "yxh_last_error": ([], C.c_char_p),
            "yxh_sizeof_op": ([], sz),
            "yxh_sizeof_conv_desc": ([], sz),
            "yxh_conv2d": ([C.POINTER(ConvDesc), vp], C.c_int),
            "yxh_head_pred": ([C.POINTER(HeadDesc), vp], C.c_int),
            "yxh_focus_pack": ([vp, i32, i32, i32, i32, i32, vp, i32, vp], C.c_int),
            "yxh_spp_maxpool": ([vp, i32, i32, i32, i32, i32, i32, i64, vp], C.c_int),
            "yxh_stem_conv": ([C.POINTER(StemDesc), vp], C.c_int),
            "yxh_stem_s2": ([C.POINTER(Stem2Desc), vp], C.c_int),
            "yxh_stem_pack": ([vp, vp, vp, vp, vp, f32, i32, i32, vp, vp, vp], C.c_int),
            "yxh_fold_bn_pack": ([vp, vp, vp, vp, vp, vp, f32, i32, i32, i32, i32, i32, i32, vp, vp, vp],
                                 C.c_int),
            "yxh_letterbox_batch": ([vp, vp, i32, i32, i32, i32, vp, vp], C.c_int),
            "yxh_augment_batch": ([vp, vp, i32, i32, i32, vp, vp, vp], C.c_int),
            "yxh_sizeof_aug_image": ([], sz),
            "yxh_postprocess_workspace_bytes": ([i32, i32], sz),
            "yxh_set_nms_mask_budget": ([sz], None),
            "yxh_postprocess": ([vp, i32, i32, i32, f32, f64, i32, i64, vp, vp, vp, sz, vp], C.c_int),
            "yxh_postprocess_ev": ([vp, i32, i32, i32, f32, f64, i32, i64, vp, vp, vp, sz, vp, vp], C.c_int),
            "yxh_postprocess_split": ([vp, i32, i32, i32, f32, f64, i32, i64, vp, vp, vp, sz, vp, vp, vp], C.c_int),
            "yxh_postprocess_scored": ([vp, vp, i32, i32, i32, f32, f64, i32, i64, vp, vp, vp, sz, vp, vp, vp], C.c_int),
            "yxh_yolox_loss_workspace_bytes": ([i32, i32, i32], sz),
            "yxh_yolox_loss": ([vp, vp, vp, i32, i32, i32, i32, vp, vp, i32, vp, vp, vp, vp, vp, vp, sz, vp],
                               C.c_int),
            "yxh_reduce_workspace_bytes": ([i32], sz),
            "yxh_bn_stats": ([i32, i32, C.POINTER(Src), vp, vp, vp, vp, f32, f32, vp, vp, sz, vp], C.c_int),
            "yxh_bn_act_fwd": ([i32, i32, C.POINTER(Src), vp, i32, C.POINTER(Src), C.POINTER(Src), vp], C.c_int),
            "yxh_bn_act_bwd": ([i32, i32, C.POINTER(Src), C.POINTER(Src), vp, vp, i32, vp, vp, vp, vp, sz, vp],
                               C.c_int),
            "yxh_channel_sum": ([i32, i32, C.POINTER(Src), vp, vp, sz, vp], C.c_int),
            "yxh_conv_wgrad": ([C.POINTER(WgradDesc), vp], C.c_int),
            "yxh_pack_dgrad_weight": ([vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp], C.c_int),
            "yxh_pack_weights_batch": ([vp, i32, i32, i32, vp], C.c_int),
            "yxh_pack_frag": ([vp, i32, i32, i32, i32, vp, vp], C.c_int),
            "yxh_spp_bwd": ([i32, i32, C.POINTER(Src), i32, vp, vp, vp], C.c_int),
            "yxh_upsample_bwd": ([vp, i32, i32, i32, i32, vp, vp], C.c_int),
            "yxh_dw_wgrad_workspace_bytes": ([i32, i32, i32, i32, i32], sz),
            "yxh_dw_wgrad": ([i32, i32, C.POINTER(Src), C.POINTER(Src), i32, i32, i32, i32, i32, i32, vp, vp, sz, vp],
                             C.c_int),
            "yxh_dw_dgrad": ([i32, i32, C.POINTER(Src), vp, i32, i32, i32, i32, i32, i32, vp, i32, i64, i32, vp],
                             C.c_int),
            "yxh_resize_bilinear": ([i32, i32, i32, i32, i32, vp, i32, i32, vp, vp], C.c_int),
            "yxh_head_decode_train": ([vp, i32, i32, i32, vp, vp, i32, vp, vp], C.c_int),
            "yxh_yolox_loss_bwd": ([vp, vp, vp, i32, i32, i32, i32, vp, vp, i32, vp, vp, vp, vp, vp, i32, i32, vp,
                                    vp, vp], C.c_int),
            "yxh_opt_chunk_elems": ([], C.c_int),
            "yxh_sgd_ema_step": ([vp, vp, i32, C.POINTER(OptHparams), vp], C.c_int),
            "yxh_amp_found_inf": ([vp, vp, i32, vp, vp], C.c_int),
            "yxh_coco_eval": ([C.POINTER(CocoParams), vp, vp, vp, vp, vp, vp, vp], C.c_int),
            "yxh_coco_iou": ([vp, i32, vp, i32, vp], C.c_int),
            "yxh_amp_update_scale": ([vp, vp, vp, f64, f64, i32, vp], C.c_int),
            "yxh_run_ops": ([C.POINTER(Op), i32, vp], C.c_int),
            "yxh_graph_create": ([C.POINTER(Op), i32, vp, C.POINTER(vp)], C.c_int),
            "yxh_graph_create_lanes": ([C.POINTER(Op), i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), i32,
                                        vp, C.POINTER(vp)], C.c_int),
            "yxh_graph_create_dag": ([C.POINTER(Op), i32, C.POINTER(i32), C.POINTER(i32), vp, C.POINTER(vp)],
                                     C.c_int),
            "yxh_graph_launch": ([vp, vp], C.c_int),
            "yxh_graph_destroy": ([vp], C.c_int),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        if L.yxh_abi_version() != ABI_VERSION:
            raise NativeError(f"ABI mismatch: library {L.yxh_abi_version()} vs binding {ABI_VERSION}")
        if (L.yxh_sizeof_op() != C.sizeof(Op) or L.yxh_sizeof_conv_desc() != C.sizeof(ConvDesc)
                or L.yxh_sizeof_aug_image() != C.sizeof(AugImage)):
            raise NativeError("struct layout mismatch between yoloxhip.h and _native.py")
        _lib = L
    return _lib


EXPORTED = ["yxh_abi_version", "yxh_last_error", "yxh_sizeof_op", "yxh_sizeof_conv_desc", "yxh_conv2d", "yxh_head_pred",
            "yxh_focus_pack", "yxh_spp_maxpool", "yxh_stem_conv", "yxh_stem_s2", "yxh_stem_pack", "yxh_fold_bn_pack", "yxh_letterbox_batch", "yxh_augment_batch", "yxh_sizeof_aug_image", "yxh_postprocess_workspace_bytes", "yxh_set_nms_mask_budget",
            "yxh_postprocess", "yxh_postprocess_ev", "yxh_postprocess_split", "yxh_postprocess_scored", "yxh_yolox_loss_workspace_bytes", "yxh_yolox_loss", "yxh_run_ops", "yxh_graph_create", "yxh_graph_create_lanes", "yxh_graph_create_dag",
            "yxh_graph_launch", "yxh_graph_destroy", "yxh_reduce_workspace_bytes", "yxh_bn_stats", "yxh_bn_act_fwd",
            "yxh_bn_act_bwd", "yxh_channel_sum", "yxh_conv_wgrad", "yxh_pack_dgrad_weight", "yxh_pack_weights_batch", "yxh_pack_frag", "yxh_spp_bwd",
            "yxh_upsample_bwd", "yxh_dw_wgrad_workspace_bytes", "yxh_dw_wgrad", "yxh_dw_dgrad", "yxh_resize_bilinear",
            "yxh_head_decode_train", "yxh_yolox_loss_bwd", "yxh_opt_chunk_elems",
            "yxh_sgd_ema_step", "yxh_amp_found_inf", "yxh_amp_update_scale", "yxh_coco_eval", "yxh_coco_iou"]


def check(rc: int, what: str = "") -> None:
    if rc != OK:
        msg = lib().yxh_last_error().decode(errors="replace")
        kind = {EINVAL: ValueError, EUNSUPPORTED: NotImplementedError}.get(rc, RuntimeError)
        raise kind(f"{what}: {msg} (rc={rc})" if what else f"{msg} (rc={rc})")


def stream_ptr(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(t: torch.Tensor, name: str = "tensor") -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be on a ROCm device (got {t.device})")
