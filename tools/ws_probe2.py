"""Probe (GPU box): time given 3x3 conv shapes with given tiles (HIP events, 20 reps) on the
library YOLOX_AMD_LIB points to (tools/ws_split.sh builds the split probes).
Usage: python tools/ws_probe2.py "S H CIN COUT TILE" ..."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd"))
from yolox_amd import _native as N  # noqa: E402

L = N.lib()
dev = torch.device("cuda:0")
st = N.stream_ptr(dev)
B = 32
tag = os.path.basename(os.environ.get("YOLOX_AMD_LIB", "libyoloxhip.so"))
for spec in sys.argv[1:]:
    S, H, K, Nc, tile = (int(v) for v in spec.split())
    Ho = H // S
    x = torch.randn(B, H, H, K, device=dev).to(torch.bfloat16)
    y = torch.empty(B, Ho, Ho, Nc, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(Nc, 3, 3, K, device=dev) / (9 * K) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Nc, device=dev) * 0.1
    d = N.ConvDesc()
    d.dtype, d.batch = N.BF16, B
    d.in_h, d.in_w, d.out_h, d.out_w = H, H, Ho, Ho
    d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups = K, Nc, 3, 3, S, 1, 1
    d.nsrc = 1
    d.src[0] = N.Src(x.data_ptr(), K, K, H * H * K, H, H, 0, 0)
    d.weight, d.bias = w.data_ptr(), b.data_ptr()
    d.dst, d.dst_dtype, d.dst_cstride, d.dst_bstride = y.data_ptr(), N.BF16, Nc, Ho * Ho * Nc
    d.act, d.tile = N.ACT_SILU, tile
    d.tile = 12  # conv_igemm reference output
    assert L.yxh_conv2d(C.byref(d), st) == N.OK
    torch.cuda.synchronize()
    ref = y.float().clone()
    y.zero_()
    d.tile = tile
    if L.yxh_conv2d(C.byref(d), st) != N.OK:
        print(f"{tag} s{S} {H} {K}->{Nc} tile {tile >> 1}: not applicable", flush=True)
        continue
    torch.cuda.synchronize()
    err = float((y.float() - ref).abs().max() / ref.abs().max())
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        L.yxh_conv2d(C.byref(d), st)
    e.record()
    e.synchronize()
    t = s.elapsed_time(e) / 20 * 1e3
    print(f"{tag} s{S} {H} {K}->{Nc} tile {tile >> 1}: {t:.1f} us {2.0 * B * Ho * Ho * Nc * 9 * K / t / 1e6:.0f} TF"
          f" err {err:.1e}", flush=True)
