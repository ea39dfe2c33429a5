"""One 3x3 conv shape of yolox_s bs32 launched 50x with a fixed tile, for rocprofv3 --pmc
passes (a --pmc run of tools/r3_probe.py; round-3 script retired).  Usage: python tools/r3_pmc.py S H CIN COUT TILE"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd"))
from yolox_amd import _native as N  # noqa: E402

L = N.lib()
dev = torch.device("cuda:0")
st = N.stream_ptr(dev)
S, H, K, Nc, tile = (int(a) for a in sys.argv[1:6])
B = 32
Ho = H // S
x = torch.randn(B, H, H, K, device=dev).to(torch.bfloat16)
y = torch.empty(B, Ho, Ho, Nc, device=dev, dtype=torch.bfloat16)
w = (torch.randn(Nc, 3, 3, K, device=dev) / (9 * K) ** 0.5).to(torch.bfloat16)
b = torch.zeros(Nc, device=dev)
d = N.ConvDesc()
d.dtype, d.batch = N.BF16, B
d.in_h, d.in_w, d.out_h, d.out_w = H, H, Ho, Ho
d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups = K, Nc, 3, 3, S, 1, 1
d.nsrc = 1
d.src[0] = N.Src(x.data_ptr(), K, K, H * H * K, H, H, 0, 0)
d.weight, d.bias = w.data_ptr(), b.data_ptr()
d.dst, d.dst_dtype, d.dst_cstride, d.dst_bstride = y.data_ptr(), N.BF16, Nc, Ho * Ho * Nc
d.act, d.tile = N.ACT_SILU, tile
for _ in range(50):
    N.check(L.yxh_conv2d(C.byref(d), st), "conv")
torch.cuda.synchronize()
print("ok")
