"""One 1x1 conv shape (M=51200, K=N=128, bf16, tile 6 = conv_igemm 64x64) launched 50x,
for rocprofv3 --pmc passes (tools/gpu_pmc.sh).  Run on the GPU box."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd"))
from yolox_amd import _native as N  # noqa: E402

L = N.lib()
dev = torch.device("cuda:0")
st = N.stream_ptr(dev)
M, K, Nc = 51200, 128, 128
tile = int(sys.argv[1]) if len(sys.argv) > 1 else 12
x = torch.randn(M, K, device=dev).to(torch.bfloat16)
y = torch.empty(M, Nc, device=dev, dtype=torch.bfloat16)
w = (torch.randn(Nc, K, device=dev) / K ** 0.5).to(torch.bfloat16)
b = torch.zeros(Nc, device=dev)
d = N.ConvDesc()
d.dtype, d.batch = N.BF16, 1
d.in_h, d.in_w, d.out_h, d.out_w = 1, M, 1, M
d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups = K, Nc, 1, 1, 1, 0, 1
d.nsrc = 1
d.src[0] = N.Src(x.data_ptr(), K, K, M * K, 1, M, 0, 0)
d.weight, d.bias = w.data_ptr(), b.data_ptr()
d.dst, d.dst_dtype, d.dst_cstride, d.dst_bstride = y.data_ptr(), N.BF16, Nc, M * Nc
d.act, d.tile = N.ACT_SILU, tile
for _ in range(50):
    N.check(L.yxh_conv2d(C.byref(d), st), "conv")
torch.cuda.synchronize()
print("ok")
