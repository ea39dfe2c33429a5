"""yxh_head_pred on yolox_s level 0 at bs 32 (80x80, 128 channels, 80 classes, bf16)
launched 50x with HIP-event timing, for rocprofv3 --pmc passes.  Usage: python tools/head_pmc.py"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd"))
from yolox_amd import _native as N  # noqa: E402

L = N.lib()
dev = torch.device("cuda:0")
st = N.stream_ptr(dev)
B, h, w, cin, nc = 32, 80, 80, 128, 80
A = 8400
feats = torch.randn(B, h, w, 2 * cin, device=dev).to(torch.bfloat16)
wro = (torch.randn(5, cin, device=dev) / cin ** 0.5).to(torch.bfloat16)
wcl = (torch.randn(nc, cin, device=dev) / cin ** 0.5).to(torch.bfloat16)
bro, bcl = torch.zeros(5, device=dev), torch.zeros(nc, device=dev)
out = torch.empty(B, A, 5 + nc, device=dev)
d = N.HeadDesc()
d.dtype, d.batch, d.h, d.w, d.cin, d.num_classes = N.BF16, B, h, w, cin, nc
for s, off in ((d.reg, 0), (d.cls, cin)):
    s.ptr = feats.data_ptr() + off * 2
    s.channels, s.cstride, s.bstride, s.h, s.w, s.upsample = cin, 2 * cin, h * w * 2 * cin, h, w, 0
d.w_reg, d.b_reg, d.w_cls, d.b_cls = wro.data_ptr(), bro.data_ptr(), wcl.data_ptr(), bcl.data_ptr()
d.out, d.out_bstride, d.a_off, d.stride, d.train = out.data_ptr(), A * (5 + nc), 0, 8.0, 0
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
N.check(L.yxh_head_pred(C.byref(d), st), "head")
e0.record()
for _ in range(50):
    N.check(L.yxh_head_pred(C.byref(d), st), "head")
e1.record()
e1.synchronize()
us = e0.elapsed_time(e1) / 50 * 1e3
mb = (B * h * w * (2 * cin * 2 + (5 + nc) * 4)) / 1e6
print(f"head_pred level0: {us:.1f} us, {mb:.0f} MB -> {mb / us:.2f} TB/s")
