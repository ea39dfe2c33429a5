"""GPU probe: which bilinear contraction matches ATen's F.interpolate on this device (prints mismatch
counts per variant; tools/resize_probe.hip, built to dbg/libresize_probe.so)."""
import ctypes as C
import os
import sys

import torch
import torch.nn.functional as F

lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dbg", "libresize_probe.so"))
lib.yxh_resize_probe.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
g = torch.Generator().manual_seed(3)
x = (torch.rand(2, 3, 640, 640, generator=g) * 255).round().cuda()
for size in [(480, 480), (544, 544), (800, 800), (353, 517)]:
    want = F.interpolate(x, size=size, mode="bilinear", align_corners=False)
    row = []
    for v in (0, 1, 2, 3, 4, 5, 10, 11, 12, 13, 14, 15):
        out = torch.empty_like(want)
        rc = lib.yxh_resize_probe(v, x.data_ptr(), 6, 640, 640, out.data_ptr(), size[0], size[1],
                                  torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        row.append((v, int((out != want).sum())))
    print(size, row, flush=True)
sys.exit(0)
