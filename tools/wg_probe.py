"""16-bit 3x3 weight-gradient probe (GPU box): one yolox_x training shape per run, every 16-bit
tile timed with HIP events, or one tile launched 20x for rocprofv3 --pmc passes.
Usage: python tools/wg_probe.py [CIN COUT H W B [TILE [STRIDE]]]  (default: dark3 Bottleneck 3x3,
160 -> 160 at 8 x 160 x 160, fp16; H x W is the input; with TILE only that tile runs, untimed;
TILE 0 times every tile at STRIDE)."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd"))
from yolox_amd import _native as N  # noqa: E402

L = N.lib()
dev = torch.device("cuda:0")
st = N.stream_ptr(dev)
a = [int(v) for v in sys.argv[1:]]
cin, cout, H, W, B = a[:5] if len(a) >= 5 else (160, 160, 160, 160, 8)
only = a[5] if len(a) > 5 and a[5] else None
S = a[6] if len(a) > 6 else 1
OH, OW = (H - 1) // S + 1, (W - 1) // S + 1
x = torch.randn(B, H, W, cin, device=dev).to(torch.float16)
dy = torch.randn(B, OH, OW, cout, device=dev).to(torch.float16)
dw = torch.zeros(cout, cin, 3, 3, device=dev)
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
d = N.WgradDesc()
d.dtype, d.batch = N.F16, B
d.in_h, d.in_w, d.out_h, d.out_w = H, W, OH, OW
d.cin, d.cout, d.kh, d.kw, d.stride, d.pad = cin, cout, 3, 3, S, 1
d.nsrc, d.cin_store = 1, cin
d.src[0] = N.Src(x.data_ptr(), cin, cin, H * W * cin, H, W, 0, 0)
d.dy = N.Src(dy.data_ptr(), cout, cout, OH * OW * cout, OH, OW, 0, 0)
d.dw, d.workspace, d.workspace_bytes = dw.data_ptr(), ws.data_ptr(), ws.numel()
flop = 2.0 * cin * cout * 9 * B * OH * OW
for tile in ([only] if only is not None else [2, 8, 25, 26, 27, 28]):
    d.tile = tile
    if L.yxh_conv_wgrad(C.byref(d), st) != N.OK:
        print(f"tile {tile}: n/a")
        continue
    reps = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        N.check(L.yxh_conv_wgrad(C.byref(d), st), "wgrad")
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"tile {tile}: {ms * 1e3:8.1f} us  {flop / ms / 1e9:7.1f} TFLOP/s", flush=True)
