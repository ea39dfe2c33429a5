"""Probe (GPU box): dense 1x1 conv shapes of yolox_s bs32 -- time every applicable tile
(existing families and conv_pwf) with HIP events, check each against tile 6 (max rel
diff).  Usage: python tools/pwf_probe.py [tile ...]"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd"))
from yolox_amd import _native as N  # noqa: E402

L = N.lib()
dev = torch.device("cuda:0")
st = N.stream_ptr(dev)
SHAPES = [(819200, 64, 64), (819200, 32, 32), (204800, 64, 64), (204800, 128, 128), (204800, 256, 128),
          (51200, 128, 128), (51200, 256, 256), (51200, 512, 256), (12800, 512, 512), (12800, 1024, 512),
          (12800, 512, 256)]
TILES = [int(t) for t in sys.argv[1:]] or [6 * 2, 9 * 2, 6 * 2 + 1, 9 * 2 + 1, 82 * 2] + [2 * i for i in range(97, 105)]


def timeit(fn, nbuf, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3):
        fn(i % nbuf)
    s.record()
    for i in range(reps):
        fn(i % nbuf)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for M, K, Nc in SHAPES:
    nbuf = max(1, min(6, int(700e6 // (M * (K + Nc) * 2))))
    xs = [torch.randn(M, K, device=dev).to(torch.bfloat16) for _ in range(nbuf)]
    ys = [torch.empty(M, Nc, device=dev, dtype=torch.bfloat16) for _ in range(nbuf)]
    w = (torch.randn(Nc, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(Nc, device=dev) * 0.1
    res = torch.randn(M, Nc, device=dev).to(torch.bfloat16) if K == Nc else None

    def conv(i, tile, with_res=False):
        d = N.ConvDesc()
        d.dtype, d.batch = N.BF16, 1
        d.in_h, d.in_w, d.out_h, d.out_w = 1, M, 1, M
        d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups = K, Nc, 1, 1, 1, 0, 1
        d.nsrc = 1
        d.src[0] = N.Src(xs[i].data_ptr(), K, K, M * K, 1, M, 0, 0)
        d.weight, d.bias = w.data_ptr(), b.data_ptr()
        d.dst, d.dst_dtype, d.dst_cstride, d.dst_bstride = ys[i].data_ptr(), N.BF16, Nc, M * Nc
        if with_res:
            d.residual, d.res_cstride, d.res_bstride = res.data_ptr(), Nc, M * Nc
        d.act, d.tile = N.ACT_SILU, tile
        return L.yxh_conv2d(C.byref(d), st)

    line = [f"M={M} K={K} N={Nc} ({M * (K + Nc) * 2 / 1e6:.0f} MB, {2 * M * K * Nc / 1e9:.1f} GF)"]
    yc = [torch.empty(M, K, device=dev, dtype=torch.bfloat16) for _ in range(nbuf)]
    line.append(f"copy {timeit(lambda i: yc[i].copy_(xs[i]), nbuf):.1f}")
    assert conv(0, 12) == N.OK
    ref = ys[0].float().clone()
    best = None
    for tile in TILES:
        if conv(0, tile) != N.OK:
            continue
        err = float((ys[0].float() - ref).abs().max() / ref.abs().max())
        t = timeit(lambda i: conv(i, tile), nbuf)
        tag = f"t{tile >> 1}/{(tile & 1) + 1} {t:.1f}" + (f" ERR {err:.2e}" if err > 2e-2 else "")
        if res is not None and tile >= 2 * 97:
            conv(0, 12, True)
            r0 = ys[0].float().clone()
            conv(0, tile, True)
            e2 = float((ys[0].float() - r0).abs().max() / r0.abs().max())
            if e2 > 2e-2:
                tag += f" RESERR {e2:.2e}"
        line.append(tag)
        if best is None or t < best[0]:
            best = (t, tile)
    line.append(f"best t{best[1] >> 1}")
    print(" | ".join(line), flush=True)
