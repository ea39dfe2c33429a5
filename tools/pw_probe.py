"""Probe: 1x1-conv time vs a plain copy of the same bytes, SiLU vs no activation,
MALL-resident (same buffers) vs rotating buffers (> 256 MB Infinity Cache).
Run on the GPU box: python tools/pw_probe.py [tile codes]"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd"))
from yolox_amd import _native as N  # noqa: E402

L = N.lib()
dev = torch.device("cuda:0")
st = N.stream_ptr(dev)
SHAPES = [(204800, 64, 64), (51200, 128, 128), (819200, 64, 64), (12800, 512, 512), (51200, 256, 256)]
if os.environ.get("PW_SHAPES"):  # "M,K,N;M,K,N": e.g. a sweep over M for the fixed vs per-pixel cost
    SHAPES = [tuple(int(v) for v in t.split(",")) for t in os.environ["PW_SHAPES"].split(";")]
TILES = [int(t) for t in sys.argv[1:]] or [97 * 2, 99 * 2, 203 * 2, 205 * 2, 206 * 2, 207 * 2]


def timeit(fn, nbuf, reps=24):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(4):
        fn(i % nbuf)
    s.record()
    for i in range(reps):
        fn(i % nbuf)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for M, K, Nc in SHAPES:
    nbuf = max(1, min(8, int(600e6 // (M * (K + Nc) * 2))))
    xs = [torch.randn(M, K, device=dev).to(torch.bfloat16) for _ in range(nbuf)]
    ys = [torch.empty(M, Nc, device=dev, dtype=torch.bfloat16) for _ in range(nbuf)]
    w = (torch.randn(Nc, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.zeros(Nc, device=dev)
    line = [f"M={M} K={K} N={Nc} ({M * (K + Nc) * 2 / 1e6:.0f} MB)"]
    yc = [torch.empty(M, K, device=dev, dtype=torch.bfloat16) for _ in range(nbuf)]
    for nb in (1, nbuf):
        line.append(f"copy[{nb}] {timeit(lambda i: yc[i].copy_(xs[i]), nb):.1f}")

    def conv(i, tile, act):
        d = N.ConvDesc()
        d.dtype, d.batch = N.BF16, 1
        d.in_h, d.in_w, d.out_h, d.out_w = 1, M, 1, M
        d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups = K, Nc, 1, 1, 1, 0, 1
        d.nsrc = 1
        d.src[0] = N.Src(xs[i].data_ptr(), K, K, M * K, 1, M, 0, 0)
        d.weight, d.bias = w.data_ptr(), b.data_ptr()
        d.dst, d.dst_dtype, d.dst_cstride, d.dst_bstride = ys[i].data_ptr(), N.BF16, Nc, M * Nc
        d.act, d.tile = act, tile
        return L.yxh_conv2d(C.byref(d), st)

    for tile in TILES:
        if conv(0, tile, N.ACT_SILU) != N.OK:
            continue
        r = [timeit(lambda i: conv(i, tile, a), nb) for a in (N.ACT_SILU, N.ACT_NONE) for nb in (1, nbuf)]
        line.append(f"t{tile >> 1}/{(tile & 1) + 1} silu {r[0]:.1f}/{r[1]:.1f} none {r[2]:.1f}/{r[3]:.1f}")
    print(" | ".join(line), flush=True)
