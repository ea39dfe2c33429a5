"""Probe (GPU box): the 3x3 conv shapes of yolox_s bs32 -- best conv_r3/conv_r3h tile vs
every conv_ws (weight-stationary) tile, timed with HIP events; each conv_ws result is
checked against the igemm tile 6 output.
Usage: python tools/ws_probe.py [tile ...]"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd"))
from yolox_amd import _native as N  # noqa: E402

L = N.lib()
dev = torch.device("cuda:0")
st = N.stream_ptr(dev)
B = int(os.environ.get("WS_BATCH", "32"))
SHAPES = [(1, 160, 32, 32), (1, 80, 64, 64), (1, 40, 128, 128), (1, 20, 256, 256), (1, 80, 128, 128),
          (1, 80, 128, 256), (1, 40, 128, 256), (1, 20, 128, 128), (1, 20, 128, 256), (2, 320, 32, 64),
          (2, 160, 64, 128), (2, 80, 128, 256), (2, 40, 256, 512), (2, 80, 128, 128), (2, 40, 256, 256)]
if os.environ.get("WS_SHAPES"):  # e.g. "1,80,128,128;1,40,128,128"
    SHAPES = [tuple(int(v) for v in sh.split(",")) for sh in os.environ["WS_SHAPES"].split(";")]
OLD = [2 * i for i in range(113, 153)]
NEW = [2 * i for i in range(161, 191)]
TILES = [int(t) for t in sys.argv[1:]] or OLD + NEW


def timeit(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for S, H, K, Nc in SHAPES:
    Ho = H // S
    x = torch.randn(B, H, H, K, device=dev).to(torch.bfloat16)
    y = torch.empty(B, Ho, Ho, Nc, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(Nc, 3, 3, K, device=dev) / (9 * K) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Nc, device=dev) * 0.1

    def conv(tile):
        d = N.ConvDesc()
        d.dtype, d.batch = N.BF16, B
        d.in_h, d.in_w, d.out_h, d.out_w = H, H, Ho, Ho
        d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups = K, Nc, 3, 3, S, 1, 1
        d.nsrc = 1
        d.src[0] = N.Src(x.data_ptr(), K, K, H * H * K, H, H, 0, 0)
        d.weight, d.bias = w.data_ptr(), b.data_ptr()
        d.dst, d.dst_dtype, d.dst_cstride, d.dst_bstride = y.data_ptr(), N.BF16, Nc, Ho * Ho * Nc
        d.act, d.tile = N.ACT_SILU, tile
        return L.yxh_conv2d(C.byref(d), st)

    flop = 2.0 * B * Ho * Ho * Nc * 9 * K
    assert conv(12) == N.OK
    ref = y.float().clone()
    res = []
    for tile in TILES:
        y.zero_()
        if conv(tile) != N.OK:
            continue
        torch.cuda.synchronize()
        err = float((y.float() - ref).abs().max() / ref.abs().max())
        t = timeit(lambda: conv(tile))
        res.append((t, tile, err))
    res.sort()
    old = [r for r in res if r[1] in OLD]
    new = [r for r in res if r[1] in NEW]
    bad = [r for r in res if r[2] > 2e-2]
    fmt = lambda r: f"{r[1] >> 1}:{r[0]:.1f}us/{flop / r[0] / 1e6:.0f}TF"  # noqa: E731
    print(f"s{S} {H}->{Ho} {K}->{Nc}: best r3 {fmt(old[0]) if old else '-'} | ws " +
          " ".join(fmt(r) for r in new) + (f" | BAD {[(r[1] >> 1, round(r[2], 4)) for r in bad]}" if bad else ""),
          flush=True)
