"""Probe (GPU box): time one conv shape at several batch sizes with a fixed tile id, to split
a launch into a fixed cost (prologue: weight loads, ramp, tail) and a per-image slope.
Usage: python tools/batch_probe.py "K H CIN COUT TILE_ID [S]" ...   (K = 1 or 3)"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd"))
from yolox_amd import _native as N  # noqa: E402

L = N.lib()
dev = torch.device("cuda:0")
st = N.stream_ptr(dev)
BATCHES = [int(v) for v in os.environ.get("PROBE_BATCHES", "1,2,4,8,16,32").split(",")]
for spec in sys.argv[1:]:
    v = [int(t) for t in spec.split()]
    k, H, K, Nc, tid = v[:5]
    S = v[5] if len(v) > 5 else 1
    pad = k // 2
    Ho = (H + 2 * pad - k) // S + 1
    Bmax = max(BATCHES)
    x = torch.randn(Bmax, H, H, K, device=dev).to(torch.bfloat16)
    y = torch.empty(Bmax, Ho, Ho, Nc, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(Nc, k, k, K, device=dev) / (k * k * K) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Nc, device=dev) * 0.1
    wf = torch.empty_like(w)
    N.check(L.yxh_pack_frag(w.data_ptr(), Nc, k * k, K, N.BF16, wf.data_ptr(), st), "pack_frag")
    row = []
    ref = None
    for B, frag in [(b_, f_) for b_ in BATCHES for f_ in (0, 1)]:
        d = N.ConvDesc()
        d.dtype, d.batch = N.BF16, B
        d.in_h, d.in_w, d.out_h, d.out_w = H, H, Ho, Ho
        d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups = K, Nc, k, k, S, pad, 1
        d.nsrc = 1
        d.src[0] = N.Src(x.data_ptr(), K, K, H * H * K, H, H, 0, 0)
        d.weight, d.bias = w.data_ptr(), b.data_ptr()
        d.dst, d.dst_dtype, d.dst_cstride, d.dst_bstride = y.data_ptr(), N.BF16, Nc, Ho * Ho * Nc
        d.act, d.tile = N.ACT_SILU, 2 * tid
        d.weight_frag = wf.data_ptr() if frag else None
        y.zero_()
        if L.yxh_conv2d(C.byref(d), st) != N.OK:
            row.append(f"B{B}: n/a")
            continue
        torch.cuda.synchronize()
        if not frag:
            ref = y[:B].clone()
        elif not torch.equal(ref, y[:B]):
            row.append("FRAG MISMATCH")
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(30):
            L.yxh_conv2d(C.byref(d), st)
        e.record()
        e.synchronize()
        t = s.elapsed_time(e) / 30 * 1e3
        row.append(f"B{B}{'f' if frag else ''}: {t:.1f}")
    print(f"k{k}s{S} {H} {K}->{Nc} id {tid}: " + "  ".join(row), flush=True)
