"""Batch-statistics BatchNorm kernels at yolox_x @1280 batch-8 shapes (BASELINE configs[4]), each
alone on an idle GPU: yxh_bn_stats (chan_reduce STATS + chan_finalize), yxh_bn_act_fwd and
yxh_bn_act_bwd (chan_reduce BWD + chan_finalize + bn_act_bwd_apply), timed with HIP events over
repeated calls; bytes = the tensors each call must read / write once.  Run under rocprofv3
--kernel-trace --stats for the per-kernel split.
Usage: python tools/bn_probe.py [reps]"""
import ctypes as C
import sys

import torch

sys.path.insert(0, "pixeltable-yolox_amd")
from yolox_amd import _native as N  # noqa: E402
from yolox_amd.train import dense_src  # noqa: E402

SHAPES = [(8, 640, 640, 80), (8, 320, 320, 160), (8, 160, 160, 320), (8, 80, 80, 640), (8, 40, 40, 1280)]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    lib = N.lib()
    st = N.stream_ptr(torch.device("cuda"))
    ws = torch.empty(int(lib.yxh_reduce_workspace_bytes(1280)), dtype=torch.uint8, device="cuda")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for B, H, W, Cc in SHAPES:
        y = (torch.randn(B, H, W, Cc, device="cuda") * 2 + 0.5).half()
        g = torch.randn(B, H, W, Cc, device="cuda")
        out = torch.empty_like(y)
        dx = torch.empty_like(y)
        gamma = torch.rand(Cc, device="cuda") + 0.5
        beta = torch.randn(Cc, device="cuda")
        rm, rv = torch.zeros(Cc, device="cuda"), torch.ones(Cc, device="cuda")
        stats = torch.empty(4, Cc, device="cuda")
        dg, db = torch.empty(Cc, device="cuda"), torch.empty(Cc, device="cuda")
        ys, gs, os_ = dense_src(y), dense_src(g), dense_src(out)
        n = y.numel()

        def stats_call():
            N.check(lib.yxh_bn_stats(N.F16, B, C.byref(ys), gamma.data_ptr(), beta.data_ptr(), rm.data_ptr(),
                                     rv.data_ptr(), 1e-3, 0.03, stats.data_ptr(), ws.data_ptr(), ws.numel(), st), "stats")

        def fwd_call():
            N.check(lib.yxh_bn_act_fwd(N.F16, B, C.byref(ys), stats.data_ptr(), N.ACT_CODE["silu"], None,
                                       C.byref(os_), st), "fwd")

        def bwd_call():
            N.check(lib.yxh_bn_act_bwd(N.F16, B, C.byref(ys), C.byref(gs), stats.data_ptr(), gamma.data_ptr(),
                                       N.ACT_CODE["silu"], dg.data_ptr(), db.data_ptr(), dx.data_ptr(), ws.data_ptr(),
                                       ws.numel(), st), "bwd")

        for name, fn, nbytes in (("bn_stats", stats_call, 2 * n), ("bn_act_fwd", fwd_call, 4 * n),
                                 ("bn_act_bwd", bwd_call, 16 * n)):  # bwd: reduce (y + g) + apply (y + g + dx)
            fn()
            torch.cuda.synchronize()
            ev0.record()
            for _ in range(reps):
                fn()
            ev1.record()
            ev1.synchronize()
            us = ev0.elapsed_time(ev1) / reps * 1e3
            print(f"{name:11s} B{B} {H}x{W} C{Cc:5d}: {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s (one read/write "
                  f"of each tensor)", flush=True)


if __name__ == "__main__":
    main()
