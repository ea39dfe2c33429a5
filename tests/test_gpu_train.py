"""Training path (yolox_amd/train.py + csrc/train.hip) on the GPU.

Per kernel, against PyTorch fp32 autograd on the CPU (the plain fp32 reference of the
same op): BN batch statistics + act (+ running stats), BN+act backward, conv weight
gradient (1x1 / 3x3 s1 / 3x3 s2, two sources, nearest-x2 source), conv data gradient
(transposed/flipped weights, zero-dilated source for stride 2), SPP max-pool backward,
upsample backward, the loss gradient w.r.t. the raw head outputs.

End to end: YoloxModule(train) fp32 on yolox_s 128x128 vs the oracle (reference
restatement pinned to the reference's train fixture): the six loss values, every
parameter gradient and the BN running statistics (north_star: 1e-3 fp32).
"""
import ctypes as C
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
TOL = {torch.float32: 1e-4, torch.bfloat16: 2e-2, torch.float16: 4e-3}


def lib():
    from yolox_amd import _native as N
    return N.lib()


def chk(rc):
    from yolox_amd import _native as N
    N.check(rc)


def src(t, coff=0, ch=None, up=0):
    from yolox_amd.train import Act
    return Act(t, coff, ch if ch is not None else t.shape[3] - coff).src(up)


def stream():
    return torch.cuda.current_stream().cuda_stream


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def ws(C_=1024):
    return torch.empty(int(lib().yxh_reduce_workspace_bytes(C_)), dtype=torch.uint8, device="cuda")


# ----------------------------------------------------------------- BatchNorm + act
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H,W,Cc", [(2, 16, 16, 32), (3, 10, 7, 64), (1, 5, 5, 512), (1, 4, 6, 1280), (2, 3, 3, 2560)])
def test_bn_stats_and_act_fwd(dtype, B, H, W, Cc):
    g = torch.Generator().manual_seed(B * 100 + Cc)
    y = (torch.randn(B, H, W, Cc, generator=g) * 3 + 5).to(dtype)
    gamma, beta = torch.rand(Cc, generator=g) + 0.5, torch.randn(Cc, generator=g)
    rm, rv = torch.randn(Cc, generator=g), torch.rand(Cc, generator=g) + 0.5
    res = torch.randn(B, H, W, Cc, generator=g).to(dtype)
    yd, rmd, rvd = y.cuda(), rm.clone().cuda(), rv.clone().cuda()
    stats = torch.empty(4, Cc, device="cuda")
    w = ws(max(Cc, 1024))
    ys = src(yd)
    gd, bd = gamma.cuda(), beta.cuda()  # held: the launch is asynchronous
    chk(lib().yxh_bn_stats(DT[dtype], B, C.byref(ys), gd.data_ptr(), bd.data_ptr(),
                           rmd.data_ptr(), rvd.data_ptr(), 1e-3, 0.03, stats.data_ptr(), w.data_ptr(), w.numel(),
                           stream()))
    out = torch.empty_like(yd)
    rd = res.cuda()
    rs, os_ = src(rd), src(out)
    chk(lib().yxh_bn_act_fwd(DT[dtype], B, C.byref(ys), stats.data_ptr(), 1, C.byref(rs), C.byref(os_), stream()))
    torch.cuda.synchronize()
    # reference: torch BN (training) + SiLU + residual, fp32 on CPU
    x = y.float().permute(0, 3, 1, 2)
    rm_ref, rv_ref = rm.clone(), rv.clone()
    ref = F.silu(F.batch_norm(x, rm_ref, rv_ref, gamma, beta, True, 0.03, 1e-3)).permute(0, 2, 3, 1) + res.float()
    assert rel(out, ref) < TOL[dtype] * (1 if dtype == torch.float32 else 2)
    assert rel(rmd, rm_ref) < 1e-5 and rel(rvd, rv_ref) < 1e-4
    mean = x.mean((0, 2, 3))
    assert rel(stats[0], mean) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H,W,Cc,act", [(2, 16, 16, 32, 1), (3, 9, 11, 64, 1), (2, 6, 6, 128, 3),
                                             (1, 4, 5, 1280, 1)])
def test_bn_act_bwd(dtype, B, H, W, Cc, act):
    g = torch.Generator().manual_seed(7 + Cc)
    y = (torch.randn(B, H, W, Cc, generator=g) * 2 + 1).to(dtype)
    gamma, beta = torch.rand(Cc, generator=g) + 0.5, torch.randn(Cc, generator=g)
    dout = torch.randn(B, H, W, Cc, generator=g)
    yd = y.cuda()
    stats = torch.empty(4, Cc, device="cuda")
    w = ws(max(Cc, 1024))
    ys = src(yd)
    gd, bd = gamma.cuda(), beta.cuda()  # held: the launches are asynchronous
    chk(lib().yxh_bn_stats(DT[dtype], B, C.byref(ys), gd.data_ptr(), bd.data_ptr(), None, None,
                           1e-3, 0.03, stats.data_ptr(), w.data_ptr(), w.numel(), stream()))
    dgam, dbet = torch.empty(Cc, device="cuda"), torch.empty(Cc, device="cuda")
    dx = torch.empty(B, H, W, Cc, dtype=dtype, device="cuda")
    dd = dout.cuda()
    gs = src(dd)
    chk(lib().yxh_bn_act_bwd(DT[dtype], B, C.byref(ys), C.byref(gs), stats.data_ptr(), gd.data_ptr(), act,
                             dgam.data_ptr(), dbet.data_ptr(), dx.data_ptr(), w.data_ptr(), w.numel(), stream()))
    torch.cuda.synchronize()
    x = y.float().permute(0, 3, 1, 2).clone().requires_grad_()
    gm, bt = gamma.clone().requires_grad_(), beta.clone().requires_grad_()
    z = F.batch_norm(x, None, None, gm, bt, True, 0.0, 1e-3)
    o = F.silu(z) if act == 1 else F.leaky_relu(z, 0.1)
    o.backward(dout.permute(0, 3, 1, 2))
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    assert rel(dgam, gm.grad) < tol and rel(dbet, bt.grad) < tol
    assert rel(dx, x.grad.permute(0, 2, 3, 1)) < tol


# ----------------------------------------------------------------- conv gradients
def wgrad(dtype, srcs, dy, cout, cin, k, s, p, in_hw, out_hw, B, cin_store=None, tile=0, ws_bytes=0):
    from yolox_amd import _native as N
    d = N.WgradDesc()
    d.dtype, d.batch = DT[dtype], B
    d.in_h, d.in_w = in_hw
    d.out_h, d.out_w = out_hw
    d.cin, d.cout, d.kh, d.kw, d.stride, d.pad = cin, cout, k, k, s, p
    d.nsrc, d.cin_store = len(srcs), cin_store or cin
    for j, q in enumerate(srcs):
        d.src[j] = q
    d.dy = dy
    dw = torch.zeros(cout, cin_store or cin, k, k, device="cuda")
    d.dw = dw.data_ptr()
    d.tile = tile
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device="cuda") if ws_bytes else None
    if ws is not None:
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws_bytes
    chk(lib().yxh_conv_wgrad(C.byref(d), stream()))
    torch.cuda.synchronize()
    return dw


WG_CASES = [  # cin0, cin1, up1, cout, k, s, H
    (32, 0, 0, 64, 3, 1, 16), (64, 0, 0, 32, 3, 2, 20), (64, 0, 0, 64, 1, 1, 12), (32, 32, 0, 64, 1, 1, 10),
    (64, 64, 1, 32, 1, 1, 8), (128, 0, 0, 128, 3, 1, 9), (16, 0, 0, 24, 3, 1, 12),
    # concat split on a 16-byte chunk but not on a K-stage boundary (yolox_m 48, yolox_x 80)
    (48, 48, 0, 64, 1, 1, 10), (80, 80, 0, 96, 1, 1, 7),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin0,cin1,up1,cout,k,s,H", WG_CASES)
def test_conv_wgrad_and_dgrad(dtype, cin0, cin1, up1, cout, k, s, H):
    """weight gradient (yxh_conv_wgrad) and data gradient (yxh_conv2d with
    yxh_pack_dgrad_weight + ACCUMULATE, zero-dilated source for stride 2)."""
    from yolox_amd import _native as N
    from yolox_amd.train import dense_src
    g = torch.Generator().manual_seed(cin0 + 7 * cout + H)
    B, W = 2, H + 2
    p = (k - 1) // 2
    x0 = torch.randn(B, H, W, cin0, generator=g).to(dtype)
    x1 = torch.randn(B, H >> up1, W >> up1, cin1, generator=g).to(dtype) if cin1 else None
    oh, ow = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(B, oh, ow, cout, generator=g).to(dtype)
    wt = torch.randn(cout, cin0 + cin1, k, k, generator=g) * 0.1
    x0d, dyd = x0.cuda(), dy.cuda()
    srcs = [src(x0d)]
    if cin1:
        x1d = x1.cuda()
        srcs.append(src(x1d, up=up1))
    dw = wgrad(dtype, srcs, src(dyd), cout, cin0 + cin1, k, s, p, (H, W), (oh, ow), B)
    # data gradient of source 0 (channels [0, cin0))
    pk = torch.empty(cin0 * k * k * cout, dtype=dtype, device="cuda")
    wtd = wt.cuda()
    chk(lib().yxh_pack_dgrad_weight(wtd.data_ptr(), cout, cin0 + cin1, k, k, 0, cin0, cout, DT[dtype], pk.data_ptr(),
                                    stream()))
    dx0 = torch.full((B, H, W, cin0), 0.5, device="cuda")  # accumulate onto 0.5
    d = N.ConvDesc()
    d.dtype, d.batch, d.in_h, d.in_w, d.out_h, d.out_w = DT[dtype], B, H, W, H, W
    d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups, d.nsrc = cout, cin0, k, k, 1, k - 1 - p, 1, 1
    d.src[0] = dense_src(dyd, up=2 if s == 2 else 0)
    zb = torch.zeros(cin0, device="cuda")
    d.weight, d.bias, d.dst, d.dst_dtype = pk.data_ptr(), zb.data_ptr(), dx0.data_ptr(), 0
    d.dst_cstride, d.dst_bstride, d.act, d.flags = cin0, H * W * cin0, 0, N.CONV_ACCUMULATE
    chk(lib().yxh_conv2d(C.byref(d), stream()))
    torch.cuda.synchronize()
    # reference
    xin = x0.float().permute(0, 3, 1, 2)
    if cin1:
        x1n = x1.float().permute(0, 3, 1, 2)
        if up1:
            x1n = F.interpolate(x1n, scale_factor=2, mode="nearest")
        xin = torch.cat([xin, x1n], 1)
    xin = xin.clone().requires_grad_()
    wr = wt.to(dtype).float().clone().requires_grad_()
    F.conv2d(xin, wr, stride=s, padding=p).backward(dy.float().permute(0, 3, 1, 2))
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert rel(dw, wr.grad) < tol
    assert rel(dx0 - 0.5, xin.grad[:, :cin0].permute(0, 2, 3, 1)) < tol


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cfwd,H,W,B", [(80, 19, 23, 2), (160, 20, 18, 2), (320, 11, 13, 2), (64, 24, 20, 3),
                                        (128, 17, 15, 2), (256, 9, 10, 2)])
def test_dgrad_conv_ws_fp32_tiles(dtype, cfwd, H, W, B):
    """The data gradient of a stride-1 3x3 conv on conv_ws's fp32-gradient tiles (281-288: yolox_x's
    80 / 160 / 320 channels, yolox_s / yolox_l's 64 / 128 / 256): dy with the transposed, flipped
    weights written into / added onto an fp32 gradient (YXH_CONV_ACCUMULATE), vs torch fp32 autograd
    and vs the register-staged conv_igemm tile of the same data gradient."""
    from yolox_amd import _native as N
    from yolox_amd.train import dense_src
    g = torch.Generator().manual_seed(cfwd + H)
    cin, cout = cfwd, cfwd
    dy = torch.randn(B, H, W, cout, generator=g).to(dtype)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * 0.05
    wtd, dyd = wt.cuda(), dy.cuda()
    pk = torch.empty(cin * 9 * cout, dtype=dtype, device="cuda")
    chk(lib().yxh_pack_dgrad_weight(wtd.data_ptr(), cout, cin, 3, 3, 0, cin, cout, DT[dtype], pk.data_ptr(), stream()))
    zb = torch.zeros(cin, device="cuda")
    xr = torch.zeros(B, cin, H, W, requires_grad=True)
    F.conv2d(xr, wt.to(dtype).float(), padding=1).backward(dy.float().permute(0, 3, 1, 2))
    want = xr.grad.permute(0, 2, 3, 1)

    def dgrad(tile, acc):
        dx = torch.full((B, H, W, cin), 0.5 if acc else float("nan"), device="cuda")
        d = N.ConvDesc()
        d.dtype, d.batch, d.in_h, d.in_w, d.out_h, d.out_w = DT[dtype], B, H, W, H, W
        d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups, d.nsrc = cout, cin, 3, 3, 1, 1, 1, 1
        d.src[0] = dense_src(dyd)
        d.weight, d.bias, d.dst, d.dst_dtype = pk.data_ptr(), zb.data_ptr(), dx.data_ptr(), 0
        d.dst_cstride, d.dst_bstride, d.act = cin, H * W * cin, 0
        d.flags, d.tile = (N.CONV_ACCUMULATE if acc else 0), tile
        rc = lib().yxh_conv2d(C.byref(d), stream())
        if rc == N.EUNSUPPORTED:
            return None
        chk(rc)
        torch.cuda.synchronize()
        return dx - 0.5 if acc else dx

    base = dgrad(2 * 1, True)  # conv_igemm
    ran = 0
    for tid in range(281, 289):
        for acc in (False, True):
            got = dgrad(2 * tid, acc)
            if got is None:
                continue
            assert rel(got, want) < 1e-4, (tid, acc)  # same rounded operands: summation order only
            assert rel(got, base) < 1e-4, (tid, acc)
            ran += 1
    assert ran >= 2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cfwd,coutf,H,W,B", [(160, 160, 20, 18, 2), (320, 640, 9, 10, 2), (64, 128, 17, 15, 3),
                                              (256, 128, 8, 8, 2), (160, 320, 13, 7, 2)])
def test_dgrad_1x1_conv_pwf_fp32(dtype, cfwd, coutf, H, W, B):
    """The data gradient of a 1x1 conv on conv_pwf's fp32-gradient epilogue (tiles 97-104, round 5):
    dy (the forward's cout channels) with the transposed weights into / onto an fp32 gradient
    (YXH_CONV_ACCUMULATE), vs torch fp32 autograd and the register-staged conv_igemm tile."""
    from yolox_amd import _native as N
    from yolox_amd.train import dense_src
    g = torch.Generator().manual_seed(cfwd + coutf + H)
    dy = torch.randn(B, H, W, coutf, generator=g).to(dtype)
    wt = torch.randn(coutf, cfwd, 1, 1, generator=g) * 0.05
    wtd, dyd = wt.cuda(), dy.cuda()
    pk = torch.empty(cfwd * coutf, dtype=dtype, device="cuda")
    chk(lib().yxh_pack_dgrad_weight(wtd.data_ptr(), coutf, cfwd, 1, 1, 0, cfwd, coutf, DT[dtype], pk.data_ptr(),
                                    stream()))
    zb = torch.zeros(cfwd, device="cuda")
    xr = torch.zeros(B, cfwd, H, W, requires_grad=True)
    F.conv2d(xr, wt.to(dtype).float()).backward(dy.float().permute(0, 3, 1, 2))
    want = xr.grad.permute(0, 2, 3, 1)

    def dgrad(tile, acc):
        dx = torch.full((B, H, W, cfwd), 0.5 if acc else float("nan"), device="cuda")
        d = N.ConvDesc()
        d.dtype, d.batch, d.in_h, d.in_w, d.out_h, d.out_w = DT[dtype], B, H, W, H, W
        d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups, d.nsrc = coutf, cfwd, 1, 1, 1, 0, 1, 1
        d.src[0] = dense_src(dyd)
        d.weight, d.bias, d.dst, d.dst_dtype = pk.data_ptr(), zb.data_ptr(), dx.data_ptr(), 0
        d.dst_cstride, d.dst_bstride, d.act = cfwd, H * W * cfwd, 0
        d.flags, d.tile = (N.CONV_ACCUMULATE if acc else 0), tile
        rc = lib().yxh_conv2d(C.byref(d), stream())
        if rc == N.EUNSUPPORTED:
            return None
        chk(rc)
        torch.cuda.synchronize()
        return dx - 0.5 if acc else dx

    base = dgrad(2 * 1, True)  # conv_igemm
    assert rel(base, want) < 1e-4
    ran = 0
    for tid in range(97, 105):
        for acc in (False, True):
            got = dgrad(2 * tid, acc)
            if got is None:
                continue
            assert rel(got, want) < 1e-4, (tid, acc)
            assert rel(got, base) < 1e-4, (tid, acc)
            ran += 1
    assert ran >= 6  # the 32-element K-stage tiles (97, 98, 103) take every K here


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cin,cout,H,W,B", [(80, 160, 19, 23, 2), (160, 320, 20, 18, 2), (64, 128, 24, 20, 2),
                                            (32, 64, 17, 15, 3), (128, 256, 9, 10, 2), (320, 640, 7, 8, 2)])
def test_dgrad_s2_parity_class_tiles(dtype, cin, cout, H, W, B):
    """The data gradient of a stride-2 3x3 conv (darknet.py:148-156 stage convs, yolo_pafpn.py
    bu_conv1/2) on the 16-bit parity-class tiles (217-220, dgrad_s2h: output pixel (2i+py, 2j+px)
    meets 1, 2, 2 or 4 taps of the un-dilated dy) written into / added onto an fp32 gradient, vs torch
    fp32 autograd and vs the zero-dilated form on the register-staged conv_igemm tile; odd and even
    input sizes (the forward's last row / column of taps may fall outside)."""
    from yolox_amd import _native as N
    from yolox_amd.train import dense_src
    g = torch.Generator().manual_seed(cin + H + W)
    oh, ow = (H + 1) // 2, (W + 1) // 2
    dy = torch.randn(B, oh, ow, cout, generator=g).to(dtype)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * 0.05
    wtd, dyd = wt.cuda(), dy.cuda()
    pk = torch.empty(cin * 9 * cout, dtype=dtype, device="cuda")
    chk(lib().yxh_pack_dgrad_weight(wtd.data_ptr(), cout, cin, 3, 3, 0, cin, cout, DT[dtype], pk.data_ptr(), stream()))
    zb = torch.zeros(cin, device="cuda")
    xr = torch.zeros(B, cin, H, W, requires_grad=True)
    y = F.conv2d(xr, wt.to(dtype).float(), stride=2, padding=1)
    assert tuple(y.shape[2:]) == (oh, ow)
    y.backward(dy.float().permute(0, 3, 1, 2))
    want = xr.grad.permute(0, 2, 3, 1)

    def dgrad(tile, acc):
        dx = torch.full((B, H, W, cin), 0.5 if acc else float("nan"), device="cuda")
        d = N.ConvDesc()
        d.dtype, d.batch, d.in_h, d.in_w, d.out_h, d.out_w = DT[dtype], B, H, W, H, W
        d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups, d.nsrc = cout, cin, 3, 3, 1, 1, 1, 1
        d.src[0] = dense_src(dyd, up=2)
        d.weight, d.bias, d.dst, d.dst_dtype = pk.data_ptr(), zb.data_ptr(), dx.data_ptr(), 0
        d.dst_cstride, d.dst_bstride, d.act = cin, H * W * cin, 0
        d.flags, d.tile = (N.CONV_ACCUMULATE if acc else 0), tile
        rc = lib().yxh_conv2d(C.byref(d), stream())
        if rc == N.EUNSUPPORTED:
            return None
        chk(rc)
        torch.cuda.synchronize()
        return dx - 0.5 if acc else dx

    base = dgrad(2 * 1, True)  # conv_igemm over the zero-dilated dy
    assert rel(base, want) < 1e-4
    ran = 0
    for tid in range(217, 221):
        for acc in (False, True):
            got = dgrad(2 * tid, acc)
            assert got is not None, tid
            assert rel(got, want) < 1e-4, (tid, acc)  # same rounded operands: summation order only
            assert rel(got, base) < 1e-4, (tid, acc)
            ran += 1
    assert ran == 8
    assert dgrad(2 * 215, False) is None  # the fp32 tiles refuse 16-bit operands


WG_TILE_CASES = [  # cin0, cin1, up1, cout, k, s, H, B
    (32, 0, 0, 64, 3, 1, 16, 2), (64, 0, 0, 32, 3, 2, 20, 3), (64, 64, 1, 128, 1, 1, 8, 2),
    (128, 0, 0, 128, 3, 1, 9, 2), (16, 0, 0, 24, 3, 1, 12, 1), (256, 0, 0, 192, 1, 1, 23, 2),
    (96, 32, 0, 136, 3, 2, 17, 2),
    # tiny head levels (rows narrower than one 8-pixel chunk): 128 px / 32 px / 8 px per batch
    (128, 0, 0, 128, 3, 1, 8, 2), (128, 0, 0, 128, 3, 1, 4, 2), (128, 0, 0, 128, 1, 1, 2, 2),
]


@pytest.mark.parametrize("ws", [0, 16 << 20])
@pytest.mark.parametrize("tile", [1, 2, 5, 6, 7, 8, 9, 10])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cin0,cin1,up1,cout,k,s,H,B", WG_TILE_CASES)
def test_conv_wgrad_tiles(ws, tile, dtype, cin0, cin1, up1, cout, k, s, H, B):
    """every weight-gradient tile (register-transposed 1-4, LDS-DMA + ds_read_b64_tr_b16
    5-10) against torch autograd: ragged pixel counts (stage tails), cout / cin not
    multiples of the tile, two sources with an upsampled second one, stride 2."""
    g = torch.Generator().manual_seed(cin0 * 3 + cout + H + tile)
    W = H + 4
    p = (k - 1) // 2
    x0 = torch.randn(B, H, W, cin0, generator=g).to(dtype)
    x1 = torch.randn(B, H >> up1, W >> up1, cin1, generator=g).to(dtype) if cin1 else None
    oh, ow = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dyc = (cout + 7) // 8 * 8
    dy = torch.randn(B, oh, ow, dyc, generator=g).to(dtype)
    x0d, dyd = x0.cuda(), dy.cuda()
    srcs = [src(x0d)]
    if cin1:
        x1d = x1.cuda()
        srcs.append(src(x1d, up=up1))
    dw = wgrad(dtype, srcs, src(dyd), cout, cin0 + cin1, k, s, p, (H, W), (oh, ow), B, tile=tile, ws_bytes=ws)
    torch.cuda.synchronize()
    xin = x0.float().permute(0, 3, 1, 2)
    if cin1:
        x1n = x1.float().permute(0, 3, 1, 2)
        if up1:
            x1n = F.interpolate(x1n, scale_factor=2, mode="nearest")
        xin = torch.cat([xin, x1n], 1)
    wr = torch.zeros(cout, cin0 + cin1, k, k, requires_grad=True)
    F.conv2d(xin, wr, stride=s, padding=p).backward(dy[..., :cout].float().permute(0, 3, 1, 2))
    assert rel(dw, wr.grad) < 1e-4  # fp32 accumulation of exact products: order-only differences


@pytest.mark.parametrize("ws", [0, 16 << 20])
@pytest.mark.parametrize("tile", [11, 12, 13, 14, 15, 16])
@pytest.mark.parametrize("cin0,cin1,up1,cout,k,s,H,B", WG_TILE_CASES + [(16, 0, 0, 32, 3, 1, 40, 2)])
def test_conv_wgrad9_fp32_tiles(ws, tile, cin0, cin1, up1, cout, k, s, H, B):
    """fp32 all-nine-taps weight gradient (tiles 11-16) against torch autograd: partial
    pixel tiles at the image edges, cout / cin tails, stride 2; other geometries are
    rejected (NotImplementedError) and run on tiles 1-4."""
    g = torch.Generator().manual_seed(cin0 * 5 + cout + H + tile)
    W = H + 4
    p = (k - 1) // 2
    x0 = torch.randn(B, H, W, cin0, generator=g)
    oh, ow = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dyc = (cout + 3) // 4 * 4
    dy = torch.randn(B, oh, ow, dyc, generator=g)
    x0d, dyd = x0.cuda(), dy.cuda()
    srcs = [src(x0d)]
    if cin1:
        srcs.append(src(torch.randn(B, H >> up1, W >> up1, cin1, generator=g).cuda(), up=up1))
    try:
        dw = wgrad(torch.float32, srcs, src(dyd), cout, cin0 + cin1, k, s, p, (H, W), (oh, ow), B, tile=tile,
                   ws_bytes=ws)
    except NotImplementedError as e:
        assert k != 3 or cin1, e
        return
    assert k == 3 and not cin1
    torch.cuda.synchronize()
    wr = torch.zeros(cout, cin0, k, k, requires_grad=True)
    F.conv2d(x0.permute(0, 3, 1, 2), wr, stride=s, padding=p).backward(dy[..., :cout].permute(0, 3, 1, 2))
    assert rel(dw, wr.grad) < 1e-4


WGF_CASES = [  # cin0, cin1, up1, cout, k, s, H, W, B, dy channels (>= cout: a strided dy view when larger)
    (64, 0, 0, 64, 1, 1, 16, 20, 2, 64), (64, 64, 1, 128, 1, 1, 8, 12, 2, 128), (256, 0, 0, 192, 1, 1, 23, 17, 2, 192),
    (48, 48, 0, 64, 1, 1, 10, 14, 3, 64), (128, 0, 0, 85, 1, 1, 6, 10, 2, 88), (512, 0, 0, 256, 1, 1, 5, 5, 4, 264),
    (32, 0, 0, 32, 1, 1, 160, 160, 1, 32), (64, 0, 0, 64, 3, 1, 20, 16, 2, 64), (128, 0, 0, 128, 3, 1, 9, 11, 2, 128),
    (32, 0, 0, 64, 3, 2, 20, 18, 2, 64), (96, 32, 0, 136, 3, 2, 17, 15, 2, 136), (16, 0, 0, 32, 3, 1, 24, 20, 1, 32),
]


@pytest.mark.parametrize("ws", [0, 8 << 20, 4096])
@pytest.mark.parametrize("tile", [17, 18, 19, 20])
@pytest.mark.parametrize("cin0,cin1,up1,cout,k,s,H,W,B,dyc", WGF_CASES)
def test_conv_wgrad_fp32_kmajor_tiles(ws, tile, cin0, cin1, up1, cout, k, s, H, W, B, dyc):
    """fp32 weight gradient on k-major MFMA operands (tiles 17-20, one tap per block) against torch
    autograd: 1x1 and 3x3 (stride 1 / 2, zero padding), pixel tails of the KP-pixel stages, cout /
    cin tails (the head preds' 85 rows of an 88-channel dy), two sources with the second upsampled,
    a wide dy read as a strided view; per-split partials through a workspace (summed in a fixed
    order), a workspace too small for them (falls back to atomics) and none (atomics)."""
    g = torch.Generator().manual_seed(cin0 * 3 + cout + H + tile + k)
    p = (k - 1) // 2
    oh, ow = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    x0 = torch.randn(B, H, W, cin0, generator=g)
    x1 = torch.randn(B, H >> up1, W >> up1, cin1, generator=g) if cin1 else None
    dy = torch.randn(B, oh, ow, dyc, generator=g)
    keep = [x0.cuda(), dy.cuda()] + ([x1.cuda()] if cin1 else [])  # the Src structs hold raw pointers
    srcs = [src(keep[0])]
    if cin1:
        srcs.append(src(keep[2], up=up1))
    dw = wgrad(torch.float32, srcs, src(keep[1]), cout, cin0 + cin1, k, s, p, (H, W), (oh, ow), B, tile=tile,
               ws_bytes=ws)
    xin = x0.permute(0, 3, 1, 2)
    if cin1:
        x1n = x1.permute(0, 3, 1, 2)
        if up1:
            x1n = F.interpolate(x1n, scale_factor=2, mode="nearest")
        xin = torch.cat([xin, x1n], 1)
    wr = torch.zeros(cout, cin0 + cin1, k, k, requires_grad=True)
    F.conv2d(xin, wr, stride=s, padding=p).backward(dy[..., :cout].permute(0, 3, 1, 2))
    assert rel(dw, wr.grad) < 1e-5


@pytest.mark.parametrize("ws", [0, 16 << 20])
@pytest.mark.parametrize("tile", [21, 22, 23, 24])
@pytest.mark.parametrize("cin0,cin1,up1,cout,k,s,H,W,B,dyc", [c for c in WGF_CASES if c[4] == 3]
                         + [(64, 64, 1, 64, 3, 1, 12, 10, 2, 64), (128, 0, 0, 128, 3, 1, 40, 40, 2, 128)])
def test_conv_wgrad9t_fp32_tiles(ws, tile, cin0, cin1, up1, cout, k, s, H, W, B, dyc):
    """fp32 3x3 weight gradient with all nine taps per block (tiles 21-24: one dY row segment and
    its three input rows staged once per stage) against torch autograd: stride 1 / 2, row
    segments past the image edge, cout / cin tails, two sources (the second upsampled)."""
    g = torch.Generator().manual_seed(cin0 * 7 + cout + H + tile)
    oh, ow = (H + 2 - 3) // s + 1, (W + 2 - 3) // s + 1
    x0 = torch.randn(B, H, W, cin0, generator=g)
    x1 = torch.randn(B, H >> up1, W >> up1, cin1, generator=g) if cin1 else None
    dy = torch.randn(B, oh, ow, dyc, generator=g)
    keep = [x0.cuda(), dy.cuda()] + ([x1.cuda()] if cin1 else [])
    srcs = [src(keep[0])]
    if cin1:
        srcs.append(src(keep[2], up=up1))
    dw = wgrad(torch.float32, srcs, src(keep[1]), cout, cin0 + cin1, 3, s, 1, (H, W), (oh, ow), B, tile=tile,
               ws_bytes=ws)
    xin = x0.permute(0, 3, 1, 2)
    if cin1:
        x1n = x1.permute(0, 3, 1, 2)
        if up1:
            x1n = F.interpolate(x1n, scale_factor=2, mode="nearest")
        xin = torch.cat([xin, x1n], 1)
    wr = torch.zeros(cout, cin0 + cin1, 3, 3, requires_grad=True)
    F.conv2d(xin, wr, stride=s, padding=1).backward(dy[..., :cout].permute(0, 3, 1, 2))
    assert rel(dw, wr.grad) < 1e-5


@pytest.mark.parametrize("ws", [0, 16 << 20])
@pytest.mark.parametrize("tile", [25, 26, 27, 28, 29, 30])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cin0,cin1,up1,cout,k,s,H,W,B,dyc", [c for c in WGF_CASES if c[4] == 3]
                         + [(64, 64, 1, 64, 3, 1, 12, 10, 2, 64), (128, 0, 0, 128, 3, 1, 40, 40, 2, 136),
                            (64, 0, 0, 128, 3, 2, 80, 70, 1, 128), (160, 0, 0, 160, 3, 1, 20, 18, 2, 160),
                            (80, 80, 0, 160, 3, 2, 24, 22, 2, 160)])
def test_conv_wgrad9t_16bit_tiles(ws, tile, dtype, cin0, cin1, up1, cout, k, s, H, W, B, dyc):
    """bf16/f16 3x3 weight gradient with all nine taps per block (tiles 25-30: one dY row segment
    and its three input rows staged once, MFMA operands read pixel-transposed by ds_read_b64_tr_b16,
    each lane naming its tap's shifted / strided pixel row) against torch autograd: stride 1 / 2,
    row segments past the image edge, cout / cin tails, two sources (the second upsampled), a wide
    dy view; tile 27 is stride-1 only; 29 / 30 = 160 x 32 / 32 x 160 (yolox_x's 160 channels)."""
    g = torch.Generator().manual_seed(cin0 * 11 + cout + H + tile)
    oh, ow = (H + 2 - 3) // s + 1, (W + 2 - 3) // s + 1
    x0 = torch.randn(B, H, W, cin0, generator=g).to(dtype)
    x1 = torch.randn(B, H >> up1, W >> up1, cin1, generator=g).to(dtype) if cin1 else None
    dy = torch.randn(B, oh, ow, dyc, generator=g).to(dtype)
    keep = [x0.cuda(), dy.cuda()] + ([x1.cuda()] if cin1 else [])
    srcs = [src(keep[0])]
    if cin1:
        srcs.append(src(keep[2], up=up1))
    try:
        dw = wgrad(dtype, srcs, src(keep[1]), cout, cin0 + cin1, 3, s, 1, (H, W), (oh, ow), B, tile=tile,
                   ws_bytes=ws)
    except NotImplementedError as e:
        assert tile == 27 and s == 2, e
        return
    assert not (tile == 27 and s == 2)
    xin = x0.float().permute(0, 3, 1, 2)
    if cin1:
        x1n = x1.float().permute(0, 3, 1, 2)
        if up1:
            x1n = F.interpolate(x1n, scale_factor=2, mode="nearest")
        xin = torch.cat([xin, x1n], 1)
    wr = torch.zeros(cout, cin0 + cin1, 3, 3, requires_grad=True)
    F.conv2d(xin, wr, stride=s, padding=1).backward(dy[..., :cout].float().permute(0, 3, 1, 2))
    assert rel(dw, wr.grad) < 1e-4  # fp32 accumulation of exact products: order-only differences


def test_conv_wgrad_fp32_workspace_is_deterministic():
    """With a workspace the split partials are summed in a fixed order: two runs agree bit for bit."""
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4, 40, 40, 128, generator=g).cuda()
    dy = torch.randn(4, 40, 40, 128, generator=g).cuda()
    a = wgrad(torch.float32, [src(x)], src(dy), 128, 128, 3, 1, 1, (40, 40), (40, 40), 4, tile=17, ws_bytes=32 << 20)
    b = wgrad(torch.float32, [src(x)], src(dy), 128, 128, 3, 1, 1, (40, 40), (40, 40), 4, tile=17, ws_bytes=32 << 20)
    assert torch.equal(a, b)


def test_wgrad_cin_store_and_strided_dy():
    """Focus stem: 16 packed channels, gradient of the 12 real ones; dy read through a
    strided view (the head's [B, A, 8] pred-gradient rows)."""
    g = torch.Generator().manual_seed(3)
    B, H, W, A0 = 2, 8, 8, 5
    x = torch.randn(B, H, W, 16, generator=g)
    rows = torch.randn(B, A0 + H * W + 3, 8, generator=g)
    xd, rd = x.cuda(), rows.cuda()
    from yolox_amd import _native as N
    dys = N.Src()
    dys.ptr = rd.data_ptr() + A0 * 8 * 4
    dys.channels, dys.cstride, dys.bstride, dys.h, dys.w = 8, 8, rows.shape[1] * 8, H, W
    dw = wgrad(torch.float32, [src(xd)], dys, 5, 16, 1, 1, 0, (H, W), (H, W), B, cin_store=12)
    torch.cuda.synchronize()
    dyr = rows[:, A0:A0 + H * W, :5].reshape(B, H, W, 5)
    ref = torch.einsum("bhwn,bhwc->nc", dyr, x[..., :12])
    assert rel(dw.view(5, 12), ref) < 1e-5


@pytest.mark.parametrize("B,H,W,c,dtype", [(2, 9, 10, 16, torch.float32), (2, 40, 40, 20, torch.float32),
                                            (1, 48, 48, 8, torch.float32), (2, 20, 20, 24, torch.float16)])
def test_spp_and_upsample_bwd(B, H, W, c, dtype):
    """SPP max-pool backward (separable gather: 4 / 2 / 1 channels per block by plane size; yolox_x
    @1280 = 40x40) and the nearest-x2 upsample backward vs torch autograd, ties included."""
    g = torch.Generator().manual_seed(11 + H)
    x = torch.randn(B, H, W, c, generator=g).to(dtype).float()
    x[0, 1, 1, :] = x[0, 1, 2, :]  # ties: first max in scan order takes the gradient
    x[-1, H - 2, :, :] = x[-1, H - 1, :, :]
    cat = torch.zeros(B, H, W, 4 * c)
    cat[..., :c] = x
    dcat = torch.randn(B, H, W, 4 * c, generator=g)
    catd = cat.to(dtype).cuda()
    chk(lib().yxh_spp_maxpool(catd.data_ptr(), DT[dtype], B, H, W, c, 4 * c, H * W * 4 * c, stream()))
    dx = torch.empty(B, H, W, c, device="cuda")
    cs = src(catd)
    dcd = dcat.cuda()
    chk(lib().yxh_spp_bwd(DT[dtype], B, C.byref(cs), c, dcd.data_ptr(), dx.data_ptr(), stream()))
    up_g = torch.randn(B, 2 * H, 2 * W, c, generator=g)
    acc = torch.ones(B, H, W, c)
    accd, ugd = acc.cuda(), up_g.cuda()
    chk(lib().yxh_upsample_bwd(ugd.data_ptr(), B, H, W, c, accd.data_ptr(), stream()))
    torch.cuda.synchronize()
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_()
    outs = torch.cat([xr] + [F.max_pool2d(xr, k, 1, k // 2) for k in (5, 9, 13)], 1)
    outs.backward(dcat.permute(0, 3, 1, 2))
    assert rel(catd[..., c:].float(), outs.detach().permute(0, 2, 3, 1)[..., c:]) == 0.0
    assert rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-6
    ref = 1 + up_g.view(B, H, 2, W, 2, c).sum((2, 4))
    assert rel(accd, ref) < 1e-6


# ----------------------------------------------------------------- loss gradient
@pytest.mark.parametrize("use_l1", [False, True])
def test_loss_bwd_matches_autograd(oracle, use_l1):
    """d total_loss / d raw head outputs vs autograd through the oracle's
    forward_train head math (decode + SimOTA targets + losses)."""
    from yolox_amd.models.losses import yolox_losses
    from yolox_amd.weights import synthetic_labels
    B, S, nc = 2, 128, 80
    hw = [(S // 8, S // 8), (S // 16, S // 16), (S // 32, S // 32)]
    A = sum(h * w for h, w in hw)
    g = torch.Generator().manual_seed(5)
    raw = torch.randn(B, A, 5 + nc, generator=g) * 0.5
    raw[..., 4:] -= 2.0
    labels = torch.from_numpy(synthetic_labels(B, S, S, max_gt=8, seed=9))
    xs, ys, st = [], [], []
    for (h, w), s in zip(hw, (8, 16, 32)):
        yv, xv = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
        xs.append(xv.reshape(-1).float()), ys.append(yv.reshape(-1).float()), st.append(torch.full((h * w,), float(s)))
    xs, ys, st = torch.cat(xs), torch.cat(ys), torch.cat(st)
    rawd = raw.cuda()
    preds = torch.empty_like(rawd)
    lhw = (C.c_int32 * 6)(*[v for t in hw for v in t])
    strides = (C.c_int32 * 3)(8, 16, 32)
    chk(lib().yxh_head_decode_train(rawd.data_ptr(), B, A, nc, lhw, strides, 3, preds.data_ptr(), stream()))
    losses, assign = yolox_losses(preds, labels.cuda(), hw, origin_reg=rawd[..., :4].contiguous() if use_l1 else None)
    g_ro = torch.empty(B, A, 8, device="cuda")
    g_cls = torch.empty(B, A, nc, device="cuda")
    gt = torch.full((), 2.0, device="cuda")
    L = labels.shape[1]
    nfg = assign["num_fg"].int().contiguous()
    labd = labels.cuda()
    fgd = assign["fg_mask"].to(torch.uint8).contiguous()
    chk(lib().yxh_yolox_loss_bwd(preds.data_ptr(), rawd.data_ptr(), labd.data_ptr(), B, A, nc, L, lhw,
                                 strides, 3, fgd.data_ptr(),
                                 assign["matched_gt_inds"].data_ptr(), assign["pred_ious"].data_ptr(), nfg.data_ptr(),
                                 gt.data_ptr(), int(use_l1), 0, g_ro.data_ptr(), g_cls.data_ptr(), stream()))
    torch.cuda.synchronize()
    # autograd reference with the device's assignment as fixed targets
    r = raw.clone().requires_grad_()
    dec = torch.cat([(r[..., :2] + torch.stack([xs, ys], 1)) * st[:, None], torch.exp(r[..., 2:4]) * st[:, None],
                     r[..., 4:]], -1)
    fg = assign["fg_mask"].cpu().bool()
    matched = assign["matched_gt_inds"].cpu().long()
    piou = assign["pred_ious"].cpu()
    num_fg = max(int(fg.sum()), 1)
    tot = 0.0
    for b in range(B):
        f = fg[b]
        gtb = labels[b][matched[b][f]]
        tot = tot + 5.0 * oracle.iou_loss(dec[b, f, :4], gtb[:, 1:5]).sum()
        tot = tot + F.binary_cross_entropy_with_logits(r[b, :, 4], f.float(), reduction="sum")
        tgt = F.one_hot(gtb[:, 0].long(), nc).float() * piou[b][f][:, None]
        tot = tot + F.binary_cross_entropy_with_logits(r[b, f, 5:], tgt, reduction="sum")
        if use_l1:
            s_ = st[f]
            l1t = torch.stack([gtb[:, 1] / s_ - xs[f], gtb[:, 2] / s_ - ys[f], torch.log(gtb[:, 3] / s_ + 1e-8),
                               torch.log(gtb[:, 4] / s_ + 1e-8)], 1)
            tot = tot + (r[b, f, :4] - l1t).abs().sum()
    (2.0 * tot / num_fg).backward()
    ref = r.grad
    assert float(losses["total_loss"]) == pytest.approx(float(tot) / num_fg, rel=1e-5)
    assert rel(g_ro[..., :5], ref[..., :5]) < 1e-5
    assert float(g_ro[..., 5:].abs().max()) == 0.0
    assert rel(g_cls, ref[..., 5:]) < 1e-5


# ----------------------------------------------------------------- end to end
def _model_and_batch(seed=0):
    from yolox_amd.config import named_config
    from yolox_amd.weights import synthetic_state_dict
    d = np.load(os.path.join(GOLDEN, "train_yolox_s_128.npz"))
    cfg = named_config("yolox_s")
    m = cfg.get_model()
    sd = synthetic_state_dict(m.state_dict(), seed=seed, bn_stats="yolox_s")
    m.load_state_dict(sd)
    x = torch.from_numpy(d["input_u8"]).permute(0, 3, 1, 2).float()
    return m, sd, x, torch.from_numpy(d["labels"]), d


@pytest.mark.parametrize("use_l1", [False, True])
def test_train_step_fp32_matches_oracle(oracle, use_l1):
    m, sd, x, labels, d = _model_and_batch()
    m = m.cuda().train()
    m.head.use_l1 = use_l1
    out = m(x.cuda(), labels.cuda())
    out["total_loss"].backward()
    torch.cuda.synchronize()
    tag = "l1" if use_l1 else "nol1"
    # losses vs the reference's own values (fixture) and vs the oracle
    for k in ("total_loss", "iou_loss", "conf_loss", "cls_loss", "l1_loss", "num_fg"):
        assert float(out[k]) == pytest.approx(float(d[f"{tag}.{k}"]), rel=1e-3, abs=1e-6), k
    # every parameter gradient vs the oracle's autograd (CPU fp32)
    sdo = {k: v.clone().float().requires_grad_(v.is_floating_point() and "running" not in k
                                               and "num_batches" not in k) for k, v in sd.items()}
    ref = oracle.forward_train(sdo, oracle.ARCHS["yolox_s"], x, labels, use_l1=use_l1)
    ref["total_loss"].backward()
    worst = 0.0
    for name, p in m.named_parameters():
        gr = sdo[name].grad
        assert p.grad is not None, name
        e = rel(p.grad, gr)
        worst = max(worst, e)
        assert e < 1e-3, (name, e)
    # reference fixture gradients (reference autograd on the same seed)
    for key in d.files:
        if key.startswith(f"{tag}.grad."):
            name = key[len(f"{tag}.grad."):]
            assert rel(dict(m.named_parameters())[name].grad, torch.from_numpy(d[key])) < 1e-3, name
    # running statistics were updated once with momentum 0.03
    for name, buf in m.named_buffers():
        if name.endswith("running_mean"):
            assert not torch.equal(buf.cpu(), sd[name]), name
            break


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H,W,Cc,s", [(2, 16, 16, 16, 1), (2, 17, 13, 32, 2), (1, 9, 10, 64, 1), (3, 8, 8, 256, 2),
                                        (2, 40, 40, 24, 2)])
def test_depthwise_gradients(dtype, B, H, W, Cc, s):
    """yxh_dw_wgrad / yxh_dw_dgrad (DWConv.dconv's gradients: F.conv2d(groups=C), 3x3, pad 1,
    stride 1 / 2) against torch fp32 autograd on the same rounded operands; the weight gradient
    twice bit-identical (fixed-order partial sums), the data gradient written or accumulated."""
    from yolox_amd import _native as N
    from yolox_amd.train import dense_src
    g = torch.Generator().manual_seed(B * 1000 + Cc + s)
    x = torch.randn(B, H, W, Cc, generator=g).to(dtype)
    oh, ow = (H + 2 - 3) // s + 1, (W + 2 - 3) // s + 1
    dy = torch.randn(B, oh, ow, Cc, generator=g).to(dtype)
    wt = (torch.randn(Cc, 1, 3, 3, generator=g) * 0.3).to(dtype).float()
    xd, dyd = x.cuda(), dy.cuda()
    wpk = wt.reshape(Cc, 9).to(dtype).cuda().contiguous()
    ws = torch.empty(int(lib().yxh_dw_wgrad_workspace_bytes(B, oh, ow, Cc, 3)), dtype=torch.uint8, device="cuda")
    dws = []
    for _ in range(2):
        dw = torch.full((Cc, 1, 3, 3), float("nan"), device="cuda")
        chk(lib().yxh_dw_wgrad(DT[dtype], B, C.byref(dense_src(xd)), C.byref(dense_src(dyd)), Cc, 3, s, 1, oh, ow,
                               dw.data_ptr(), ws.data_ptr(), ws.numel(), stream()))
        dws.append(dw)
    prev = torch.randn(B, H, W, Cc, generator=g)
    dx = prev.clone().cuda()
    chk(lib().yxh_dw_dgrad(DT[dtype], B, C.byref(dense_src(dyd)), wpk.data_ptr(), Cc, 3, s, 1, H, W, dx.data_ptr(),
                           Cc, H * W * Cc, 1, stream()))
    dx0 = torch.full((B, H, W, Cc), float("nan"), device="cuda")
    chk(lib().yxh_dw_dgrad(DT[dtype], B, C.byref(dense_src(dyd)), wpk.data_ptr(), Cc, 3, s, 1, H, W, dx0.data_ptr(),
                           Cc, H * W * Cc, 0, stream()))
    torch.cuda.synchronize()
    xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_()
    wr = wt.clone().requires_grad_()
    F.conv2d(xr, wr, None, s, 1, 1, Cc).backward(dy.float().permute(0, 3, 1, 2))
    assert torch.equal(dws[0], dws[1])
    assert rel(dws[0], wr.grad) < 1e-5
    want = xr.grad.permute(0, 2, 3, 1)
    assert rel(dx0, want) < 1e-5
    assert rel(dx, want + prev) < 1e-5


@pytest.mark.parametrize("name", ["yolox_m", "yolox_x", "yolox_nano"])
def test_train_step_other_widths_match_oracle(oracle, name):
    """yolox_m / yolox_x widths (48/80-channel CSP halves: concat splits that are not
    K-stage aligned) and yolox_nano (DWConv everywhere: the depthwise convs' gradients on
    yxh_dw_wgrad / yxh_dw_dgrad, network_blocks.py:55-74) train through the HIP path: fp32
    losses and every parameter gradient vs the oracle's autograd (1e-3), and an fp16 autocast
    step (the --fp16 of BASELINE configs[4]) gives a finite loss close to the fp32 one."""
    from yolox_amd.config import named_config
    from yolox_amd.weights import synthetic_images, synthetic_labels, synthetic_state_dict
    m = named_config(name).get_model()
    sd = synthetic_state_dict(m.state_dict(), seed=3, bn_stats=name)
    m.load_state_dict(sd)
    x = torch.from_numpy(synthetic_images(2, 64, 64, seed=5)).permute(0, 3, 1, 2).float()
    labels = torch.from_numpy(synthetic_labels(2, 64, 64, max_gt=6, seed=7))
    m = m.cuda().train()
    out = m(x.cuda(), labels.cuda())
    out["total_loss"].backward()
    torch.cuda.synchronize()
    sdo = {k: v.clone().float().requires_grad_(v.is_floating_point() and "running" not in k
                                               and "num_batches" not in k) for k, v in sd.items()}
    ref = oracle.forward_train(sdo, oracle.ARCHS[name], x, labels, use_l1=False)
    ref["total_loss"].backward()
    for k in ("total_loss", "iou_loss", "conf_loss", "cls_loss", "num_fg"):
        assert float(out[k]) == pytest.approx(float(ref[k]), rel=1e-3, abs=1e-6), k
    for pname, prm in m.named_parameters():
        assert rel(prm.grad, sdo[pname].grad) < 1e-3, pname
    m.load_state_dict(sd)
    m.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.float16):
        out16 = m(x.cuda().half(), labels.cuda())
    out16["total_loss"].backward()
    torch.cuda.synchronize()
    l16 = float(out16["total_loss"])
    assert np.isfinite(l16) and abs(l16 - float(out["total_loss"])) < 0.05 * float(out["total_loss"])
    assert all(torch.isfinite(prm.grad).all() for prm in m.parameters())


def test_train_step_bf16_autocast_close_to_fp32(oracle, monkeypatch):
    """bf16 compute (autocast, as --fp16 training does with fp16) against the oracle's fp32 autograd
    within bounds DERIVED from the oracle run with bf16 storage (oracle.stored_as(bfloat16) in train
    mode), as configs[4]'s fp16 test does: each loss and every parameter gradient with > 1k elements
    may be off the fp32 oracle by at most FACTOR x the emulation's own distance (+ 1e-3 of the
    tensor's max).  Both oracle runs take the device's SimOTA assignment (routed: the matching is
    discrete, so a bf16 rounding that moves one anchor across a level would otherwise swap whole
    loss terms); the oracle's own assignment may differ on at most 5 % of the fg anchors.  Tile
    tuning is off (by-shape tiles)."""
    import yolox_amd.train as T
    from test_gpu_configs import _device_train_step, _f, _oracle_train_step
    monkeypatch.setenv("YOLOX_AMD_TRAIN_TUNE", "0")
    monkeypatch.setattr(T, "_TRAIN_TILES", {})
    FACTOR = 3.0
    m, sd, x, labels, _ = _model_and_batch()
    m = m.cuda().train()
    out16, spp_in = _device_train_step(monkeypatch, m, x, labels, torch.bfloat16)
    assign = {k: v.clone() for k, v in m._train_graph.assign.items()}
    grads = {n: p.grad.cpu().float().clone() for n, p in m.named_parameters() if p.numel() > 1000}
    flips = []
    ref, sdo = _oracle_train_step(oracle, monkeypatch, m, "yolox_s", x, labels, spp_in, assign, flips)
    nfg = int(assign["fg_mask"].bool().sum())
    assert nfg > 0 and sum(flips) <= max(2, 0.05 * nfg), (flips, nfg)
    with oracle.stored_as(torch.bfloat16):
        emu, sde = _oracle_train_step(oracle, monkeypatch, m, "yolox_s", x, labels, spp_in, assign)
    stats = {}
    for k in ("total_loss", "iou_loss", "conf_loss", "cls_loss"):
        r = _f(ref[k])
        d_dev, d_emu = abs(float(out16[k]) - r), abs(_f(emu[k]) - r)
        stats[k] = (d_dev / abs(r), d_emu / abs(r))
        assert d_dev <= FACTOR * d_emu + 1e-3 * abs(r), (k, stats[k])
    for name, g in grads.items():
        gr = sdo[name].grad
        scale = float(gr.abs().max()) + 1e-12
        d_dev = float((g - gr).abs().max()) / scale
        d_emu = float((sde[name].grad - gr).abs().max()) / scale
        stats[name] = (d_dev, d_emu)
        assert d_dev <= FACTOR * d_emu + 1e-3, (name, stats[name])
    worst = max((v[0] / (v[1] + 1e-3), k) for k, v in stats.items())
    print(f"bf16 step (dev, emulation) distances from the fp32 oracle, worst ratio {worst}; "
          f"SimOTA routed from the device, the oracle's own assignment differs on {flips} of {nfg}")


def test_sgd_step_changes_eval_plan():
    """After an optimizer step the eval plan repacks the new weights."""
    m, _, x, labels, _ = _model_and_batch()
    m = m.cuda().train()
    m.eval()
    y0 = m(x.cuda()).clone()
    m.train()
    m(x.cuda(), labels.cuda())["total_loss"].backward()
    torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, nesterov=True).step()
    m.eval()
    y1 = m(x.cuda())
    assert not torch.equal(y0, y1)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_batched_weight_repack_matches_per_conv(monkeypatch, dtype):
    """Steps after the first repack every forward / data-gradient weight layout in ONE
    yxh_pack_weights_batch launch: after an optimizer step, each packed buffer is
    bit-identical to the per-conv yxh_fold_bn_pack / yxh_pack_dgrad_weight result, and the
    step's losses equal those of a per-conv (YOLOX_AMD_BATCH_PACK=0) graph."""
    from yolox_amd import _native as N
    import yolox_amd.train as T
    monkeypatch.setenv("YOLOX_AMD_TRAIN_TUNE", "0")
    monkeypatch.setattr(T, "_TRAIN_TILES", {})
    m, sd, x, labels, _ = _model_and_batch()
    m = m.cuda().train()
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, nesterov=True)

    def step(mod):
        ctx = torch.autocast("cuda", dtype=dtype) if dtype != torch.float32 else torch.autocast("cuda", enabled=False)
        with ctx:
            out = mod(x.cuda(), labels.cuda())
        out["total_loss"].backward()
        return out

    step(m)
    opt.step()
    m.zero_grad(set_to_none=True)
    out = step(m)  # batched repack of the updated weights
    torch.cuda.synchronize()
    g = m._train_graph
    assert g._batched and g._pack_table is not None and g._pack_table[1] == len(g._pack_jobs) > 50
    st = N.stream_ptr()
    for key, (job, elems, _) in g._pack_jobs.items():
        if key[0] == "fwd":
            conv = next(c for c in m.modules() if id(c) == key[1])
            got = g._fwd_w[key[1]][0]
        else:
            conv = next(c for c in m.modules() if id(c) == key[1])
            got = g._dgrad_w[key]
        want = torch.empty_like(got)
        if job.kind == N.PACK_FWD:
            bias = torch.empty(job.cout, dtype=torch.float32, device="cuda")
            chk(lib().yxh_fold_bn_pack(conv.weight.data_ptr(), conv.bias.data_ptr() if conv.bias is not None else None,
                                       None, None, None, None, 0.0, job.cout, job.cin, job.kh, job.kw, job.pad,
                                       DT[dtype], want.data_ptr(), bias.data_ptr(), st))
        else:
            chk(lib().yxh_pack_dgrad_weight(conv.weight.data_ptr(), job.cout, job.cin, job.kh, job.kw, job.c_begin,
                                            job.c_count, job.pad, DT[dtype], want.data_ptr(), st))
        torch.cuda.synchronize()
        assert torch.equal(got.view(torch.int16 if dtype != torch.float32 else torch.int32),
                           want.view(torch.int16 if dtype != torch.float32 else torch.int32)), key
    # the same step through per-conv repacks
    m2, _, _, _, _ = _model_and_batch()
    m2 = m2.cuda().train()
    m2.load_state_dict(m.state_dict())
    m2.train()
    monkeypatch.setenv("YOLOX_AMD_BATCH_PACK", "0")
    ref = step(m2)
    assert not m2._train_graph.batch_pack
    for k in ("total_loss", "iou_loss", "conf_loss", "cls_loss", "num_fg"):
        assert float(out[k]) == float(ref[k]), k


def test_captured_train_step_fp16_gradscaler_matches_eager(monkeypatch):
    """The bench's --fp16 configs[4] form: CapturedTrainStep(grad_scale=scaler._scale) +
    FusedStep.step(scaler) (train_one_iter(captured=...)) against the eager fp16 step with the
    same GradScaler + FusedStep, bit for bit over five steps: losses, every parameter, the EMA
    weights, the scale and the growth tracker.  Step 2 forces an overflow (scale 2^60: every
    replay reads the live scale, so the captured step overflows too) -- a skipped step and a
    backoff of the scale happen between two replays; from step 3 on a scale of 2^10 with
    growth_interval 2 makes it grow after steps 3 and 4."""
    from yolox_amd.optim import FusedStep
    from yolox_amd.trainer import ModelEMA, train_one_iter
    import yolox_amd.train as T
    monkeypatch.setenv("YOLOX_AMD_TRAIN_TUNE", "0")
    monkeypatch.setattr(T, "_TRAIN_TILES", {})
    m1, sd, x, labels, _ = _model_and_batch()
    m2, _, _, _, _ = _model_and_batch()
    xs, ls = x.cuda().half(), labels.cuda()
    runs = []
    for m in (m1, m2):
        m = m.cuda().train()
        opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, nesterov=True)
        ema = ModelEMA(m, 0.9998)
        scaler = torch.amp.GradScaler("cuda", growth_interval=2)
        fused = FusedStep(m, opt, ema)
        train_one_iter(m, opt, xs, ls, amp_dtype=torch.float16, scaler=scaler, ema=ema, fused=fused)  # warm-up
        runs.append([m, opt, ema, scaler, fused, None])
    m, opt, ema, scaler, fused, _ = runs[1]
    opt.zero_grad(set_to_none=True)
    runs[1][5] = T.CapturedTrainStep(m, xs, ls, dtype=torch.float16, grad_scale=scaler._scale)
    scales = []
    for it in range(5):
        if it in (2, 3):  # step 2: forced overflow; step 3: a scale that does not overflow
            for r in runs:
                r[3]._scale.fill_(2.0 ** 60 if it == 2 else 2.0 ** 10)
                r[3]._growth_tracker.zero_()
        outs = []
        for m, opt, ema, scaler, fused, cap in runs:
            outs.append(train_one_iter(m, opt, xs, ls, amp_dtype=torch.float16, scaler=scaler, ema=ema, fused=fused,
                                       captured=cap))
        torch.cuda.synchronize()
        for k in ("total_loss", "iou_loss", "conf_loss", "cls_loss", "num_fg"):
            assert float(outs[0][k]) == float(outs[1][k]), (it, k)
        (a, _, ea, sa, _, _), (b, _, eb, sb, _, _) = runs
        assert torch.equal(sa._scale, sb._scale) and torch.equal(sa._growth_tracker, sb._growth_tracker), it
        for (n, p), q in zip(a.named_parameters(), b.parameters()):
            assert torch.equal(p, q), (it, n)
        for p, q in zip(ea.ema.parameters(), eb.ema.parameters()):
            assert torch.equal(p, q), it
        scales.append(float(sa._scale))
    assert scales[2] == 2.0 ** 59  # the forced overflow: step skipped, scale backed off
    assert scales[3] == 2.0 ** 10 and scales[4] == 2.0 ** 11  # two good steps: grown (growth_interval 2)


@pytest.mark.parametrize("opt_kind", ["sgd", "fused"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_captured_train_step_matches_eager(monkeypatch, dtype, opt_kind):
    """CapturedTrainStep (the forward + reverse pass as hipGraph segments: main-stream graphs
    between weight-gradient forks, side-stream graphs behind events) gives the eager step's
    losses, parameter gradients and BN running statistics bit for bit, over three optimizer
    steps (torch SGD or the fused HIP SGD step) between replays; the replay repacks the
    updated master weights, and another model's eager step runs between two replays
    (allocating and freeing from the caching allocator).  Round 3's version of this test
    failed on the second replay: the five hipMemsetAsync nodes SimOTA's setup captured broke
    every replay after the first (replaced by the sim_init kernel, tools/cap_probe.py)."""
    from yolox_amd.optim import FusedStep
    import yolox_amd.train as T
    monkeypatch.setenv("YOLOX_AMD_TRAIN_TUNE", "0")
    monkeypatch.setattr(T, "_TRAIN_TILES", {})
    m1, sd, x, labels, _ = _model_and_batch()
    m2, _, _, _, _ = _model_and_batch()
    xs, ls = x.cuda(), labels.cuda()
    ctx = ((lambda: torch.autocast("cuda", dtype=dtype)) if dtype != torch.float32
           else (lambda: torch.autocast("cuda", enabled=False)))
    mods = []
    for m in (m1, m2):
        m = m.cuda().train()
        opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, nesterov=True)
        step = FusedStep(m, opt, None).step if opt_kind == "fused" else opt.step
        with ctx():
            m(xs, ls)["total_loss"].backward()  # eager warm-up (tiles, repack table)
        step()
        mods.append((m, opt, step))
    (m1, o1, s1), (m2, o2, s2) = mods
    with ctx():
        cap = T.CapturedTrainStep(m2, xs, ls)
    for it in range(3):
        o1.zero_grad(set_to_none=True)
        with ctx():
            ref = m1(xs, ls)
        ref["total_loss"].backward()
        got = cap(xs, ls)
        torch.cuda.synchronize()
        for k in ("total_loss", "iou_loss", "conf_loss", "cls_loss", "num_fg"):
            assert float(got[k]) == float(ref[k]), (it, k)
        p1, p2 = dict(m1.named_parameters()), dict(m2.named_parameters())
        for name in p1:
            assert torch.equal(p1[name].grad, p2[name].grad), (it, name)
        b1, b2 = dict(m1.named_buffers()), dict(m2.named_buffers())
        for name in b1:
            assert torch.equal(b1[name], b2[name]), (it, name)
        s1()
        s2()
