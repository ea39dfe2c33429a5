"""Per-op parity of the HIP kernels (through the C ABI) against the CPU oracle.

fp32 path: the MFMA f32 instruction is an exact fp32 FMA chain, so the only
difference to the CPU reference is summation order -> tolerance 1e-4 relative.
bf16 / fp16 paths: inputs and weights rounded to 8 / 11 mantissa bits, fp32
accumulation -> tolerance 3e-2 / 5e-3 of the output scale.
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = {torch.float32: 1e-4, torch.bfloat16: 3e-2, torch.float16: 5e-3}


def N():
    from yolox_amd import _native
    return _native


def nhwc(x: torch.Tensor, dtype, cpad=None) -> torch.Tensor:
    t = x.permute(0, 2, 3, 1).contiguous()
    if cpad and cpad > t.shape[-1]:
        t = F.pad(t, (0, cpad - t.shape[-1]))
    return t.to(DEV, dtype).contiguous()


def make_conv(cin, cout, k, s, groups=1, seed=0, bias=False, bn=True):
    g = torch.Generator().manual_seed(seed)
    conv = torch.nn.Conv2d(cin, cout, k, s, (k - 1) // 2, groups=groups, bias=bias)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / np.sqrt(cin // groups * k * k))
        if bias:
            conv.bias.copy_(torch.randn(cout, generator=g) * 0.1)
    bnm = None
    if bn:
        bnm = torch.nn.BatchNorm2d(cout, eps=1e-3)
        with torch.no_grad():
            bnm.weight.uniform_(0.5, 1.5, generator=g)
            bnm.bias.normal_(0, 0.2, generator=g)
            bnm.running_mean.normal_(0, 0.2, generator=g)
            bnm.running_var.uniform_(0.5, 1.5, generator=g)
        bnm.eval()
    return conv, bnm


def pack(conv, bn, dtype, cin_pad=None):
    n = N()
    cout = conv.out_channels
    cin_g = conv.in_channels // conv.groups
    kh, kw = conv.kernel_size
    cin_pad = cin_pad or cin_g
    w = torch.empty(cout * kh * kw * cin_pad, dtype=dtype, device=DEV)
    b = torch.empty(cout, dtype=torch.float32, device=DEV)
    f = lambda t: t.detach().float().contiguous().to(DEV) if t is not None else None  # noqa: E731
    args = [f(conv.weight), f(conv.bias)] + ([f(bn.weight), f(bn.bias), f(bn.running_mean), f(bn.running_var)]
                                             if bn is not None else [None] * 4)
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    n.check(n.lib().yxh_fold_bn_pack(*[p(a) for a in args], float(bn.eps) if bn is not None else 0.0, cout, cin_g,
                                     kh, kw, cin_pad, n.DTYPE_CODE[dtype], w.data_ptr(), b.data_ptr(),
                                     n.stream_ptr()), "pack")
    return w, b


def ref_conv(x, conv, bn, act):
    y = F.conv2d(x, conv.weight, conv.bias, conv.stride, conv.padding, groups=conv.groups)
    if bn is not None:
        y = F.batch_norm(y, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)
    return {"silu": F.silu, "relu": F.relu, "lrelu": lambda t: F.leaky_relu(t, 0.1), "none": lambda t: t}[act](y)


def run_conv(srcs, conv, bn, dtype, act="silu", residual=None, out=None, out_coff=0, out_c=None, tile=0, flags=0,
             pre=None, groups2=False, frag=False, post=None, head=None):
    """srcs: list of (nhwc tensor [B,h,w,C], coff, ch, upsample).  post: (packed weight, bias,
    (post_src tensor, coff, ch) or None, post_dst tensor, coff, post_cout): a 1x1 post conv
    whose output goes to post_dst instead of the conv's own output."""
    n = N()
    B = srcs[0][0].shape[0]
    ups = srcs[0][3]
    in_h, in_w = srcs[0][0].shape[1] << ups, srcs[0][0].shape[2] << ups
    k, s, pd = conv.kernel_size[0], conv.stride[0], conv.padding[0]
    oh, ow = (in_h + 2 * pd - k) // s + 1, (in_w + 2 * pd - k) // s + 1
    cin = sum(c for _, _, c, _ in srcs)
    w, b = pack(conv, bn, dtype, (cin // 2 if groups2 else cin) if conv.groups == 1 else None)
    cout = conv.out_channels
    if out is None:
        out = torch.zeros(B, oh, ow, out_c or cout, dtype=dtype, device=DEV)
    d = n.ConvDesc()
    d.dtype, d.batch, d.in_h, d.in_w, d.out_h, d.out_w = n.DTYPE_CODE[dtype], B, in_h, in_w, oh, ow
    d.cin, d.cout, d.kh, d.kw, d.stride, d.pad, d.groups = cin, cout, k, k, s, pd, conv.groups
    d.nsrc = len(srcs)
    for j, (t, coff, ch, up) in enumerate(srcs):
        sd = d.src[j]
        sd.ptr = t.data_ptr() + coff * t.element_size()
        sd.channels, sd.cstride, sd.bstride = ch, t.shape[3], t.shape[1] * t.shape[2] * t.shape[3]
        sd.h, sd.w, sd.upsample = t.shape[1], t.shape[2], up
    d.weight, d.bias = w.data_ptr(), b.data_ptr()
    if frag:  # the fragment-major copy (yxh_pack_frag) the weight-stationary tiles read
        wf = torch.empty_like(w)
        n.check(n.lib().yxh_pack_frag(w.data_ptr(), cout, k * k, cin // 2 if groups2 else cin, n.DTYPE_CODE[dtype],
                                      wf.data_ptr(), n.stream_ptr()), "pack_frag")
        d.weight_frag = wf.data_ptr()
    if residual is not None:
        t, coff = residual
        d.residual = t.data_ptr() + coff * t.element_size()
        d.res_cstride, d.res_bstride = t.shape[3], t.shape[1] * t.shape[2] * t.shape[3]
    d.dst = out.data_ptr() + out_coff * out.element_size()
    d.dst_dtype = n.DTYPE_CODE[out.dtype]
    d.dst_cstride, d.dst_bstride = out.shape[3], out.shape[1] * out.shape[2] * out.shape[3]
    d.act = n.ACT_CODE[act]
    d.tile = tile
    d.flags = flags
    if pre is not None:  # fused Bottleneck conv1 (packed weight, bias)
        d.pre_weight, d.pre_bias = pre[0].data_ptr(), pre[1].data_ptr()
    if groups2:  # output half g reads source channels [g*cin, (g+1)*cin)
        d.cin = cin // 2
        d.flags = flags | n.CONV_GROUPS2
    if post is not None:
        pw, pb, psrc, pdst, pcoff, pcout = post
        d.post_weight, d.post_bias, d.post_cout = pw.data_ptr(), pb.data_ptr(), pcout
        if psrc is not None:
            t, coff, ch = psrc
            ps = d.post_src
            ps.ptr = t.data_ptr() + coff * t.element_size()
            ps.channels, ps.cstride, ps.bstride = ch, t.shape[3], t.shape[1] * t.shape[2] * t.shape[3]
            ps.h, ps.w = t.shape[1], t.shape[2]
        d.post_dst = pdst.data_ptr() + pcoff * pdst.element_size()
        d.post_dst_cstride, d.post_dst_bstride = pdst.shape[3], pdst.shape[1] * pdst.shape[2] * pdst.shape[3]
    if head is not None:  # head form: (w_cls, b_cls, w_ro, b_ro, rows [B, A, 5+C] fp32, a_off, stride)
        wcl, bcl, wro, bro, rows, a_off, stride = head
        C = wcl.shape[0]
        d.post_weight, d.post_bias, d.post_weight2, d.post_bias2 = wcl.data_ptr(), bcl.data_ptr(), wro.data_ptr(), \
            bro.data_ptr()
        d.post_cout, d.post_cout2, d.post_stride = C, 5, stride
        d.post_dst = rows.data_ptr() + a_off * (5 + C) * 4
        d.post_dst_cstride, d.post_dst_bstride = 5 + C, rows.shape[1] * (5 + C)
    n.check(n.lib().yxh_conv2d(ctypes.byref(d), n.stream_ptr()), "conv2d")
    torch.cuda.synchronize()
    return out


def close(got: torch.Tensor, want: torch.Tensor, dtype):
    got = got.float().cpu()
    scale = want.abs().max().item() + 1e-6
    err = (got - want).abs().max().item() / scale
    assert err < TOL[dtype], f"max rel err {err:.3e} (tol {TOL[dtype]})"


DTYPES = [torch.float32, torch.bfloat16, torch.float16]
GEOMS = [  # cin, cout, k, s, H, W
    (32, 16, 1, 1, 16, 16), (32, 32, 3, 1, 16, 16), (64, 48, 3, 2, 17, 15), (64, 64, 1, 1, 20, 20),
    (64, 80, 1, 1, 8, 8), (128, 128, 3, 1, 10, 10), (128, 256, 3, 2, 12, 12), (96, 192, 1, 1, 7, 9),
    (24, 24, 3, 1, 13, 13), (256, 5, 1, 1, 6, 6), (512, 1024, 1, 1, 4, 4), (16, 32, 3, 1, 9, 11)]


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("geom", GEOMS)
def test_conv_matches_reference(dtype, geom):
    cin, cout, k, s, H, W = geom
    conv, bn = make_conv(cin, cout, k, s, seed=cin + cout + k)
    x = torch.randn(2, cin, H, W, generator=torch.Generator().manual_seed(1))
    y = run_conv([(nhwc(x, dtype), 0, cin, 0)], conv, bn, dtype)
    close(y.permute(0, 3, 1, 2), ref_conv(x, conv, bn, "silu"), dtype)


@pytest.mark.parametrize("act", ["relu", "lrelu", "none"])
def test_conv_activations(act):
    conv, bn = make_conv(32, 32, 3, 1, seed=5)
    x = torch.randn(2, 32, 9, 9)
    y = run_conv([(nhwc(x, torch.float32), 0, 32, 0)], conv, bn, torch.float32, act=act)
    close(y.permute(0, 3, 1, 2), ref_conv(x, conv, bn, act), torch.float32)


@pytest.mark.parametrize("dtype", DTYPES)
def test_two_sources_with_upsample_and_slices(dtype):
    """cat([upsample(a), b]) -> 1x1 conv, with `a` a channel slice of a wider buffer
    (the PAFPN pattern, yolo_pafpn.py:97-99) and the output written into a slice."""
    a_full = torch.randn(2, 192, 5, 6)  # a = channels [64, 192)
    b = torch.randn(2, 64, 10, 12)
    conv, bn = make_conv(128 + 64, 96, 1, 1, seed=9)
    A, Bt = nhwc(a_full, dtype), nhwc(b, dtype)
    out = torch.zeros(2, 10, 12, 160, dtype=dtype, device=DEV)
    run_conv([(A, 64, 128, 1), (Bt, 0, 64, 0)], conv, bn, dtype, out=out, out_coff=32)
    ref = ref_conv(torch.cat([F.interpolate(a_full[:, 64:], scale_factor=2, mode="nearest"), b], 1), conv, bn,
                   "silu")
    close(out[..., 32:128].permute(0, 3, 1, 2), ref, dtype)
    assert out[..., :32].abs().max().item() == 0 and out[..., 128:].abs().max().item() == 0


@pytest.mark.parametrize("dtype", DTYPES)
def test_residual_in_place(dtype):
    """Bottleneck: y = conv(t) + x written over x (network_blocks.py:97-99)."""
    x = torch.randn(2, 64, 12, 12)
    t = torch.randn(2, 32, 12, 12)
    conv, bn = make_conv(32, 32, 3, 1, seed=3)
    X = nhwc(x, dtype)
    run_conv([(nhwc(t, dtype), 0, 32, 0)], conv, bn, dtype, residual=(X, 16), out=X, out_coff=16)
    ref = ref_conv(t, conv, bn, "silu") + x[:, 16:48]
    close(X[..., 16:48].permute(0, 3, 1, 2), ref, dtype)
    close(X[..., :16].permute(0, 3, 1, 2), x[:, :16].to(dtype).float(), dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("s", [1, 2])
def test_depthwise(dtype, s):
    conv, bn = make_conv(48, 48, 3, s, groups=48, seed=11)
    x = torch.randn(2, 48, 13, 11)
    y = run_conv([(nhwc(x, dtype), 0, 48, 0)], conv, bn, dtype)
    close(y.permute(0, 3, 1, 2), ref_conv(x, conv, bn, "silu"), dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("hw,B,C", [((20, 20), 2, 32), ((13, 7), 2, 32), ((40, 40), 2, 32),
                                    ((20, 20), 32, 256), ((20, 20), 64, 512)])
def test_spp_maxpool(dtype, hw, B, C):
    """bit-exact vs torch max_pool2d; the batch-32/64 cases take the 2- and 4-chunk blocks; +-inf,
    zeros and large negatives exercise bf16's order-preserving int16 keys."""
    n = N()
    H, W = hw
    x = torch.randn(B, C, H, W)
    x[:, :, 0, 0], x[:, :, 1, 2], x[:, :, 2, 1] = float("-inf"), float("inf"), 0.0
    x[:, ::3, 3, 3] = -3.0e38
    buf = torch.zeros(B, H, W, 4 * C, dtype=dtype, device=DEV)
    buf[..., :C] = nhwc(x, dtype)
    n.check(n.lib().yxh_spp_maxpool(buf.data_ptr(), n.DTYPE_CODE[dtype], B, H, W, C, 4 * C, H * W * 4 * C,
                                    n.stream_ptr()), "spp")
    torch.cuda.synchronize()
    xr = x.to(dtype).float()
    want = torch.cat([xr] + [F.max_pool2d(xr, k, 1, k // 2) for k in (5, 9, 13)], 1)
    assert torch.equal(buf.float().cpu().permute(0, 3, 1, 2), want)  # max is exact


@pytest.mark.parametrize("layout,idt", [("nchw", torch.float32), ("nhwc", torch.uint8), ("nhwc", torch.bfloat16)])
@pytest.mark.parametrize("dtype", DTYPES)
def test_focus_pack(layout, idt, dtype):
    n = N()
    img = torch.randint(0, 256, (2, 3, 8, 12)).float()
    src = img if layout == "nchw" else img.permute(0, 2, 3, 1)
    src = src.to(DEV, idt).contiguous()
    dst = torch.empty(2, 4, 6, 16, dtype=dtype, device=DEV)
    n.check(n.lib().yxh_focus_pack(src.data_ptr(), n.NCHW if layout == "nchw" else n.NHWC, n.DTYPE_CODE[idt], 2, 8,
                                   12, dst.data_ptr(), n.DTYPE_CODE[dtype], n.stream_ptr()), "focus")
    torch.cuda.synchronize()
    ref = torch.cat([img[..., ::2, ::2], img[..., 1::2, ::2], img[..., ::2, 1::2], img[..., 1::2, 1::2]], 1)
    got = dst.float().cpu()
    assert torch.equal(got[..., :12].permute(0, 3, 1, 2), ref)
    assert got[..., 12:].abs().max().item() == 0


@pytest.mark.parametrize("layout,idt", [("nchw", torch.float32), ("nhwc", torch.uint8), ("nhwc", torch.float16)])
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("hw,cout", [((8, 12), 32), ((70, 198), 16), ((136, 260), 24), ((66, 130), 48),
                                     ((34, 64), 80)])
def test_stem_conv_fused_focus(layout, idt, dtype, hw, cout):
    """yxh_stem_conv (Focus + 3x3 BaseConv as one 6x6 s2 conv on the image) vs the
    reference order: space-to-depth slicing, conv, BN, SiLU in fp32."""
    n = N()
    H, W = hw
    es = torch.empty((), dtype=dtype).element_size()
    if (cout * es) % 16:
        pytest.skip("stem output rows must be whole 16-byte chunks")
    img = torch.randint(0, 256, (2, 3, H, W)).float()
    src = (img if layout == "nchw" else img.permute(0, 2, 3, 1)).to(DEV, idt).contiguous()
    conv, bn = make_conv(12, cout, 3, 1, seed=cout)
    f = lambda t: t.detach().float().contiguous().to(DEV)  # noqa: E731
    args = [f(conv.weight), f(bn.weight), f(bn.bias), f(bn.running_mean), f(bn.running_var)]
    cpad = (cout + 15) // 16 * 16
    w = torch.empty(cpad * 6 * 32, dtype=dtype, device=DEV)
    b = torch.empty(cpad, dtype=torch.float32, device=DEV)
    n.check(n.lib().yxh_stem_pack(*[a.data_ptr() for a in args], float(bn.eps), cout, n.DTYPE_CODE[dtype],
                                  w.data_ptr(), b.data_ptr(), n.stream_ptr()), "stem pack")
    cs = cout + 16  # write into a wider buffer: the extra channels must stay untouched
    dst = torch.full((2, H // 2, W // 2, cs), 7.0, dtype=dtype, device=DEV)
    d = n.StemDesc()
    d.img, d.layout, d.img_dtype = src.data_ptr(), n.NCHW if layout == "nchw" else n.NHWC, n.DTYPE_CODE[idt]
    d.batch, d.h, d.w, d.dtype, d.cout, d.act = 2, H, W, n.DTYPE_CODE[dtype], cout, n.ACT_CODE["silu"]
    d.weight, d.bias, d.dst = w.data_ptr(), b.data_ptr(), dst.data_ptr()
    d.dst_cstride, d.dst_bstride = cs, (H // 2) * (W // 2) * cs
    n.check(n.lib().yxh_stem_conv(ctypes.byref(d), n.stream_ptr()), "stem")
    torch.cuda.synchronize()
    x = torch.cat([img[..., ::2, ::2], img[..., 1::2, ::2], img[..., ::2, 1::2], img[..., 1::2, 1::2]], 1)
    want = ref_conv(x.to(dtype).float(), conv, bn, "silu")
    got = dst.float().cpu().permute(0, 3, 1, 2)
    assert (got[:, cout:] == 7.0).all()
    err = (got[:, :cout] - want).abs().max().item() / want.abs().max().item()
    assert err < TOL[dtype], err


def test_letterbox_identity_and_pad():
    """r == 1 (e.g. 640x480 into 640x640) is an exact copy + 114 padding."""
    from yolox_amd.models.processor import letterbox_batch
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)
    b = rng.integers(0, 256, (640, 320, 3), dtype=np.uint8)
    out = letterbox_batch([a, b], (640, 640)).cpu()
    ref_a = np.full((3, 640, 640), 114, np.float32)
    ref_a[:, :480, :640] = a.transpose(2, 0, 1)
    ref_b = np.full((3, 640, 640), 114, np.float32)
    ref_b[:, :640, :320] = b.transpose(2, 0, 1)
    assert np.array_equal(out[0].numpy(), ref_a) and np.array_equal(out[1].numpy(), ref_b)
    u8 = letterbox_batch([a], (640, 640), "u8_nhwc").cpu().numpy()
    assert np.array_equal(u8[0].transpose(2, 0, 1).astype(np.float32), ref_a)
    bf = letterbox_batch([a, b], (640, 640), "bf16_nhwc").cpu().float().numpy()
    assert np.array_equal(bf[1].transpose(2, 0, 1), ref_b)


def test_letterbox_resize_cases():
    """Downscale paths: exact 2x (cv2 INTER_AREA fast path) and a generic bilinear
    ratio (restated cv2 fixed point; parity unpinned, so checked against a direct
    numpy statement of the same scheme and against float bilinear within 1 LSB)."""
    from yolox_amd.models.processor import letterbox_batch
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, (64, 96, 3), dtype=np.uint8)
    out = letterbox_batch([a], (32, 48)).cpu().numpy()[0]
    ref = ((a[0::2, 0::2].astype(int) + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2] + 2) >> 2)
    assert np.array_equal(out, ref.transpose(2, 0, 1).astype(np.float32))
    b = rng.integers(0, 256, (100, 150, 3), dtype=np.uint8)
    out = letterbox_batch([b], (64, 64)).cpu().numpy()[0]
    r = min(64 / 100, 64 / 150)
    rh, rw = int(100 * r), int(150 * r)
    assert (out[:, rh:, :] == 114).all() and (out[:, :, rw:] == 114).all()
    fl = F.interpolate(torch.from_numpy(b).permute(2, 0, 1)[None].float(), size=(rh, rw), mode="bilinear",
                       align_corners=False)[0].numpy()
    assert np.abs(out[:, :rh, :rw] - fl).max() <= 1.01


# conv_glds (ids 17-25) two-slab staging of the wide tiles spilled to scratch (round 4): not built
GLDS_K2_WITHDRAWN = {17, 18, 20, 23, 24}


@pytest.mark.parametrize("dtype", DTYPES)
def test_every_tile_variant(dtype):
    """All tile configurations x K-slab counts x both kernels (register-staged and
    LDS-DMA) the autotuner may pick agree."""
    conv, bn = make_conv(64, 96, 3, 1, seed=21)
    x = torch.randn(2, 64, 11, 13, generator=torch.Generator().manual_seed(2))
    want = ref_conv(x, conv, bn, "silu")
    X = nhwc(x, dtype)
    for tid in list(range(1, 10)) + list(range(17, 26)):
        for ks in (1, 2):
            if ks == 2 and tid in GLDS_K2_WITHDRAWN:
                with pytest.raises(NotImplementedError, match="spilled"):
                    run_conv([(X, 0, 64, 0)], conv, bn, dtype, tile=2 * tid + ks - 1)
                continue
            y = run_conv([(X, 0, 64, 0)], conv, bn, dtype, tile=2 * tid + ks - 1)
            close(y.permute(0, 3, 1, 2), want, dtype)


ROW_GEOMS = [  # cin, cout, s, H, W (input)
    (64, 96, 1, 11, 13), (24, 64, 1, 83, 41), (128, 64, 1, 20, 20), (64, 128, 2, 40, 40), (32, 48, 2, 17, 35),
    (256, 256, 1, 10, 10), (16, 5, 1, 9, 9)]


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("geom", ROW_GEOMS)
def test_row_tiled_conv3x3(dtype, geom):
    """conv_rows (ids 33-38): every pixel-tile shape x K-slab count, stride 1/2,
    partial channel blocks / cout tiles / spatial tiles, vs the fp32 reference."""
    cin, cout, s, H, W = geom
    conv, bn = make_conv(cin, cout, 3, s, seed=cin + cout)
    x = torch.randn(2, cin, H, W, generator=torch.Generator().manual_seed(s))
    want = ref_conv(x, conv, bn, "silu")
    X = nhwc(x, dtype)
    for tid in range(33, 52):
        for ks in (1, 2):
            epc = 16 // torch.empty((), dtype=dtype).element_size()
            if ks == 2 and cin < 8 * epc:
                with pytest.raises(ValueError, match="2-slab"):
                    run_conv([(X, 0, cin, 0)], conv, bn, dtype, tile=2 * tid + ks - 1)
                continue
            if s == 2 and ks == 2:
                with pytest.raises(NotImplementedError, match="stride 2"):
                    run_conv([(X, 0, cin, 0)], conv, bn, dtype, tile=2 * tid + ks - 1)
                continue
            try:
                y = run_conv([(X, 0, cin, 0)], conv, bn, dtype, tile=2 * tid + ks - 1)
            except NotImplementedError as e:  # variant not built for this dtype / too much LDS
                assert tid > 38 or ks == 2, e
                assert ("bf16/f16 only" in str(e) and dtype == torch.float32) or "160 KiB" in str(e), e
                continue
            close(y.permute(0, 3, 1, 2), want, dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_row_tiled_residual_and_strided_dst(dtype):
    """Bottleneck form: 3x3 conv + in-place residual, output into a channel slice of a
    wider buffer (the CSP concat)."""
    conv, bn = make_conv(64, 64, 3, 1, seed=3)
    x = torch.randn(2, 64, 20, 20, generator=torch.Generator().manual_seed(4))
    r = torch.randn(2, 64, 20, 20, generator=torch.Generator().manual_seed(5))
    want = ref_conv(x, conv, bn, "silu") + r.to(dtype).float()
    buf = torch.zeros(2, 20, 20, 128, dtype=dtype, device=DEV)
    buf[..., 64:] = nhwc(r, dtype)
    for tid in (33, 34, 36):
        buf[..., 64:] = nhwc(r, dtype)
        y = run_conv([(nhwc(x, dtype), 0, 64, 0)], conv, bn, dtype, residual=(buf, 64), out=buf, out_coff=64,
                     tile=2 * tid)
        close(y[..., 64:].permute(0, 3, 1, 2), want, dtype)


PW_GEOMS = [  # cin, cout, H, W
    (32, 16, 16, 16), (64, 64, 20, 20), (96, 192, 7, 9), (256, 5, 6, 6), (128, 80, 33, 17), (512, 256, 4, 4),
    (1024, 512, 4, 4)]


def pw_call(fn, dtype, tid, ks):
    """Run a conv_pw variant; returns None when it is documented as not applicable."""
    try:
        return fn(2 * tid + ks - 1)
    except NotImplementedError as e:
        msg = str(e)
        assert "exceed" in msg or "160 KiB" in msg or (dtype == torch.float32 and "bf16/f16 only" in msg), msg
        return None
    except ValueError as e:
        assert "2-slab" in str(e), e
        return None


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("geom", PW_GEOMS)
def test_streaming_pointwise_conv(dtype, geom):
    """conv_pw (ids 65-70): persistent 1x1 conv with resident weights, every variant
    x K-stage size vs the fp32 reference; at least one variant runs for bf16/f16."""
    cin, cout, H, W = geom
    conv, bn = make_conv(cin, cout, 1, 1, seed=cin + 3 * cout)
    x = torch.randn(3, cin, H, W, generator=torch.Generator().manual_seed(7))
    want = ref_conv(x, conv, bn, "silu")
    X = nhwc(x, dtype)
    ran = 0
    for tid in range(65, 71):
        for ks in (1, 2):
            y = pw_call(lambda t: run_conv([(X, 0, cin, 0)], conv, bn, dtype, tile=t), dtype, tid, ks)
            if y is not None:
                close(y.permute(0, 3, 1, 2), want, dtype)
                ran += 1
    assert ran > 0 or dtype == torch.float32 or cin * 64 * 2 > 64 * 1024


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_streaming_pointwise_two_sources_upsample(dtype):
    """conv_pw on the PAFPN pattern: cat([upsample(slice of a), b]) into an output slice."""
    a_full = torch.randn(2, 192, 5, 6)
    b = torch.randn(2, 64, 10, 12)
    conv, bn = make_conv(128 + 64, 96, 1, 1, seed=9)
    A, Bt = nhwc(a_full, dtype), nhwc(b, dtype)
    ref = ref_conv(torch.cat([F.interpolate(a_full[:, 64:], scale_factor=2, mode="nearest"), b], 1), conv, bn,
                   "silu")
    for tid in range(65, 71):
        for ks in (1, 2):
            out = torch.zeros(2, 10, 12, 160, dtype=dtype, device=DEV)
            y = pw_call(lambda t: run_conv([(A, 64, 128, 1), (Bt, 0, 64, 0)], conv, bn, dtype, out=out, out_coff=32,
                                           tile=t), dtype, tid, ks)
            if y is None:
                continue
            close(out[..., 32:128].permute(0, 3, 1, 2), ref, dtype)
            assert out[..., :32].abs().max().item() == 0 and out[..., 128:].abs().max().item() == 0


def test_streaming_pointwise_rejects_residual_and_3x3():
    conv, bn = make_conv(32, 32, 3, 1, seed=1)
    x = nhwc(torch.randn(1, 32, 8, 8), torch.bfloat16)
    with pytest.raises(NotImplementedError, match="conv_pw"):
        run_conv([(x, 0, 32, 0)], conv, bn, torch.bfloat16, tile=2 * 65)


def test_row_tiled_rejects_other_geometries():
    conv, bn = make_conv(32, 32, 1, 1, seed=1)
    x = nhwc(torch.randn(1, 32, 8, 8), torch.bfloat16)
    with pytest.raises(NotImplementedError, match="conv_rows"):
        run_conv([(x, 0, 32, 0)], conv, bn, torch.bfloat16, tile=2 * 33)


def test_tile_variant_rejected_when_inapplicable():
    n = N()
    conv, bn = make_conv(16, 32, 3, 1, seed=1)
    x = torch.randn(1, 16, 8, 8)
    with pytest.raises(ValueError, match="2-slab"):
        run_conv([(nhwc(x, torch.bfloat16), 0, 16, 0)], conv, bn, torch.bfloat16, tile=2 * 2 + 1)
    with pytest.raises(ValueError, match="tile"):
        run_conv([(nhwc(x, torch.bfloat16), 0, 16, 0)], conv, bn, torch.bfloat16, tile=2 * 12)
    assert n is not None


def _stem_run(src, idt, dtype, H, W, cout, conv, bn, force_tiles=False):
    n = N()
    f = lambda t: t.detach().float().contiguous().to(DEV)  # noqa: E731
    args = [f(conv.weight), f(bn.weight), f(bn.bias), f(bn.running_mean), f(bn.running_var)]
    cpad = (cout + 15) // 16 * 16
    w = torch.empty(cpad * 6 * 32, dtype=dtype, device=DEV)
    b = torch.empty(cpad, dtype=torch.float32, device=DEV)
    n.check(n.lib().yxh_stem_pack(*[a.data_ptr() for a in args], float(bn.eps), cout, n.DTYPE_CODE[dtype],
                                  w.data_ptr(), b.data_ptr(), n.stream_ptr()), "stem pack")
    cs = cout + 16
    dst = torch.full((2, H // 2, W // 2, cs), 7.0, dtype=dtype, device=DEV)
    d = n.StemDesc()
    d.img, d.layout, d.img_dtype = src.data_ptr(), n.NHWC, n.DTYPE_CODE[idt]
    d.batch, d.h, d.w, d.dtype, d.cout, d.act = 2, H, W, n.DTYPE_CODE[dtype], cout, n.ACT_CODE["silu"]
    d.weight, d.bias, d.dst = w.data_ptr(), b.data_ptr(), dst.data_ptr()
    d.dst_cstride, d.dst_bstride = cs, (H // 2) * (W // 2) * cs
    d.reserved = 1 if force_tiles else 0
    n.check(n.lib().yxh_stem_conv(ctypes.byref(d), n.stream_ptr()), "stem")
    torch.cuda.synchronize()
    return dst


@pytest.mark.parametrize("idt", [torch.uint8, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("hw,cout", [((64, 640), 32), ((42, 96), 48), ((20, 16), 80), ((30, 48), 16)])
def test_stem_full_row_strips_match_tiles(idt, dtype, hw, cout):
    """NHWC images whose rows are whole 16-byte chunks take the full-row strip kernel;
    it is bit-identical to the 4x64-tile kernel (forced by yxh_stem_desc.reserved = 1)
    and matches the reference order (space-to-depth, conv, BN, SiLU in fp32)."""
    H, W = hw
    img = torch.randint(0, 256, (2, 3, H, W)).float()
    src = img.permute(0, 2, 3, 1).to(DEV, idt).contiguous()
    conv, bn = make_conv(12, cout, 3, 1, seed=cout + W)
    strip = _stem_run(src, idt, dtype, H, W, cout, conv, bn)
    tiles = _stem_run(src, idt, dtype, H, W, cout, conv, bn, force_tiles=True)
    assert torch.equal(strip, tiles)
    x = torch.cat([img[..., ::2, ::2], img[..., 1::2, ::2], img[..., ::2, 1::2], img[..., 1::2, 1::2]], 1)
    want = ref_conv(x.to(dtype).float(), conv, bn, "silu")
    got = strip.float().cpu().permute(0, 3, 1, 2)
    assert (got[:, cout:] == 7.0).all()
    err = (got[:, :cout] - want).abs().max().item() / want.abs().max().item()
    assert err < TOL[dtype], err


PWR_GEOMS = [  # cin, cout, H, W (cin <= 256: the whole K in registers)
    (32, 16, 16, 16), (64, 64, 20, 20), (96, 192, 7, 9), (256, 5, 6, 6), (128, 80, 33, 17), (256, 256, 4, 4),
    (16, 32, 9, 11), (64, 255, 5, 7)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("geom", PWR_GEOMS)
def test_register_pointwise_conv(dtype, geom):
    """conv_pwr (ids 81-82): 1x1 conv with the pixel operand loaded straight into MFMA
    fragments, both channel tilings, into a compute-dtype and an fp32 destination, vs
    the fp32 reference (ragged pixel / channel tails included)."""
    cin, cout, H, W = geom
    conv, bn = make_conv(cin, cout, 1, 1, seed=cin + 5 * cout)
    x = torch.randn(3, cin, H, W, generator=torch.Generator().manual_seed(11))
    want = ref_conv(x, conv, bn, "silu")
    X = nhwc(x, dtype)
    for tid in (81, 82):
        y = run_conv([(X, 0, cin, 0)], conv, bn, dtype, tile=2 * tid)
        close(y.permute(0, 3, 1, 2), want, dtype)
        out = torch.zeros(3, H, W, cout, dtype=torch.float32, device=DEV)
        run_conv([(X, 0, cin, 0)], conv, bn, dtype, out=out, tile=2 * tid)
        close(out.permute(0, 3, 1, 2), want, dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_register_pointwise_two_sources_upsample(dtype):
    """conv_pwr on the PAFPN pattern: cat([upsample(slice of a), b]) into an output slice."""
    a_full = torch.randn(2, 192, 5, 6)
    b = torch.randn(2, 64, 10, 12)
    conv, bn = make_conv(128 + 64, 96, 1, 1, seed=9)
    A, Bt = nhwc(a_full, dtype), nhwc(b, dtype)
    ref = ref_conv(torch.cat([F.interpolate(a_full[:, 64:], scale_factor=2, mode="nearest"), b], 1), conv, bn,
                   "silu")
    for tid in (81, 82):
        out = torch.zeros(2, 10, 12, 160, dtype=dtype, device=DEV)
        run_conv([(A, 64, 128, 1), (Bt, 0, 64, 0)], conv, bn, dtype, out=out, out_coff=32, tile=2 * tid)
        close(out[..., 32:128].permute(0, 3, 1, 2), ref, dtype)
        assert out[..., :32].abs().max().item() == 0 and out[..., 128:].abs().max().item() == 0


def test_register_pointwise_rejects():
    x = nhwc(torch.randn(1, 32, 8, 8), torch.bfloat16)
    conv3, bn3 = make_conv(32, 32, 3, 1, seed=1)
    with pytest.raises(NotImplementedError, match="conv_pwr"):
        run_conv([(x, 0, 32, 0)], conv3, bn3, torch.bfloat16, tile=2 * 81)
    conv1, bn1 = make_conv(32, 32, 1, 1, seed=2)
    with pytest.raises(NotImplementedError, match="conv_pwr"):
        run_conv([(nhwc(torch.randn(1, 32, 8, 8), torch.float32), 0, 32, 0)], conv1, bn1, torch.float32,
                 tile=2 * 81)
    with pytest.raises(NotImplementedError, match="conv_pwr"):
        run_conv([(x, 0, 32, 0)], conv1, bn1, torch.bfloat16, residual=(x.clone(), 0), tile=2 * 81)
    big, bnb = make_conv(512, 32, 1, 1, seed=3)
    with pytest.raises(NotImplementedError, match="conv_pwr"):
        run_conv([(nhwc(torch.randn(1, 512, 4, 4), torch.bfloat16), 0, 512, 0)], big, bnb, torch.bfloat16,
                 tile=2 * 81)


PWF_GEOMS = [  # cin, cout, H, W
    (32, 16, 16, 16), (64, 64, 20, 20), (128, 80, 33, 17), (512, 256, 4, 4), (1024, 512, 4, 4), (256, 5, 6, 6),
    (64, 192, 7, 9)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("geom", PWF_GEOMS)
def test_dense_pointwise_conv_pwf(dtype, geom):
    """conv_pwf (ids 97-104): dense 1x1 conv with the branch-free LDS-DMA loader, every
    variant (one tile per block / persistent) vs the fp32 reference, incl. pixel and
    channel tails; K stages of 32 or 64 channels (cin not a multiple -> rejected)."""
    cin, cout, H, W = geom
    conv, bn = make_conv(cin, cout, 1, 1, seed=cin + 5 * cout)
    x = torch.randn(3, cin, H, W, generator=torch.Generator().manual_seed(11))
    want = ref_conv(x, conv, bn, "silu")
    X = nhwc(x, dtype)
    ran = 0
    for tid in range(97, 105):
        try:
            y = run_conv([(X, 0, cin, 0)], conv, bn, dtype, tile=2 * tid)
        except NotImplementedError as e:
            assert "multiple" in str(e) or (cout * 2) % 8, e  # K stage / 8-byte output rows
            continue
        close(y.permute(0, 3, 1, 2), want, dtype)
        ran += 1
    assert ran >= 3 or (cout * 2) % 8


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_dense_pointwise_two_sources_slice_dst(dtype):
    """conv_pwf over cat([a, b]) (split on a 64-channel stage boundary) into a channel
    slice of a wider output buffer (the CSP concat)."""
    a = torch.randn(2, 64, 9, 11)
    b = torch.randn(2, 128, 9, 11)
    conv, bn = make_conv(192, 96, 1, 1, seed=13)
    want = ref_conv(torch.cat([a, b], 1), conv, bn, "silu")
    A, Bt = nhwc(a, dtype), nhwc(b, dtype)
    for tid in (99, 100, 101, 102):
        out = torch.zeros(2, 9, 11, 160, dtype=dtype, device=DEV)
        run_conv([(A, 0, 64, 0), (Bt, 0, 128, 0)], conv, bn, dtype, out=out, out_coff=32, tile=2 * tid)
        close(out[..., 32:128].permute(0, 3, 1, 2), want, dtype)
        assert out[..., :32].abs().max().item() == 0 and out[..., 128:].abs().max().item() == 0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_pointwise_pwf_upsampled_first_source(dtype):
    """conv_pwf over cat([upsample2x(a), b]) -- the PAFPN lateral 1x1 -- with `a` a channel
    slice of a wider buffer: the upsampled source's row offsets are rebuilt per pixel tile
    (incl. the pixel tail of the last tile)."""
    a = torch.randn(3, 128, 5, 7)
    b = torch.randn(3, 64, 10, 14)
    conv, bn = make_conv(192, 64, 1, 1, seed=17)
    want = ref_conv(torch.cat([F.interpolate(a, scale_factor=2, mode="nearest"), b], 1), conv, bn, "silu")
    wide = torch.zeros(3, 5, 7, 192, dtype=dtype, device=DEV)
    wide[..., 32:160] = nhwc(a, dtype)
    Bt = nhwc(b, dtype)
    ran = 0
    for tid in range(97, 105):
        try:
            y = run_conv([(wide, 32, 128, 1), (Bt, 0, 64, 0)], conv, bn, dtype, tile=2 * tid)
        except NotImplementedError as e:
            assert "multiple" in str(e), e
            continue
        close(y.permute(0, 3, 1, 2), want, dtype)
        ran += 1
    assert ran >= 4


R3_WITHDRAWN = {125, 127, 135, 136, 137}  # spilled to scratch (round 4): EINVAL; 141 is fp32-only now
R3_GEOMS = [  # cin, cout, s, H, W (input)
    (64, 96, 1, 11, 13), (32, 64, 1, 83, 41), (128, 64, 1, 20, 20), (64, 128, 2, 40, 40), (32, 48, 2, 17, 35),
    (256, 256, 1, 10, 10), (128, 256, 2, 21, 19)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("geom", R3_GEOMS)
def test_conv_r3_3x3(dtype, geom):
    """conv_r3 / conv_r3h (ids 113-152; fp32: the conv_r3h tiles): every tile of the matching stride vs the fp32 reference;
    zero padding comes from the buffer descriptor's range check (image borders, partial
    spatial tiles, channel tails of cout)."""
    cin, cout, s, H, W = geom
    conv, bn = make_conv(cin, cout, 3, s, seed=cin + cout + 7)
    x = torch.randn(2, cin, H, W, generator=torch.Generator().manual_seed(s + 3))
    want = ref_conv(x, conv, bn, "silu")
    X = nhwc(x, dtype)
    ran = 0
    for tid in range(113, 153):
        if tid in R3_WITHDRAWN or (tid == 141 and dtype != torch.float32):
            continue
        try:
            y = run_conv([(X, 0, cin, 0)], conv, bn, dtype, tile=2 * tid)
        except NotImplementedError as e:
            assert "stride" in str(e) or "multiple" in str(e) or (dtype == torch.float32 and "only" in str(e)), e
            continue
        close(y.permute(0, 3, 1, 2), want, dtype)
        ran += 1
    assert ran >= (1 if dtype == torch.float32 else 3)


@pytest.mark.parametrize("s", [1, 2])
def test_conv_r3h_fp32_accumulate(s):
    """The training data-gradient form: fp32 conv_r3h accumulating into an fp32 dst
    (YXH_CONV_ACCUMULATE), no bias/act, vs torch fp32."""
    n = N()
    conv, bn = make_conv(64, 48, 3, s, seed=11)
    x = torch.randn(2, 64, 18, 22, generator=torch.Generator().manual_seed(12))
    want_conv = ref_conv(x, conv, bn, "none")
    base = torch.randn(want_conv.shape, generator=torch.Generator().manual_seed(13))
    out = nhwc(base, torch.float32).contiguous()
    ran = 0
    for tid in (141, 142, 143, 144, 145, 150, 151, 152):
        out.copy_(nhwc(base, torch.float32))
        try:
            run_conv([(nhwc(x, torch.float32), 0, 64, 0)], conv, bn, torch.float32, act="none", out=out, tile=2 * tid,
                     flags=n.CONV_ACCUMULATE)
        except NotImplementedError as e:
            assert "stride" in str(e), e
            continue
        close(out.permute(0, 3, 1, 2), base + want_conv, torch.float32)
        ran += 1
    assert ran >= 1


@pytest.mark.parametrize("dtype", [torch.bfloat16])
def test_conv_r3_residual_and_strided_dst(dtype):
    conv, bn = make_conv(64, 64, 3, 1, seed=3)
    x = torch.randn(2, 64, 20, 20, generator=torch.Generator().manual_seed(4))
    r = torch.randn(2, 64, 20, 20, generator=torch.Generator().manual_seed(5))
    want = ref_conv(x, conv, bn, "silu") + r.to(dtype).float()
    buf = torch.zeros(2, 20, 20, 128, dtype=dtype, device=DEV)
    for tid in (113, 117, 126, 133, 138, 140, 142, 144, 150):
        buf[..., 64:] = nhwc(r, dtype)
        y = run_conv([(nhwc(x, dtype), 0, 64, 0)], conv, bn, dtype, residual=(buf, 64), out=buf, out_coff=64,
                     tile=2 * tid)
        close(y[..., 64:].permute(0, 3, 1, 2), want, dtype)


WS_WITHDRAWN = {169, 170}  # spilled to scratch / missed the occupancy target (round 4): EINVAL now
WS_GEOMS = [  # cin, cout, s, H, W (input), batch
    (32, 32, 1, 37, 45, 3), (32, 64, 2, 66, 70, 2), (64, 64, 1, 80, 80, 8), (64, 128, 2, 42, 38, 2),
    (128, 128, 1, 40, 40, 16), (128, 256, 1, 20, 22, 2), (128, 96, 2, 41, 40, 2), (256, 256, 1, 20, 20, 4),
    (256, 64, 1, 9, 11, 2)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("geom", WS_GEOMS)
def test_conv_ws_3x3(dtype, geom):
    """conv_ws (ids 161-190): weight-stationary persistent 3x3 conv, every variant built for
    this (cin, stride) vs the fp32 reference: partial spatial tiles, cout tails, several
    tiles per persistent block, K split over waves, a channel-slice source."""
    cin, cout, s, H, W, B = geom
    conv, bn = make_conv(cin, cout, 3, s, seed=cin + cout + s)
    x = torch.randn(B, cin, H, W, generator=torch.Generator().manual_seed(H + W))
    want = ref_conv(x, conv, bn, "silu")
    wide = torch.zeros(B, H, W, cin + 32, dtype=dtype, device=DEV)
    wide[..., 16:16 + cin] = nhwc(x, dtype)
    ran = 0
    for tid in range(161, 191):
        if tid in WS_WITHDRAWN:
            continue
        try:
            y = run_conv([(wide, 16, cin, 0)], conv, bn, dtype, tile=2 * tid)
        except NotImplementedError as e:
            assert "input channels" in str(e), e
            continue
        close(y.permute(0, 3, 1, 2), want, dtype)
        if cout % 16 == 0:  # fragment-major weights: the same values, bit for bit
            yf = run_conv([(wide, 16, cin, 0)], conv, bn, dtype, tile=2 * tid, frag=True)
            assert torch.equal(yf, y), tid
        ran += 1
    assert ran >= 1


@pytest.mark.parametrize("geom", [(128, 128, 1, 40, 40, 4), (64, 64, 1, 37, 45, 3), (160, 160, 1, 40, 38, 2),
                                  (256, 256, 1, 20, 20, 8)])
def test_conv_ws_no_activation(geom):
    """Round 6 (YXH_WS_ACT_CT / YXH_WS1_ACT_CT): the one-wave-per-SIMD conv_ws / conv_ws1 tiles run one
    copy of their tile loop per activation -- the no-activation copy (the 16-bit training forward's
    convs, BatchNorm applied after) vs torch fp32, every tile built for this cin, and the SiLU copy
    of the same tiles on the same input."""
    cin, cout, s, H, W, B = geom
    dtype = torch.bfloat16
    for k in ((3, 1) if cin != 160 else (3,)):
        conv, bn = make_conv(cin, cout, k, s, seed=cin + cout + k)
        x = torch.randn(B, cin, H, W, generator=torch.Generator().manual_seed(H + k))
        tids = (list(range(161, 191)) + list(range(261, 281))) if k == 3 else \
            (list(range(201, 211)) + list(range(241, 249)) + [253, 254, 255, 257, 258])
        ran = 0
        for act in ("none", "silu"):
            want = ref_conv(x, conv, bn, act)
            for tid in tids:
                if tid in WS_WITHDRAWN or tid in {270, 273, 275, 277, 278}:
                    continue
                try:
                    y = run_conv([(nhwc(x, dtype), 0, cin, 0)], conv, bn, dtype, act=act, tile=2 * tid)
                except NotImplementedError as e:
                    assert "input channels" in str(e), e
                    continue
                close(y.permute(0, 3, 1, 2), want, dtype)
                ran += 1
        assert ran >= 2, (geom, k)


WS_WIDE_WITHDRAWN = {270, 273, 275, 277, 278}  # spilled (10- / 16-wave blocks): EINVAL
WS_WIDE_GEOMS = [  # cin, cout, s, H, W (input), batch: yolox_x (80 / 160 / 320) and yolox_l (512) 3x3s
    (80, 80, 1, 35, 41, 2), (80, 160, 2, 66, 70, 2), (160, 160, 1, 40, 38, 2), (160, 320, 2, 42, 38, 2),
    (320, 320, 1, 20, 22, 2), (320, 320, 2, 20, 20, 2), (320, 640, 2, 21, 19, 2), (512, 512, 1, 12, 14, 2),
    (320, 96, 1, 9, 7, 3), (16, 80, 1, 40, 36, 2)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("geom", WS_WIDE_GEOMS)
def test_conv_ws_3x3_wide_channels(dtype, geom):
    """conv_ws tiles 261-280 (80 -- as K 96 with zero chunks --, 160, 320, 512 input channels: the
    yolox_x / yolox_l 3x3s) vs the fp32 reference: every variant built for this (cin, stride),
    channel-slice sources, partial tiles, cout tails, K split over up to ten waves."""
    cin, cout, s, H, W, B = geom
    conv, bn = make_conv(cin, cout, 3, s, seed=cin + cout + s)
    x = torch.randn(B, cin, H, W, generator=torch.Generator().manual_seed(H + W))
    want = ref_conv(x, conv, bn, "silu")
    wide = torch.zeros(B, H, W, cin + 32, dtype=dtype, device=DEV)
    wide[..., 16:16 + cin] = nhwc(x, dtype)
    ran = 0
    for tid in list(range(261, 281)) + [289]:  # 289: the training stem's 16 -> 80 (K 32, upper half zero)
        if tid in WS_WIDE_WITHDRAWN:
            continue
        try:
            y = run_conv([(wide, 16, cin, 0)], conv, bn, dtype, tile=2 * tid)
        except NotImplementedError as e:
            assert "input channels" in str(e), e
            continue
        close(y.permute(0, 3, 1, 2), want, dtype)
        if cout % 16 == 0 and cin % 32 == 0:  # fragment-major weights: the same values, bit for bit
            yf = run_conv([(wide, 16, cin, 0)], conv, bn, dtype, tile=2 * tid, frag=True)
            assert torch.equal(yf, y), tid
        ran += 1
    assert ran >= 1, geom


POST_GEOMS = [  # cin(=cout), stride, post_src channels, post_cout, H, W (input), batch
    (32, 1, 32, 64, 37, 45, 3), (32, 1, 32, 64, 160, 160, 2), (64, 1, 64, 128, 40, 24, 3),
    (64, 1, 64, 128, 80, 80, 4), (64, 2, 0, 128, 42, 38, 2), (64, 2, 0, 128, 160, 160, 2)]


@pytest.mark.parametrize("residual", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("geom", POST_GEOMS)
def test_conv_ws_post_conv(dtype, geom, residual):
    """conv_ws post tiles (ids 221-230, round 4): a Bottleneck's 3x3 (+ shortcut) followed by
    CspLayer.conv3 over [y | x_2] (network_blocks.py:95-99, 180-183), or a stage's stride-2 3x3
    followed by its CspLayer conv1 | conv2 (darknet.py:148-156, network_blocks.py:176-178), in
    one launch -- y never leaves LDS.  vs torch fp32 with y rounded to the compute dtype as the
    split launches store it; partial tiles, channel-slice sources / destinations, the
    destination's other channels untouched, every post tile built for the shape."""
    cin, s, c2, pout, H, W, B = geom
    if residual and s == 2:
        pytest.skip("stride-2 convs have no shortcut")
    conv, bn = make_conv(cin, cin if s == 1 else 2 * cin, 3, s, seed=cin + H)
    cout = conv.out_channels
    pconv, pbn = make_conv(cout + c2, pout, 1, 1, seed=cin + W)
    g = torch.Generator().manual_seed(H * W + cin)
    x = torch.randn(B, cin, H, W, generator=g)
    oh, ow = (H - 1) // s + 1, (W - 1) // s + 1
    r = torch.randn(B, cout, oh, ow, generator=g)
    x2 = torch.randn(B, c2, oh, ow, generator=g) if c2 else None
    y = ref_conv(x, conv, bn, "silu") + (r.to(dtype).float() if residual else 0)
    yq = y.to(dtype).float()
    zin = torch.cat([yq, x2.to(dtype).float()], 1) if c2 else yq
    want = ref_conv(zin, pconv, pbn, "silu")
    X = nhwc(x, dtype)
    R = nhwc(r, dtype, cout + 8)  # residual in a wider buffer
    X2 = torch.zeros(B, oh, ow, c2 + 32, dtype=dtype, device=DEV)
    if c2:
        X2[..., 32:] = nhwc(x2, dtype)
    pw, pb = pack(pconv, pbn, dtype)
    ran = 0
    for tid in range(221, 231):
        Z = torch.full((B, oh, ow, pout + 16), 3.0, dtype=dtype, device=DEV)
        try:
            run_conv([(X, 0, cin, 0)], conv, bn, dtype, residual=(R, 0) if residual else None, tile=2 * tid,
                     post=(pw, pb, (X2, 32, c2) if c2 else None, Z, 8, pout))
        except NotImplementedError:
            continue
        close(Z[..., 8:8 + pout].permute(0, 3, 1, 2), want, dtype)
        assert (Z[..., :8] == 3.0).all() and (Z[..., 8 + pout:] == 3.0).all()
        ran += 1
    assert ran >= 1
    with pytest.raises(NotImplementedError):  # plain tiles refuse a post conv
        run_conv([(X, 0, cin, 0)], conv, bn, dtype, tile=2 * 166,
                 post=(pw, pb, (X2, 32, c2) if c2 else None, torch.zeros(B, oh, ow, pout, dtype=dtype, device=DEV),
                       0, pout))


@pytest.mark.parametrize("geom", POST_GEOMS)
def test_conv_ws_post_conv_bit_exact_vs_two_launches(geom):
    """A post tile computes exactly what the two launches it replaces compute: the plain
    conv_ws tile with the same wave tiling (same MFMA order, y rounded to bf16) storing y, then
    a dense 1x1 (conv_pwf: K in the same 32-deep order) over [y | x_2] -- bit for bit."""
    cin, s, c2, pout, H, W, B = geom
    dtype = torch.bfloat16
    conv, bn = make_conv(cin, cin if s == 1 else 2 * cin, 3, s, seed=cin + H + 1)
    cout = conv.out_channels
    pconv, pbn = make_conv(cout + c2, pout, 1, 1, seed=cin + W + 1)
    g = torch.Generator().manual_seed(H * W + cin + 1)
    X = nhwc(torch.randn(B, cin, H, W, generator=g), dtype)
    oh, ow = (H - 1) // s + 1, (W - 1) // s + 1
    residual = s == 1
    cat = torch.zeros(B, oh, ow, cout + c2, dtype=dtype, device=DEV)
    if residual:
        cat[..., :cout] = nhwc(torch.randn(B, cout, oh, ow, generator=g), dtype)
    if c2:
        cat[..., cout:] = nhwc(torch.randn(B, c2, oh, ow, generator=g), dtype)
    pw, pb = pack(pconv, pbn, dtype)
    plain = {(32, 1): 178, (64, 1): 166, (64, 2): 168}[(cin, s)]  # conv_ws ids 18 / 6 / 8
    post = {(32, 1): 221, (64, 1): 223, (64, 2): 225}[(cin, s)]   # the same wave tiling + post conv
    Z = torch.zeros(B, oh, ow, pout, dtype=dtype, device=DEV)
    run_conv([(X, 0, cin, 0)], conv, bn, dtype, residual=(cat, 0) if residual else None, tile=2 * post,
             post=(pw, pb, (cat, cout, c2) if c2 else None, Z, 0, pout))
    y = run_conv([(X, 0, cin, 0)], conv, bn, dtype, residual=(cat, 0) if residual else None, out=cat.clone(),
                 tile=2 * plain)
    z = run_conv([(y, 0, cout + c2, 0)], pconv, pbn, dtype, tile=2 * 97)
    assert torch.equal(Z, z), (Z.float() - z.float()).abs().max().item()


@pytest.mark.parametrize("cin,plain,chain,H,W,B", [
    (64, 165, 232, 40, 36, 3), (64, 165, 234, 21, 19, 2), (128, 187, 235, 20, 20, 4), (128, 186, 236, 13, 22, 2)])
def test_conv_ws_bottleneck_chain_bit_exact_vs_two_launches(cin, plain, chain, H, W, B):
    """Chain tiles (ids 232 / 234-236, YXH_CONV_POST_STORE, round 4): Bottleneck i's 3x3 + shortcut
    with Bottleneck i+1's conv1 as the post conv (network_blocks.py:95-99 in a CspLayer's chain)
    store the 3x3's output AND the 1x1 over it, bit for bit what the plain conv_ws tile (same
    K order) + a dense 1x1 (conv_pwf) compute; in place over the shortcut buffer, as planned."""
    n = N()
    dtype = torch.bfloat16
    conv, bn = make_conv(cin, cin, 3, 1, seed=cin + H)
    pconv, pbn = make_conv(cin, cin, 1, 1, seed=cin + W)
    g = torch.Generator().manual_seed(H * W + cin)
    T = nhwc(torch.randn(B, cin, H, W, generator=g), dtype)
    X1 = nhwc(torch.randn(B, cin, H, W, generator=g), dtype)
    pw, pb = pack(pconv, pbn, dtype)
    y_ref = run_conv([(T, 0, cin, 0)], conv, bn, dtype, residual=(X1, 0), out=torch.zeros_like(X1), tile=2 * plain)
    z_ref = run_conv([(y_ref, 0, cin, 0)], pconv, pbn, dtype, tile=2 * 97)
    Y = X1.clone()  # the chain runs in place over its shortcut
    Z = torch.zeros_like(X1)
    run_conv([(T, 0, cin, 0)], conv, bn, dtype, residual=(Y, 0), out=Y, tile=2 * chain, flags=n.CONV_POST_STORE,
             post=(pw, pb, None, Z, 0, cin))
    assert torch.equal(Y, y_ref), (Y.float() - y_ref.float()).abs().max().item()
    assert torch.equal(Z, z_ref), (Z.float() - z_ref.float()).abs().max().item()
    # default chain tile (tile 0) and the flag's argument checks
    Z0 = torch.zeros_like(X1)
    Y0 = X1.clone()
    run_conv([(T, 0, cin, 0)], conv, bn, dtype, residual=(Y0, 0), out=Y0, flags=n.CONV_POST_STORE,
             post=(pw, pb, None, Z0, 0, cin))
    assert torch.equal(Y0, y_ref) and torch.equal(Z0, z_ref)
    with pytest.raises(ValueError, match="POST_STORE"):
        run_conv([(T, 0, cin, 0)], conv, bn, dtype, flags=n.CONV_POST_STORE)


@pytest.mark.parametrize("hw", [(80, 80), (20, 22), (13, 8)])
def test_conv_ws_head_form_bit_exact_vs_two_launches(hw):
    """Head-form tiles (ids 231 / 233, round 4): a level's cls_convs[k][1] | reg_convs[k][1]
    (two groups) with each group's preds + decode in the same launch compute exactly what the
    two launches they replace compute -- the plain two-group conv_ws tile with the same wave
    tiling storing [cls | reg], then yxh_head_pred over it (yolo_head.py:149-251) -- bit for
    bit, into rows [a_off, a_off + h*w) of a wider [B, A, 85] output (other rows untouched)."""
    import ctypes as Cc
    n = N()
    H, W = hw
    B, cin, C, stride = 3, 128, 80, 8.0
    A, a_off = H * W + 40, 24
    dtype = torch.bfloat16
    conv, bn = make_conv(cin, 2 * cin, 3, 1, seed=H + 5)
    g = torch.Generator().manual_seed(H * W)
    X = nhwc(torch.randn(B, 2 * cin, H, W, generator=g), dtype)
    wro = (torch.randn(5, cin, generator=g) / cin ** 0.5).to(DEV, dtype)
    wcl = (torch.randn(C, cin, generator=g) / cin ** 0.5).to(DEV, dtype)
    bro = (torch.randn(5, generator=g) * 0.2).to(DEV)
    bcl = (torch.randn(C, generator=g) * 0.2 - 2).to(DEV)
    for plain, fused in ((185, 231), (186, 233)):
        y = run_conv([(X, 0, 2 * cin, 0)], conv, bn, dtype, tile=2 * plain, groups2=True)
        ref = torch.full((B, A, 5 + C), -7.0, device=DEV)
        d = n.HeadDesc()
        d.dtype, d.batch, d.h, d.w, d.cin, d.num_classes = n.DTYPE_CODE[dtype], B, H, W, cin, C
        esz = y.element_size()
        for src, off in ((d.reg, cin), (d.cls, 0)):
            src.ptr = y.data_ptr() + off * esz
            src.channels, src.cstride, src.bstride, src.h, src.w, src.upsample = cin, 2 * cin, H * W * 2 * cin, H, W, 0
        d.w_reg, d.b_reg, d.w_cls, d.b_cls = wro.data_ptr(), bro.data_ptr(), wcl.data_ptr(), bcl.data_ptr()
        d.out, d.out_bstride, d.a_off, d.stride, d.train = ref.data_ptr(), A * (5 + C), a_off, stride, 0
        n.check(n.lib().yxh_head_pred(Cc.byref(d), n.stream_ptr()), "head_pred")
        got = torch.full((B, A, 5 + C), -7.0, device=DEV)
        run_conv([(X, 0, 2 * cin, 0)], conv, bn, dtype, tile=2 * fused, groups2=True,
                 head=(wcl, bcl, wro, bro, got, a_off, stride))
        torch.cuda.synchronize()
        assert torch.equal(got, ref), (fused, (got - ref).abs().max().item())
        assert (got[:, :a_off] == -7.0).all() and (got[:, a_off + H * W:] == -7.0).all()


def test_pack_frag_layout():
    """yxh_pack_frag: block (nf, tap, kb) of 1 KiB, lane l = 16 q + r holds channel 16 nf + r,
    inputs 32 kb + 8 q .. + 8 -- against the same permutation done in torch."""
    n = N()
    cout, taps, cin = 48, 9, 64
    w = torch.randn(cout, taps, cin).to(torch.bfloat16).to(DEV)
    out = torch.empty_like(w)
    n.check(n.lib().yxh_pack_frag(w.data_ptr(), cout, taps, cin, n.BF16, out.data_ptr(), n.stream_ptr()), "pack_frag")
    want = w.view(cout // 16, 16, taps, cin // 32, 4, 8).permute(0, 2, 3, 4, 1, 5).reshape(-1)
    assert torch.equal(out.view(-1), want)
    with pytest.raises(ValueError):
        n.check(n.lib().yxh_pack_frag(w.data_ptr(), 40, taps, cin, n.BF16, out.data_ptr(), n.stream_ptr()))


PW1F_GEOMS = [  # sources (channels, upsample), cout, H, W (output), batch
    ([(64, 0)], 64, 20, 24, 2), ([(128, 0)], 85, 8, 10, 2), ([(48, 0), (48, 0)], 64, 10, 14, 3),
    ([(64, 1), (64, 0)], 128, 8, 12, 2), ([(512, 0)], 256, 5, 7, 4), ([(32, 0)], 32, 40, 40, 2)]


@pytest.mark.parametrize("geom", PW1F_GEOMS)
def test_conv_pw1f_fp32(geom):
    """conv_pw1f (ids 211-214): fp32 1x1 GEMM of the training path vs torch fp32 -- one or two
    sources (the first nearest-x2 upsampled), cout tails (the head preds' 85), a channel-slice
    destination, and YXH_CONV_ACCUMULATE (data gradients add into the input gradient)."""
    srcs, cout, H, W, B = geom
    cin = sum(c for c, _ in srcs)
    conv, bn = make_conv(cin, cout, 1, 1, seed=cin + cout)
    g = torch.Generator().manual_seed(H * W + cin)
    parts, bufs = [], []
    for c, up in srcs:
        x = torch.randn(B, c, H >> up, W >> up, generator=g)
        parts.append(F.interpolate(x, scale_factor=2, mode="nearest") if up else x)
        bufs.append((nhwc(x, torch.float32), 0, c, up))
    want = ref_conv(torch.cat(parts, 1), conv, bn, "silu")
    ran = 0
    cpad = (cout + 3) // 4 * 4 + 8  # 16-byte pixel rows (the kernel's store granule)
    for tid in range(211, 215):
        out = torch.zeros(B, H, W, cpad, dtype=torch.float32, device=DEV)
        y = run_conv(bufs, conv, bn, torch.float32, out=out, out_coff=4, tile=2 * tid)
        close(y[..., 4:4 + cout].permute(0, 3, 1, 2), want, torch.float32)
        assert not y[..., :4].any() and not y[..., 4 + cout:].any()
        out.fill_(0.25)  # accumulate onto it (no activation: a data gradient)
        y = run_conv(bufs, conv, bn, torch.float32, act="none", out=out, out_coff=4, tile=2 * tid,
                     flags=N().CONV_ACCUMULATE)
        close(y[..., 4:4 + cout].permute(0, 3, 1, 2) - 0.25, ref_conv(torch.cat(parts, 1), conv, bn, "none"),
              torch.float32)
        ran += 1
    assert ran == 4


@pytest.mark.parametrize("ch,H,W,B", [(32, 37, 45, 2), (64, 40, 24, 3), (128, 20, 22, 4), (64, 80, 80, 4)])
@pytest.mark.parametrize("shortcut", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_conv_ws_fused_bottleneck(ch, H, W, B, shortcut, dtype):
    """Fused Bottleneck (ids 191-196; network_blocks.py:77-99): conv1 1x1 + SiLU computed on
    the 3x3's halo in LDS (zero outside the image), conv2 3x3 + SiLU, + x, vs torch fp32 on
    the same rounded operands (t rounded to the compute dtype as the kernel holds it)."""
    c1, bn1 = make_conv(ch, ch, 1, 1, seed=ch + 1)
    c3, bn3 = make_conv(ch, ch, 3, 1, seed=ch + 2)
    x = torch.randn(B, ch, H, W, generator=torch.Generator().manual_seed(H * W))
    xq = x.to(dtype).float()
    w1, b1 = pack(c1, bn1, dtype, ch)
    t = ref_conv(xq, c1, bn1, "silu").to(dtype).float()
    want = ref_conv(t, c3, bn3, "silu") + (xq if shortcut else 0)
    X = nhwc(x, dtype)
    ran = 0
    for tid in range(191, 197):
        try:
            y = run_conv([(X, 0, ch, 0)], c3, bn3, dtype, residual=(X, 0) if shortcut else None, tile=2 * tid,
                         pre=(w1, b1))
        except NotImplementedError as e:
            assert "input channels" in str(e), e
            continue
        close(y.permute(0, 3, 1, 2), want, dtype)
        ran += 1
    assert ran >= 1
    with pytest.raises(NotImplementedError):  # a plain tile refuses a fused descriptor
        run_conv([(X, 0, ch, 0)], c3, bn3, dtype, tile=2 * 166, pre=(w1, b1))


@pytest.mark.parametrize("c0,c1,cout,H,W,B", [(256, 256, 256, 40, 40, 3), (128, 128, 128, 30, 22, 2),
                                             (256, 256, 256, 14, 10, 5), (256, 256, 256, 40, 40, 16)])
def test_conv_ws1_upsampled_source(c0, c1, cout, H, W, B):
    """conv_ws1 tiles 249-252 (round 4): a 1x1 over [nearest-x2 upsample(src0) | src1] -- the
    PAFPN's C3_p4 / C3_p3 conv1 | conv2 over the upsampled lateral map and the backbone map
    (yolo_pafpn.py:98-112) -- vs torch fp32; src0 a channel slice of a wider half-resolution
    buffer."""
    dtype = torch.bfloat16
    conv, bn = make_conv(c0 + c1, cout, 1, 1, seed=c0 + H)
    g = torch.Generator().manual_seed(H * W + c0)
    x0 = torch.randn(B, c0, H // 2, W // 2, generator=g)
    x1 = torch.randn(B, c1, H, W, generator=g)
    buf0 = torch.zeros(B, H // 2, W // 2, c0 + 64, dtype=dtype, device=DEV)
    buf0[..., 32:32 + c0] = nhwc(x0, dtype)
    X1 = nhwc(x1, dtype)
    want = ref_conv(torch.cat([F.interpolate(x0, scale_factor=2, mode="nearest"), x1], 1), conv, bn, "silu")
    srcs = [(buf0, 32, c0, 1), (X1, 0, c1, 0)]
    ran = 0
    for tid in list(range(249, 253)) + [256]:
        try:
            y = run_conv(srcs, conv, bn, dtype, tile=2 * tid)
        except NotImplementedError as e:
            assert "input channels" in str(e), e
            continue
        close(y.permute(0, 3, 1, 2), want, dtype)
        assert torch.equal(run_conv(srcs, conv, bn, dtype, tile=2 * tid), y), tid  # deterministic
        ran += 1
    assert ran >= 1


WS1_GEOMS = [  # sources (channels, buffer channels, channel offset), cout, H, W, batch
    ([(64, 64, 0)], 64, 37, 45, 3), ([(32, 64, 0), (32, 32, 0)], 64, 40, 24, 2), ([(128, 160, 16)], 128, 20, 21, 4),
    ([(128, 256, 0), (128, 128, 0)], 256, 20, 20, 2), ([(256, 256, 0)], 128, 23, 17, 3),
    ([(256, 512, 256), (256, 256, 0)], 512, 11, 13, 4), ([(1024, 1024, 0)], 512, 10, 10, 4),
    ([(256, 256, 0)], 256, 40, 40, 32), ([(128, 128, 0)], 256, 19, 23, 2), ([(512, 512, 0)], 256, 12, 14, 3),
    ([(256, 256, 0)], 240, 9, 11, 2),
    # the bench's 20x20 x 32 shapes: several pixel tiles per block, so the 3-4-buffer row pipelines run
    # with tiles in flight beside the K-split partial exchange (tiles 246 / 255 / 256: that exchange once sat
    # on the third row buffer -- nondeterministic outputs, caught by the configs[1] replay check)
    ([(512, 512, 0)], 256, 20, 20, 32), ([(256, 512, 0), (256, 256, 0)], 512, 20, 20, 32)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("geom", WS1_GEOMS)
def test_conv_ws1_1x1(dtype, geom):
    """conv_ws1 (ids 201-210, 241-248: 3-4 row buffers in flight, 253-258: every output channel in
    one block, round 5): weight-stationary
    persistent 1x1 conv over one or two dense sources (channel slices of wider buffers), output
    into a channel slice, every variant built for this cin vs torch fp32; partial last pixel
    tile, cout tails of the block."""
    srcs, cout, H, W, B = geom
    cin = sum(c for c, _, _ in srcs)
    conv, bn = make_conv(cin, cout, 1, 1, seed=cin + cout)
    g = torch.Generator().manual_seed(H * W + cin)
    parts, bufs = [], []
    for c, cb, off in srcs:
        x = torch.randn(B, c, H, W, generator=g)
        buf = torch.zeros(B, H, W, cb, dtype=dtype, device=DEV)
        buf[..., off:off + c] = nhwc(x, dtype)
        parts.append(x)
        bufs.append((buf, off, c, 0))
    want = ref_conv(torch.cat(parts, 1), conv, bn, "silu")
    out = torch.zeros(B, H, W, cout + 16, dtype=dtype, device=DEV)
    ran = 0
    # odd codes (round 6): the same tiles with the 16-byte-store epilogue (v_permlane16_swap pairs of channel
    # fragments): bit-identical to the 8-byte form
    for tid in list(range(201, 211)) + list(range(241, 249)) + [253, 254, 255, 257, 258]:
        y8 = None
        for code in (2 * tid, 2 * tid + 1):
            out.zero_()
            try:
                y = run_conv(bufs, conv, bn, dtype, out=out, out_coff=8, tile=code)
            except NotImplementedError as e:
                assert "input channels" in str(e) or "16-byte epilogue" in str(e), e
                continue
            close(y[..., 8:8 + cout].permute(0, 3, 1, 2), want, dtype)
            assert not y[..., :8].any() and not y[..., 8 + cout:].any()
            y = y.clone()
            yf = run_conv(bufs, conv, bn, dtype, out=out, out_coff=8, tile=code, frag=True)
            assert torch.equal(yf, y), code
            if y8 is None:
                y8 = y
            else:
                assert torch.equal(y, y8), code
            ran += 1
    assert ran >= 1


@pytest.mark.parametrize("cin,H,W,B", [(128, 20, 22, 3), (128, 80, 80, 4), (256, 20, 20, 2)])
def test_conv_ws_two_groups(cin, H, W, B):
    """YXH_CONV_GROUPS2 (a head level's cls_convs[k][1] | reg_convs[k][1] over [cls | reg] as one
    launch): output half g = conv of source half g with weight rows of half g, vs torch fp32."""
    dtype = torch.bfloat16
    conv, bn = make_conv(cin, 2 * cin, 3, 1, seed=cin + H)  # weights [2 cin][cin][3][3]: the two stacked
    x = torch.randn(B, 2 * cin, H, W, generator=torch.Generator().manual_seed(H * W))
    want = ref_conv_groups2(x, conv, bn, cin)
    X = nhwc(x, dtype)
    ran = 0
    for tid in range(161, 191):
        if tid in WS_WITHDRAWN:
            continue
        try:
            y = run_conv([(X, 0, 2 * cin, 0)], conv, bn, dtype, tile=2 * tid, groups2=True)
        except NotImplementedError as e:
            assert "input channels" in str(e), e
            continue
        close(y.permute(0, 3, 1, 2), want, dtype)
        yf = run_conv([(X, 0, 2 * cin, 0)], conv, bn, dtype, tile=2 * tid, groups2=True, frag=True)
        assert torch.equal(yf, y), tid
        ran += 1
    assert ran >= 1
    with pytest.raises(NotImplementedError):  # the other kernel families refuse the two-group form
        run_conv([(X, 0, 2 * cin, 0)], conv, bn, dtype, tile=2 * 141, groups2=True)


def ref_conv_groups2(x, conv, bn, cin):
    y = F.conv2d(x, conv.weight, None, 1, 1, groups=2)
    y = F.batch_norm(y, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)
    return F.silu(y)


def test_conv_ws_residual_and_strided_dst():
    dtype = torch.bfloat16
    conv, bn = make_conv(64, 64, 3, 1, seed=3)
    x = torch.randn(3, 64, 24, 40, generator=torch.Generator().manual_seed(4))
    r = torch.randn(3, 64, 24, 40, generator=torch.Generator().manual_seed(5))
    want = ref_conv(x, conv, bn, "silu") + r.to(dtype).float()
    buf = torch.zeros(3, 24, 40, 128, dtype=dtype, device=DEV)
    for tid in (165, 166):
        buf[..., 64:] = nhwc(r, dtype)
        y = run_conv([(nhwc(x, dtype), 0, 64, 0)], conv, bn, dtype, residual=(buf, 64), out=buf, out_coff=64,
                     tile=2 * tid)
        close(y[..., 64:].permute(0, 3, 1, 2), want, dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cin,h,w,train", [(128, 8, 12, 0), (64, 20, 20, 0), (256, 4, 8, 1), (128, 10, 10, 1),
                                           (128, 6, 6, 2), (64, 12, 8, 1), (256, 10, 10, 0), (256, 6, 6, 2)])
def test_head_pred_fused_level(dtype, cin, h, w, train, monkeypatch):
    """yxh_head_pred: reg/obj/cls 1x1 preds + cat + sigmoid + decode of one level into
    rows [a_off, a_off + h*w) of a [B, A, 85] output, vs torch fp32 on the same (rounded)
    operands; other rows untouched.  Features are channel slices of wider buffers.  train = 2:
    decode_in_inference = False (reg raw, obj / cls sigmoid).  For 64 / 128 / 256 channels the
    per-wave head_pred2 runs, bit-identical to the tile kernel (YXH_HEAD_V1=1) -- 10 x 10 and
    6 x 6 levels put 16-pixel groups across image boundaries."""
    import ctypes as Cc
    n = N()
    B, C, A, a_off, stride = 3, 80, 4 * 7 + h * w + 12, 28, 16.0
    g = torch.Generator().manual_seed(cin + h)
    feats = torch.randn(B, h, w, 2 * cin, generator=g).to(dtype)
    reg, cls = feats[..., :cin], feats[..., cin:]
    w_ro = (torch.randn(5, cin, generator=g) / cin ** 0.5).to(dtype)
    w_cl = (torch.randn(C, cin, generator=g) / cin ** 0.5).to(dtype)
    b_ro, b_cl = torch.randn(5, generator=g) * 0.2, torch.randn(C, generator=g) * 0.2 - 2
    out = torch.full((B, A, 5 + C), -7.0)
    outd = out.to(DEV)
    fd = feats.to(DEV)
    wro, wcl, bro, bcl = w_ro.to(DEV), w_cl.to(DEV), b_ro.to(DEV), b_cl.to(DEV)
    d = n.HeadDesc()
    d.dtype, d.batch, d.h, d.w, d.cin, d.num_classes = n.DTYPE_CODE[dtype], B, h, w, cin, C
    esz = fd.element_size()
    for src, off in ((d.reg, 0), (d.cls, cin)):
        src.ptr = fd.data_ptr() + off * esz
        src.channels, src.cstride, src.bstride, src.h, src.w, src.upsample = cin, 2 * cin, h * w * 2 * cin, h, w, 0
    d.w_reg, d.b_reg, d.w_cls, d.b_cls = wro.data_ptr(), bro.data_ptr(), wcl.data_ptr(), bcl.data_ptr()
    d.out, d.out_bstride, d.a_off, d.stride, d.train = outd.data_ptr(), A * (5 + C), a_off, stride, train
    n.check(n.lib().yxh_head_pred(Cc.byref(d), n.stream_ptr()), "head_pred")
    got = outd.cpu()
    monkeypatch.setenv("YXH_HEAD_V1", "1")
    outd.fill_(-7.0)
    n.check(n.lib().yxh_head_pred(Cc.byref(d), n.stream_ptr()), "head_pred (v1)")
    assert torch.equal(outd.cpu(), got)
    monkeypatch.delenv("YXH_HEAD_V1")
    ro = reg.float().reshape(B, h * w, cin) @ w_ro.float().T + b_ro
    cl = cls.float().reshape(B, h * w, cin) @ w_cl.float().T + b_cl
    gy, gx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    want = torch.cat([ro, cl], -1)
    if train != 2:
        want[..., 0] = (want[..., 0] + gx.reshape(-1)) * stride
        want[..., 1] = (want[..., 1] + gy.reshape(-1)) * stride
        want[..., 2:4] = torch.exp(want[..., 2:4]) * stride
    if train != 1:
        want[..., 4:] = torch.sigmoid(want[..., 4:])
    lvl = got[:, a_off:a_off + h * w]
    torch.testing.assert_close(lvl, want, rtol=1e-4, atol=1e-4)
    assert (got[:, :a_off] == -7.0).all() and (got[:, a_off + h * w:] == -7.0).all()


@pytest.mark.parametrize("idt", [torch.uint8, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("hw", [(128, 128), (100, 68), (36, 260), (4, 8)])
def test_stem_s2_fused_vs_reference(idt, dtype, hw):
    """yxh_stem_s2 (Focus + stem BaseConv + dark2[0] 3x3 s2 in one launch, the stem map only
    in LDS) vs the reference order in fp32: space-to-depth, conv, BN, SiLU, rounded to the
    compute dtype (the map the unfused path stores), conv s2, BN, SiLU.  Partial tiles at the
    right / bottom edges; a wider destination whose extra channels must stay untouched."""
    n = N()
    H, W = hw
    img = torch.randint(0, 256, (2, 3, H, W)).float()
    src = img.permute(0, 2, 3, 1).to(DEV, idt).contiguous()
    c1, bn1 = make_conv(12, 32, 3, 1, seed=5)
    c2, bn2 = make_conv(32, 64, 3, 2, seed=6)
    f = lambda t: t.detach().float().contiguous().to(DEV)  # noqa: E731
    args = [f(c1.weight), f(bn1.weight), f(bn1.bias), f(bn1.running_mean), f(bn1.running_var)]
    w1 = torch.empty(32 * 6 * 32, dtype=dtype, device=DEV)
    b1 = torch.empty(32, dtype=torch.float32, device=DEV)
    n.check(n.lib().yxh_stem_pack(*[a.data_ptr() for a in args], float(bn1.eps), 32, n.DTYPE_CODE[dtype],
                                  w1.data_ptr(), b1.data_ptr(), n.stream_ptr()), "stem pack")
    w2, b2 = pack(c2, bn2, dtype)
    oh, ow = (H // 2 - 1) // 2 + 1, (W // 2 - 1) // 2 + 1
    cs = 80
    dst = torch.full((2, oh, ow, cs), 7.0, dtype=dtype, device=DEV)
    d = n.Stem2Desc()
    d.img, d.layout, d.img_dtype, d.batch, d.h, d.w = src.data_ptr(), n.NHWC, n.DTYPE_CODE[idt], 2, H, W
    d.dtype, d.c1, d.c2, d.act = n.DTYPE_CODE[dtype], 32, 64, n.ACT_SILU
    d.w1, d.b1, d.w2, d.b2 = w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr()
    d.dst, d.dst_cstride, d.dst_bstride = dst.data_ptr(), cs, oh * ow * cs
    n.check(n.lib().yxh_stem_s2(ctypes.byref(d), n.stream_ptr()), "stem_s2")
    torch.cuda.synchronize()
    x = torch.cat([img[..., ::2, ::2], img[..., 1::2, ::2], img[..., ::2, 1::2], img[..., 1::2, 1::2]], 1)
    x = x.to(idt).float()
    s = ref_conv(x, c1, bn1, "silu").to(dtype).float()
    want = ref_conv(s, c2, bn2, "silu")
    got = dst.float().cpu().permute(0, 3, 1, 2)
    assert (got[:, 64:] == 7.0).all()
    err = (got[:, :64] - want).abs().max().item() / want.abs().max().item()
    assert err < TOL[dtype], err


@pytest.mark.parametrize("with4", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("hw", [(128, 128), (100, 68), (36, 260)])
def test_stem_s2_csp_form_vs_reference(dtype, hw, with4):
    """yxh_stem_s2's CSP form (round 4): the stride-2 map stays in LDS; dark2's CspLayer
    conv1 | conv2 (1x1 64 -> 64, network_blocks.py:176-178) over it goes to dst3 and the first
    Bottleneck's conv1 (1x1 32 -> 32, :95-96) over its x_1 half to dst4 -- vs the reference
    order in fp32 with every stored map rounded to the compute dtype.  Destinations wider than
    the written channels keep their other channels."""
    n = N()
    H, W = hw
    img = torch.randint(0, 256, (2, 3, H, W)).float()
    src = img.permute(0, 2, 3, 1).to(DEV, torch.uint8).contiguous()
    c1, bn1 = make_conv(12, 32, 3, 1, seed=5)
    c2, bn2 = make_conv(32, 64, 3, 2, seed=6)
    c3, bn3 = make_conv(64, 64, 1, 1, seed=7)
    c4, bn4 = make_conv(32, 32, 1, 1, seed=8)
    f = lambda t: t.detach().float().contiguous().to(DEV)  # noqa: E731
    args = [f(c1.weight), f(bn1.weight), f(bn1.bias), f(bn1.running_mean), f(bn1.running_var)]
    w1 = torch.empty(32 * 6 * 32, dtype=dtype, device=DEV)
    b1 = torch.empty(32, dtype=torch.float32, device=DEV)
    n.check(n.lib().yxh_stem_pack(*[a.data_ptr() for a in args], float(bn1.eps), 32, n.DTYPE_CODE[dtype],
                                  w1.data_ptr(), b1.data_ptr(), n.stream_ptr()), "stem pack")
    w2, b2 = pack(c2, bn2, dtype)
    w3, b3 = pack(c3, bn3, dtype)
    w4, b4 = pack(c4, bn4, dtype)
    oh, ow = (H // 2 - 1) // 2 + 1, (W // 2 - 1) // 2 + 1
    cs3, cs4 = 72, 40
    dst3 = torch.full((2, oh, ow, cs3), 7.0, dtype=dtype, device=DEV)
    dst4 = torch.full((2, oh, ow, cs4), 7.0, dtype=dtype, device=DEV)
    d = n.Stem2Desc()
    d.img, d.layout, d.img_dtype, d.batch, d.h, d.w = src.data_ptr(), n.NHWC, n.U8, 2, H, W
    d.dtype, d.c1, d.c2, d.act = n.DTYPE_CODE[dtype], 32, 64, n.ACT_SILU
    d.w1, d.b1, d.w2, d.b2 = w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr()
    d.dst = None
    d.w3, d.b3, d.dst3, d.dst3_cstride, d.dst3_bstride = w3.data_ptr(), b3.data_ptr(), dst3.data_ptr(), cs3, oh * ow * cs3
    if with4:
        d.w4, d.b4, d.dst4, d.dst4_cstride, d.dst4_bstride = (w4.data_ptr(), b4.data_ptr(), dst4.data_ptr(), cs4,
                                                              oh * ow * cs4)
    n.check(n.lib().yxh_stem_s2(ctypes.byref(d), n.stream_ptr()), "stem_s2 csp")
    torch.cuda.synchronize()
    x = torch.cat([img[..., ::2, ::2], img[..., 1::2, ::2], img[..., ::2, 1::2], img[..., 1::2, 1::2]], 1)
    s = ref_conv(x, c1, bn1, "silu").to(dtype).float()
    y = ref_conv(s, c2, bn2, "silu").to(dtype).float()
    z = ref_conv(y, c3, bn3, "silu")
    got3 = dst3.float().cpu().permute(0, 3, 1, 2)
    assert (got3[:, 64:] == 7.0).all()
    assert (got3[:, :64] - z).abs().max().item() / z.abs().max().item() < TOL[dtype]
    got4 = dst4.float().cpu().permute(0, 3, 1, 2)
    if with4:
        t = ref_conv(z.to(dtype).float()[:, :32], c4, bn4, "silu")
        assert (got4[:, 32:] == 7.0).all()
        assert (got4[:, :32] - t).abs().max().item() / t.abs().max().item() < TOL[dtype]
    else:
        assert (got4 == 7.0).all()


def test_stem_s2_rejects_what_it_does_not_build():
    n = N()
    d = n.Stem2Desc()
    x = torch.zeros(1, 64, 64, 3, dtype=torch.uint8, device=DEV)
    w = torch.zeros(64 * 9 * 32, dtype=torch.bfloat16, device=DEV)
    b = torch.zeros(64, dtype=torch.float32, device=DEV)
    y = torch.zeros(1, 16, 16, 64, dtype=torch.bfloat16, device=DEV)
    d.img, d.layout, d.img_dtype, d.batch, d.h, d.w = x.data_ptr(), n.NHWC, n.U8, 1, 64, 64
    d.dtype, d.c1, d.c2, d.act = n.BF16, 32, 64, n.ACT_SILU
    d.w1, d.b1, d.w2, d.b2, d.dst, d.dst_cstride, d.dst_bstride = (w.data_ptr(), b.data_ptr(), w.data_ptr(),
                                                                   b.data_ptr(), y.data_ptr(), 64, 16 * 16 * 64)
    for field, bad in (("layout", n.NCHW), ("dtype", n.F32), ("c1", 48), ("h", 66)):
        good = getattr(d, field)
        setattr(d, field, bad)
        assert n.lib().yxh_stem_s2(ctypes.byref(d), n.stream_ptr()) == n.EINVAL
        setattr(d, field, good)
