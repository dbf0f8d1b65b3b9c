"""Op-level numerics of librdmi on the MI355X, each against a plain PyTorch fp32 reference of the
same op computed from the same f16-rounded inputs (tolerances stated per test: f16 storage of the
output dominates, ~2⁻¹¹ relative)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _k():
    from rollingdepth_amd import kernels as K
    return K


@pytest.fixture(params=["auto", "classic", "pingpong", "halo4", "halo128w8", "halo256"])
def engine(request, monkeypatch):
    """GEMM/conv engine: by size (auto: the two-workgroups-per-CU halo conv for Cout % 128 == 0, the
    two-workgroups-per-CU GEMM for K ≤ 640), the 3-slot classic engine only, the ping-pong engine
    forced for every launch it supports (N % 256 == 0), the 4-phase halo conv with the
    two-workgroups-per-CU GEMM for every dense GEMM, the 8-wave 128-channel halo conv, or the 256-wide
    8-wave ping-pong halo conv for Cout % 256 == 0 (RDMI_GEMM_PP / RDMI_CONV_HALO / RDMI_GEMM_OCC2,
    gemm.hip)."""
    pp = {"auto": "1", "classic": "0", "pingpong": "2", "halo4": "1", "halo128w8": "1", "halo256": "1"}
    halo = {"auto": "3", "classic": "0", "pingpong": "0", "halo4": "1", "halo128w8": "4", "halo256": "2"}
    occ2 = {"auto": "1", "classic": "0", "pingpong": "0", "halo4": "2", "halo128w8": "0",
            "halo256": "1"}  # halo4: every dense GEMM
    monkeypatch.setenv("RDMI_GEMM_PP", pp[request.param])
    monkeypatch.setenv("RDMI_CONV_HALO", halo[request.param])
    monkeypatch.setenv("RDMI_GEMM_OCC2", occ2[request.param])
    return request.param


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (300, 320, 320), (1000, 960, 320), (77, 64, 1024), (5, 1280, 320),
                                   (513, 200, 40), (1000, 256, 320), (700, 128, 1024), (1300, 512, 40),
                                   (33, 384, 96), (600, 640, 2880)])
def test_gemm_bias_residual(M, N, K, engine):
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(0)
    a = torch.randn(M, K, device=DEV, generator=g).half()
    w = torch.randn(N, K, device=DEV, generator=g).half() / math.sqrt(K)
    b = torch.randn(N, device=DEV, generator=g)
    r = torch.randn(M, N, device=DEV, generator=g).half()
    wp = K_.pack_linear(w.float(), DEV)
    y = K_.gemm(a, wp, K, bias=b, residual=r)
    ref = a.float() @ w.float().t() + b + r.float()
    assert _rel(y, ref) < 4e-3


def test_gemm_rowbias_alpha_f32out_batched(engine):
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(1)
    B, M, N, K = 3, 200, 256, 96
    a = torch.randn(B, M, K, device=DEV, generator=g).half()
    w = torch.randn(B, N, K, device=DEV, generator=g).half()
    y = K_.gemm(a, w, K, alpha=0.125, out_f32=True)
    ref = torch.bmm(a.float(), w.float().transpose(1, 2)) * 0.125
    assert _rel(y, ref) < 1e-5 * 50
    rb = torch.randn(4, N, device=DEV, generator=g)
    a2 = torch.randn(400, K, device=DEV, generator=g).half()
    w2 = K_.pack_linear(torch.randn(N, K, device=DEV, generator=g), DEV)
    y2 = K_.gemm(a2, w2, K, rowbias=rb, rows_per_group=100)
    ref2 = a2.float() @ w2[:, :K].float().t() + rb.repeat_interleave(100, 0)
    assert _rel(y2, ref2) < 4e-3


def test_gemm_geglu(engine):
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(2)
    M, C = 333, 320
    a = torch.randn(M, C, device=DEV, generator=g).half()
    w = torch.randn(8 * C, C, device=DEV, generator=g) / math.sqrt(C)
    b = torch.randn(8 * C, device=DEV, generator=g) * 0.1
    wp, bp = K_.geglu_permute(w.cpu(), b.cpu())
    # NaN-filled output: an epilogue that leaves elements unwritten fails here
    y = torch.full((M, 4 * C), float("nan"), dtype=torch.float16, device=DEV)
    K_.gemm(a, K_.pack_linear(wp, DEV), C, out=y, bias=bp.to(DEV), geglu=True)
    h, gate = (a.float() @ w.half().float().t() + b).chunk(2, dim=-1)
    ref = h * F.gelu(gate)
    assert y.shape == (M, 4 * C)
    assert _rel(y, ref) < 4e-3


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,stride,pad,up", [
    (2, 16, 16, 320, 320, 3, 1, 1, False), (1, 24, 20, 8, 320, 3, 1, 1, False), (2, 12, 12, 128, 128, 3, 2, 1, False),
    (1, 9, 7, 64, 64, 3, 1, 1, True), (2, 10, 10, 3, 32, 3, 1, 1, False), (1, 8, 8, 64, 4, 3, 1, 1, False),
    (2, 11, 13, 40, 24, 1, 1, 0, False), (2, 20, 18, 256, 256, 3, 1, 1, False), (1, 17, 15, 128, 128, 3, 1, 1, True),
    (2, 14, 14, 8, 128, 3, 1, 1, False), (1, 13, 11, 320, 640, 3, 2, 1, False), (2, 9, 10, 512, 512, 3, 1, 1, True),
    (1, 12, 12, 40, 256, 3, 1, 1, False), (1, 13, 11, 64, 256, 3, 2, 1, False), (2, 7, 9, 192, 256, 3, 1, 1, True),
    (1, 15, 17, 64, 512, 1, 1, 0, False),
    # halo engine (3x3 s1 p1, Cin % 64 == 0, 16x16 output patches, Cout % 256 == 0)
    (2, 32, 48, 128, 256, 3, 1, 1, False), (1, 16, 16, 64, 512, 3, 1, 1, False), (1, 8, 16, 192, 256, 3, 1, 1, True),
    (3, 16, 32, 320, 256, 3, 1, 1, False), (2, 32, 16, 128, 128, 3, 1, 1, False), (1, 16, 8, 256, 128, 3, 1, 1, True),
    (1, 16, 32, 128, 384, 3, 1, 1, False), (2, 16, 16, 640, 640, 3, 1, 1, False), (1, 8, 8, 192, 384, 3, 1, 1, True),
    (2, 16, 32, 320, 320, 3, 1, 1, False), (1, 16, 16, 960, 320, 3, 1, 1, False), (1, 16, 16, 64, 64, 3, 1, 1, False),
    # 32×32×16 halo conv (conv_halo32_kernel: Cout, Cin % 128 == 0, Ho % 8, Wo % 32)
    (2, 16, 64, 128, 128, 3, 1, 1, False), (1, 24, 32, 256, 128, 3, 1, 1, False), (1, 16, 96, 128, 384, 3, 1, 1, False)])
def test_conv2d(B, H, W, Cin, Cout, k, stride, pad, up, engine, h32):
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(B, Cin, H, W, device=DEV, generator=g).half()
    w = (torch.randn(Cout, Cin, k, k, device=DEV, generator=g) / math.sqrt(Cin * k * k)).half()
    b = torch.randn(Cout, device=DEV, generator=g)
    xin = F.interpolate(x.float(), scale_factor=2.0, mode="nearest") if up else x.float()
    ref = F.conv2d(xin, w.float(), b, stride=stride, padding=pad)
    cp = K_.pad_channels(Cin)
    xn = K_.nchw_to_nhwc(x, cp)
    y = K_.conv2d(xn, K_.pack_conv(w.float().cpu(), DEV, cp), Cout, k, stride=stride, pad=pad, upsample=up, bias=b)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 4e-3


@pytest.mark.parametrize("B,H,W,Cin,Cout,bias", [(2, 24, 20, 256, 128, True), (1, 37, 29, 128, 256, True),
                                                  (3, 16, 16, 128, 128, False), (2, 192, 192, 256, 128, True)])
def test_conv1x1_stream_bitwise(B, H, W, Cin, Cout, bias, monkeypatch):
    """The streaming 1×1 conv (conv1x1.hip, the VAE conv_shortcut shapes) against fp32, and bitwise
    against the GEMM engines (RDMI_CONV1X1=0): the same MFMA per K-step, the same epilogue.  Ragged
    last strip (1 073 pixels) and several strips per wave (73 728 pixels)."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(B, Cin, H, W, device=DEV, generator=g).half()
    w = (torch.randn(Cout, Cin, 1, 1, device=DEV, generator=g) / math.sqrt(Cin)).half()
    b = torch.randn(Cout, device=DEV, generator=g) if bias else None
    ref = F.conv2d(x.float(), w.float(), b)
    xn = K_.nchw_to_nhwc(x, Cin)
    wp = K_.pack_conv(w.float().cpu(), DEV, Cin)
    monkeypatch.setenv("RDMI_CONV1X1", "1")
    y = K_.conv2d(xn, wp, Cout, 1, pad=0, bias=b)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 4e-3
    monkeypatch.setenv("RDMI_CONV1X1", "0")
    y0 = K_.conv2d(xn, wp, Cout, 1, pad=0, bias=b)
    assert torch.equal(y.view(torch.int16), y0.view(torch.int16))


def test_conv2d_vae_downsample_rowbias_residual(engine):
    """Downsample2D with padding=0: F.pad(0,1,0,1) then 3x3 s2 (downsampling.py:141-146)."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(4)
    B, C, H, W = 2, 64, 16, 16
    x = torch.randn(B, C, H, W, device=DEV, generator=g).half()
    w = (torch.randn(C, C, 3, 3, device=DEV, generator=g) / 24).half()
    ref = F.conv2d(F.pad(x.float(), (0, 1, 0, 1)), w.float(), stride=2)
    y = K_.conv2d(K_.nchw_to_nhwc(x, C), K_.pack_conv(w.float().cpu(), DEV), C, 3, stride=2, pad=0, pad_tl=0,
                  out_hw=(H // 2, W // 2))
    assert _rel(y.permute(0, 3, 1, 2), ref) < 4e-3
    rb = torch.randn(B, C, device=DEV, generator=g)
    res = torch.randn(B, H, W, C, device=DEV, generator=g).half()
    y2 = K_.conv2d(K_.nchw_to_nhwc(x, C), K_.pack_conv(w.float().cpu(), DEV), C, 3, rowbias=rb, residual=res)
    ref2 = F.conv2d(x.float(), w.float(), padding=1) + rb[:, :, None, None] + res.float().permute(0, 3, 1, 2)
    assert _rel(y2.permute(0, 3, 1, 2), ref2) < 4e-3
    # per-image time-embedding row bias on the halo engines (UNet conv1: 320 channels, 2 images)
    x3 = torch.randn(2, 32, 16, 320, device=DEV, generator=g).half()
    w3 = torch.randn(320, 320, 3, 3, device=DEV, generator=g) / 40
    rb3 = torch.randn(2, 320, device=DEV, generator=g)
    y3 = K_.conv2d(x3, K_.pack_conv(w3.cpu(), DEV), 320, 3, rowbias=rb3, gn=True)
    ref3 = F.conv2d(x3.float().permute(0, 3, 1, 2), w3.half().float(), padding=1) + rb3[:, :, None, None]
    assert _rel(y3.permute(0, 3, 1, 2), ref3) < 4e-3


@pytest.mark.parametrize("C,G,HW,silu,eps", [(320, 32, 9216, True, 1e-5), (128, 32, 1000, False, 1e-6),
                                            (2560, 32, 64, True, 1e-5), (1920, 32, 100, True, 1e-5),
                                            (40, 8, 77, False, 1e-6)])
def test_groupnorm(C, G, HW, silu, eps):
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(5)
    B = 3
    x = (torch.randn(B, HW, C, device=DEV, generator=g) * 2 + 0.7).half()
    gm = 1 + 0.1 * torch.randn(C, device=DEV, generator=g)
    bt = 0.1 * torch.randn(C, device=DEV, generator=g)
    y = K_.groupnorm(x, gm, bt, G, eps, silu)
    ref = F.group_norm(x.float().permute(0, 2, 1), G, gm, bt, eps).permute(0, 2, 1)
    if silu:
        ref = F.silu(ref)
    assert (y.float() - ref).abs().max().item() < 1e-2


@pytest.mark.parametrize("C,HW,silu,dtype", [(512, 9216, True, torch.float16), (320, 1001, False, torch.float16),
                                              (128, 37, True, torch.float16), (512, 2309, True, torch.float32),
                                              (1280, 5, False, torch.float16)])
def test_groupnorm_apply_row_unroll_bitwise(C, HW, silu, dtype, monkeypatch):
    """gn_apply's four-rows-per-trip form (default) against one row per trip (RDMI_GN_APPLY_U=1): the same
    per-element formula, so bitwise equal — ragged row counts exercise the tail loop."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(12)
    x = (torch.randn(3, HW, C, device=DEV, generator=g) * 2 + 0.3).to(dtype)
    gm = 1 + 0.1 * torch.randn(C, device=DEV, generator=g)
    bt = 0.1 * torch.randn(C, device=DEV, generator=g)
    monkeypatch.setenv("RDMI_GN_APPLY_U", "4")
    y4 = K_.groupnorm(x, gm, bt, 32, 1e-6, silu)
    monkeypatch.setenv("RDMI_GN_APPLY_U", "1")
    y1 = K_.groupnorm(x, gm, bt, 32, 1e-6, silu)
    iv = torch.int16 if dtype == torch.float16 else torch.int32
    assert torch.equal(y4.view(iv), y1.view(iv))


def test_conv1x1_stream_alpha_and_ld(monkeypatch):
    """The streaming 1×1 conv with alpha ≠ 1 and a strided output (y_ld > Cout): bitwise the GEMM engines."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(13)
    B, H, W, Cin, Cout = 2, 33, 31, 256, 128
    x = torch.randn(B, H, W, Cin, device=DEV, generator=g).half()
    w = (torch.randn(Cout, Cin, 1, 1, device=DEV, generator=g) / math.sqrt(Cin)).half()
    b = torch.randn(Cout, device=DEV, generator=g)
    wp = K_.pack_conv(w.float().cpu(), DEV, Cin)
    outs = []
    for mode in ("1", "0"):
        monkeypatch.setenv("RDMI_CONV1X1", mode)
        big = torch.full((B, H, W, Cout + 64), float("nan"), dtype=torch.float16, device=DEV)
        y = big[..., 16:16 + Cout]
        K_.conv2d(x, wp, Cout, 1, pad=0, bias=b, alpha=0.18215, out=y)
        outs.append(big)
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float()) * 0.18215 + b[None, :, None, None]
    assert _rel(outs[0][..., 16:16 + Cout].permute(0, 3, 1, 2), ref) < 4e-3
    assert torch.isnan(outs[0][..., :16]).all() and torch.isnan(outs[0][..., 16 + Cout:]).all()


@pytest.mark.parametrize("B,H,W,Cin,Cout,up", [(2, 16, 16, 64, 128, False), (3, 12, 12, 128, 256, True),
                                                (1, 24, 20, 256, 512, False), (2, 16, 32, 128, 256, False),
                                                (2, 8, 8, 64, 256, True), (2, 16, 32, 128, 128, False),
                                                (1, 16, 64, 256, 128, False)])
def test_groupnorm_moments_from_conv(B, H, W, Cin, Cout, up, engine, h32):
    """Conv epilogue-emitted GroupNorm moments (rdmi.h gn_part) vs the standalone stats pass and an
    fp32 reference; the moments of each image are bitwise independent of the batch they ran in."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(B, H, W, Cin, device=DEV, generator=g).half()
    w = K_.pack_conv(torch.randn(Cout, Cin, 3, 3) / math.sqrt(Cin * 9), DEV)
    res = torch.randn(B, 2 * H if up else H, 2 * W if up else W, Cout, device=DEV, generator=g).half()
    y = K_.conv2d(x, w, Cout, 3, upsample=up, residual=res, gn=True)
    assert getattr(y, K_._GN_ATTR) is not None
    mr_fused = K_.groupnorm_stats(y, 32, 1e-6)
    y_plain = y.clone()  # no moments attached: standalone stats pass
    mr_plain = K_.groupnorm_stats(y_plain, 32, 1e-6)
    HW = y.shape[1] * y.shape[2]
    yf = y.float().view(B, HW, 32, Cout // 32)
    mean = yf.mean(dim=(1, 3)).flatten()
    rstd = (yf.var(dim=(1, 3), unbiased=False).flatten() + 1e-6).rsqrt()
    assert torch.allclose(mr_fused.view(-1, 2)[:, 0], mean, atol=1e-5, rtol=1e-5)
    assert torch.allclose(mr_fused.view(-1, 2)[:, 1], rstd, rtol=1e-4)
    assert torch.allclose(mr_fused, mr_plain, rtol=1e-5, atol=1e-6)
    # batch invariance: image 0 alone
    y0 = K_.conv2d(x[:1], w, Cout, 3, upsample=up, residual=res[:1], gn=True)
    assert torch.equal(y0, y[:1])
    mr0 = K_.groupnorm_stats(y0, 32, 1e-6)
    assert torch.equal(mr0, mr_fused[: mr0.numel()])


@pytest.mark.parametrize("B,H,W,Cin,Cout,res", [(2, 16, 16, 256, 256, False), (1, 32, 48, 512, 512, False),
                                                 (3, 16, 32, 128, 256, True), (1, 48, 16, 64, 512, True),
                                                 (2, 8, 24, 256, 256, False), (2, 16, 16, 128, 128, True),
                                                 (1, 16, 32, 64, 320, False)])
def test_conv2d_up2_phases(B, H, W, Cin, Cout, res, monkeypatch):
    """Upsample2D's nearest ×2 + 3×3 conv as four 2×2 phase convs on the source grid with hi + lo
    merged weights (rdmi_conv_args.w_up2, conv_halo_occ2_kernel MODE 3, RDMI_UP2=1) against the
    9-tap form: the same products, so the f16 outputs differ only where the f32 accumulation order
    moves a value across an f16 rounding boundary — at most 1 ulp, on a small fraction of the
    outputs; also against the fp32 conv, with the epilogue's GroupNorm moments and per-image batch
    invariance.  (2, 8, 24): Ho = 16 is not a phase-tile multiple — the 9-tap form runs (bitwise).
    Cout 128 / 320: 128-channel tiles, the last one ragged."""
    K_ = _k()
    monkeypatch.setenv("RDMI_UP2", "1")
    g = torch.Generator(device=DEV).manual_seed(13)
    x = torch.randn(B, H, W, Cin, device=DEV, generator=g).half()
    w = torch.randn(Cout, Cin, 3, 3) / math.sqrt(Cin * 9)
    wp, wu = K_.pack_conv(w, DEV), K_.pack_conv_up2(w, DEV)
    b = torch.randn(Cout, device=DEV, generator=g) * 0.1
    r = torch.randn(B, 2 * H, 2 * W, Cout, device=DEV, generator=g).half() if res else None
    y = K_.conv2d(x, wp, Cout, 3, upsample=True, bias=b, residual=r, gn=True, w_up2=wu)
    y9 = K_.conv2d(x, wp, Cout, 3, upsample=True, bias=b, residual=r, gn=True)
    monkeypatch.setenv("RDMI_UP2", "0")  # phase weights given but not used
    assert torch.equal(K_.conv2d(x, wp, Cout, 3, upsample=True, bias=b, residual=r, gn=True, w_up2=wu), y9)
    monkeypatch.setenv("RDMI_UP2", "1")
    xin = F.interpolate(x.float().permute(0, 3, 1, 2), scale_factor=2.0, mode="nearest")
    ref = F.conv2d(xin, w.half().float().to(DEV), b, padding=1)
    if res:
        ref = ref + r.float().permute(0, 3, 1, 2)
    err, err9 = _rel(y.permute(0, 3, 1, 2), ref), _rel(y9.permute(0, 3, 1, 2), ref)
    d = (y.float() - y9.float()).abs()
    ulp = torch.exp2(torch.floor(torch.log2(y9.float().abs().clamp_min(2.0 ** -14))) - 10)
    frac = (d > 0).float().mean().item()
    print(f"up2 B={B} {H}x{W} {Cin}->{Cout}: rel {err:.2e} (9-tap {err9:.2e}); vs 9-tap: max {d.max().item():.2e}, "
          f"{frac:.2e} of outputs differ, max {(d / ulp).max().item():.0f} ulp")
    assert err < 4e-3 and abs(err - err9) < 1e-3
    # ≤ 1 ulp of the value, or f32 summation noise (≪ the output's scale) where a result cancels to ~0
    assert (d <= torch.clamp(ulp, min=1e-4 * ref.abs().max().item())).all() and frac < 0.05
    if (2 * H) % 32:
        assert torch.equal(y, y9)
    mr = K_.groupnorm_stats(y, 32, 1e-6)
    assert torch.allclose(mr, K_.groupnorm_stats(y.clone(), 32, 1e-6), rtol=1e-5, atol=1e-6)
    y0 = K_.conv2d(x[:1], wp, Cout, 3, upsample=True, bias=b, residual=None if r is None else r[:1], gn=True,
                   w_up2=wu)
    assert torch.equal(y0, y[:1])
    assert torch.equal(K_.groupnorm_stats(y0, 32, 1e-6), mr[: 2 * 32])


def test_groupnorm_moments_from_gemm(engine):
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(12)
    B, HW, C = 2, 576, 512
    a = torch.randn(B * HW, 256, device=DEV, generator=g).half()
    w = K_.pack_linear(torch.randn(C, 256, device=DEV, generator=g) / 16, DEV)
    r = torch.randn(B * HW, C, device=DEV, generator=g).half()
    y = K_.gemm(a, w, 256, residual=r, gn=True)
    yv = K_.gn_view(y, (B, 24, 24, C))
    gm = torch.ones(C, device=DEV)
    bt = torch.zeros(C, device=DEV)
    out = K_.groupnorm(yv, gm, bt, 32, 1e-6, True)
    ref = F.silu(F.group_norm(yv.float().permute(0, 3, 1, 2), 32, gm, bt, 1e-6)).permute(0, 2, 3, 1)
    assert (out.float() - ref).abs().max().item() < 1e-2


@pytest.mark.parametrize("B,H,W,Cin,Cout,up,silu,G", [
    (2, 32, 48, 128, 256, False, True, 32), (1, 16, 16, 512, 512, False, True, 32), (2, 8, 16, 256, 256, True, True, 32),
    (2, 32, 16, 128, 128, False, True, 32), (1, 16, 8, 256, 128, True, False, 32), (3, 16, 32, 320, 256, False, True, 32),
    (1, 16, 16, 1024, 256, False, True, 16), (2, 16, 16, 64, 128, False, True, 8),
    (2, 16, 16, 128, 384, False, True, 32), (1, 16, 16, 256, 640, True, True, 32), (2, 16, 16, 192, 320, False, True, 32),
    (2, 16, 64, 128, 128, False, True, 32), (1, 16, 32, 256, 128, False, True, 32), (2, 16, 32, 128, 128, False, False, 32),
    # Cin > 256 through the scale / shift table (rdmi.h in_affine) on the two-workgroups-per-CU engine
    (2, 16, 16, 640, 320, False, True, 32), (1, 32, 16, 960, 320, False, True, 32), (2, 16, 16, 512, 128, False, True, 32),
    (1, 16, 16, 1280, 640, False, True, 32), (1, 8, 8, 512, 512, True, True, 32),
    # Cin > 1024 with Cout % 256 == 0 / Cout == 128: under halo256 / halo128w8 these must still reach the
    # engine that reads the in_affine table (the others hold a 1024-entry LDS table)
    (1, 32, 32, 1280, 1280, False, True, 32), (1, 16, 16, 1280, 128, False, True, 32)])
def test_conv2d_fused_input_groupnorm(B, H, W, Cin, Cout, up, silu, G, engine, h32):
    """GroupNorm(+SiLU) applied inside the halo conv's input path (rdmi_conv_args.in_*) against the
    unfused groupnorm → conv2d pair on the same data: the same normalised f16 values feed the same
    MFMA order, so the outputs agree bitwise; plus an fp32 torch reference.  Images get distinct
    statistics (per-image scale/offset) so a wrong image index would show."""
    if engine in ("classic", "pingpong"):
        pytest.skip("input GroupNorm runs on the halo engines only")
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(21)
    scale = torch.arange(1, B + 1, device=DEV).view(B, 1, 1, 1) * 0.7
    x = (torch.randn(B, H, W, Cin, device=DEV, generator=g) * scale + scale).half()
    w = torch.randn(Cout, Cin, 3, 3) / math.sqrt(Cin * 9)
    wp = K_.pack_conv(w, DEV)
    b = torch.randn(Cout, device=DEV, generator=g)
    gm = 1 + 0.2 * torch.randn(Cin, device=DEV, generator=g)
    bt = 0.2 * torch.randn(Cin, device=DEV, generator=g)
    assert K_.conv2d_in_gn_supported(x, wp, Cout, 3, G, upsample=up)
    mr = K_.groupnorm_stats(x, G, 1e-6)
    y = K_.conv2d(x, wp, Cout, 3, upsample=up, bias=b, in_gn=(mr, gm, bt, G, silu))
    h = K_.groupnorm(x, gm, bt, G, 1e-6, silu)
    y_ref = K_.conv2d(h, wp, Cout, 3, upsample=up, bias=b)
    assert torch.equal(y, y_ref)
    hf = F.group_norm(x.float().permute(0, 3, 1, 2), G, gm, bt, 1e-6)
    hf = F.silu(hf) if silu else hf
    hf = F.interpolate(hf, scale_factor=2.0, mode="nearest") if up else hf
    ref = F.conv2d(hf, w.to(DEV), b, padding=1)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 4e-3
    # the helper picks the fused path and matches as well
    y2 = K_.gn_conv2d(x, gm, bt, G, 1e-6, silu, wp, Cout, 3, upsample=up, bias=b)
    assert torch.equal(y2, y_ref)


@pytest.fixture(params=["0", "1"])
def h32(request, monkeypatch):
    """conv_halo32_kernel opt-in (RDMI_CONV_H32) for the conv tests that cover its shapes."""
    monkeypatch.setenv("RDMI_CONV_H32", request.param)
    return request.param


def test_conv2d_h32_epilogue(monkeypatch):
    """The 32×32×16 halo conv's epilogue (bias, per-image row bias, residual, input GroupNorm+SiLU,
    GroupNorm moments of the output) against an fp32 torch reference and against the
    two-workgroups-per-CU 16×16×32 engine (RDMI_CONV_H32=0) — f32 rounding apart (the MFMA's k
    reduction differs), and bitwise batch-invariant."""
    K_ = _k()
    monkeypatch.setenv("RDMI_CONV_H32", "1")
    g = torch.Generator(device=DEV).manual_seed(31)
    B, H, W, Cin, Cout = 3, 16, 64, 256, 128
    x = (torch.randn(B, H, W, Cin, device=DEV, generator=g) * 1.3 + 0.2).half()
    w = torch.randn(Cout, Cin, 3, 3) / math.sqrt(Cin * 9)
    wp = K_.pack_conv(w, DEV)
    b = torch.randn(Cout, device=DEV, generator=g)
    rb = torch.randn(B, Cout, device=DEV, generator=g)
    res = torch.randn(B, H, W, Cout, device=DEV, generator=g).half()
    gm = 1 + 0.2 * torch.randn(Cin, device=DEV, generator=g)
    bt = 0.2 * torch.randn(Cin, device=DEV, generator=g)
    mr = K_.groupnorm_stats(x, 32, 1e-6)

    def run(xx, i0, i1):
        return K_.conv2d(xx, wp, Cout, 3, bias=b, rowbias=rb[i0:i1], residual=res[i0:i1], gn=True,
                         in_gn=(mr[i0 * 64:i1 * 64], gm, bt, 32, True))

    y = run(x, 0, B)
    hf = F.silu(F.group_norm(x.float().permute(0, 3, 1, 2), 32, gm, bt, 1e-6))
    ref = F.conv2d(hf, w.to(DEV), b, padding=1) + rb[:, :, None, None] + res.float().permute(0, 3, 1, 2)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 4e-3
    mr_y = K_.groupnorm_stats(y, 32, 1e-6)
    assert torch.allclose(mr_y, K_.groupnorm_stats(y.clone(), 32, 1e-6), rtol=1e-5, atol=1e-6)
    assert torch.equal(run(x[1:2], 1, 2), y[1:2])
    monkeypatch.setenv("RDMI_CONV_H32", "0")
    y_occ2 = run(x, 0, B)
    assert _rel(y, y_occ2) < 2e-3


def test_conv2d_fused_input_groupnorm_unsupported():
    """Shapes outside the halo engine refuse an input GroupNorm loudly; gn_conv2d falls back to the
    unfused pair."""
    K_ = _k()
    x = torch.randn(1, 12, 12, 64, device=DEV).half()
    wp = K_.pack_conv(torch.randn(64, 64, 3, 3) / 24, DEV)
    gm, bt = torch.ones(64, device=DEV), torch.zeros(64, device=DEV)
    assert not K_.conv2d_in_gn_supported(x, wp, 64, 3, 32)
    mr = K_.groupnorm_stats(x, 32, 1e-6)
    with pytest.raises(RuntimeError):
        K_.conv2d(x, wp, 64, 3, in_gn=(mr, gm, bt, 32, True))
    y = K_.gn_conv2d(x, gm, bt, 32, 1e-6, True, wp, 64, 3)
    assert torch.equal(y, K_.conv2d(K_.groupnorm(x, gm, bt, 32, 1e-6, True), wp, 64, 3))


@pytest.mark.parametrize("B,H,W,C,silu", [(2, 24, 20, 128, True), (1, 7, 9, 64, False), (3, 33, 17, 128, True)])
def test_conv3x3_to1_gn(B, H, W, C, silu):
    """Fused decoder head (convhead.hip) vs GroupNorm(+SiLU) → conv2d(pad 1) to one channel in fp32."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(14)
    x = (torch.randn(B, H, W, C, device=DEV, generator=g) * 1.5 + 0.3).half()
    gm = 1 + 0.1 * torch.randn(C, device=DEV, generator=g)
    bt = 0.1 * torch.randn(C, device=DEV, generator=g)
    w = torch.randn(1, C, 3, 3, device=DEV, generator=g) / math.sqrt(9 * C)
    b = 0.3
    w9 = w[0].permute(1, 2, 0).reshape(9, C).contiguous()
    y = K_.conv3x3_to1_gn(x, gm, bt, 32, 1e-6, silu, w9, b)
    n = F.group_norm(x.float().permute(0, 3, 1, 2), 32, gm, bt, 1e-6)
    if silu:
        n = F.silu(n)
    ref = F.conv2d(n, w, torch.tensor([b], device=DEV), padding=1).permute(0, 2, 3, 1)
    assert y.shape == (B, H, W, 1)
    assert (y.float() - ref).abs().max().item() < 5e-3
    # f32 output (the f16 pipeline's decoded depth, rdmi_conv3x3_to1_gn y_dtype): the same f32 sums,
    # unrounded — the f16 output is exactly its rounding
    y32 = K_.conv3x3_to1_gn(x, gm, bt, 32, 1e-6, silu, w9, b, out_dtype=torch.float32)
    assert y32.dtype == torch.float32 and torch.equal(y32.half(), y)
    assert (y32 - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("C", [320, 640, 1280])
def test_layernorm(C):
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(6)
    x = (torch.randn(3, 577, C, device=DEV, generator=g) * 3).half()
    gm = 1 + 0.1 * torch.randn(C, device=DEV, generator=g)
    bt = 0.1 * torch.randn(C, device=DEV, generator=g)
    y = K_.layernorm(x, gm, bt, 1e-5)
    ref = F.layer_norm(x.float(), (C,), gm, bt, 1e-5)
    assert (y.float() - ref).abs().max().item() < 1e-2


def _sdpa_ref(q, k, v, heads):
    B, Sq, HD = q.shape
    D = HD // heads
    qh = q.float().view(B, Sq, heads, D).transpose(1, 2)
    kh = k.float().view(B, -1, heads, D).transpose(1, 2)
    vh = v.float().view(B, -1, heads, D).transpose(1, 2)
    o = F.scaled_dot_product_attention(qh, kh, vh)
    return o.transpose(1, 2).reshape(B, Sq, HD)


@pytest.fixture(params=["d64", "pipe"])
def attn_engine(request, monkeypatch):
    """Both head-dim-64 flash kernels: attn_fwd_d64 (two waves per SIMD, MFMA block ∥ softmax block;
    the default) and attn_fwd_d64_pipe (RDMI_ATTN_PIPE=1: each wave interleaves its own softmax with
    its MFMAs)."""
    monkeypatch.setenv("RDMI_ATTN_PIPE", "1" if request.param == "pipe" else "0")
    return request.param


@pytest.mark.parametrize("B,S,H", [(1, 192, 2), (2, 768, 5), (1, 432, 20), (3, 100, 1), (1, 3072, 5), (2, 65, 3),
                                   (1, 31, 2), (2, 1000, 1)])
def test_attention_fused_qkv(B, S, H, attn_engine):
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(7)
    C = H * 64
    qkv = torch.randn(B, S, 3 * C, device=DEV, generator=g).half()
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    o = K_.attention(q, k, v, H)
    ref = _sdpa_ref(q, k, v, H)
    assert (o.float() - ref).abs().max().item() < 5e-3


@pytest.mark.parametrize("B,S,H", [(2, 27648, 5), (1, 49152, 5)])
def test_attention_pipeline_sizes_sampled_rows(B, S, H, attn_engine):
    """Level-0 cross-frame attention at the metric config (768²: S = 3·96² = 27 648, H = 5) and at
    1024² (S = 3·128² = 49 152), QKV as the fused projection writes it, against fp32 SDPA over all
    keys for 512 sampled query rows per snippet (the full fp32 reference would need S² scores)."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(21)
    C = H * 64
    qkv = (torch.randn(B, S, 3 * C, device=DEV, generator=g) * 0.7).half()
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    o = K_.attention(q, k, v, H)
    rows = torch.randint(0, S, (512,), device=DEV, generator=g)
    ref = _sdpa_ref(q[:, rows].contiguous(), k, v, H)
    err = (o[:, rows].float() - ref).abs()
    print(f"S={S}: max {err.max().item():.2e} mean {err.mean().item():.2e}")
    assert torch.isfinite(o).all()
    assert err.max().item() < 5e-3 and err.mean().item() < 5e-4


def test_attention_softmax_rescale_branch(attn_engine):
    """A key spike late in the sequence forces the running-max rescale (guide rule 26)."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(8)
    B, S, H = 1, 640, 2
    C = H * 64
    q = torch.randn(B, S, C, device=DEV, generator=g).half()
    k = torch.randn(B, S, C, device=DEV, generator=g).half()
    v = torch.randn(B, S, C, device=DEV, generator=g).half()
    k[0, 500] = (q[0, 3] * 3).half()  # query 3's max jumps at tile 7
    o = K_.attention(q, k, v, H)
    ref = _sdpa_ref(q, k, v, H)
    assert (o.float() - ref).abs().max().item() < 5e-3


@pytest.mark.parametrize("qscale,S", [(6.0, 700), (0.02, 300), (-4.0, 1000)])
def test_attention_large_and_tiny_scores(qscale, S, attn_engine):
    """Score ranges far outside the first tile's max (|scores| up to ~±60 in log2 units: the m̃
    re-set path fires on many tiles) and nearly uniform softmax (scores ≈ 0)."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(12)
    B, H = 1, 3
    C = H * 64
    q = (torch.randn(B, S, C, device=DEV, generator=g) * qscale).half()
    k = torch.randn(B, S, C, device=DEV, generator=g).half()
    v = torch.randn(B, S, C, device=DEV, generator=g).half()
    o = K_.attention(q, k, v, H)
    ref = _sdpa_ref(q, k, v, H)
    # |scores| up to ~60 log2 units: the f16 rounding of Q·scale (2^-12 relative) alone moves a score by
    # ~0.015, i.e. ~1 % of a dominant probability, on outputs of magnitude ~2 (f16 ulp 2^-10)
    assert (o.float() - ref).abs().max().item() < (8e-3 if abs(qscale) > 1 else 5e-3)


def test_attention_growing_max(attn_engine):
    """Key norms grow along the sequence so the row max rises by a few units per tile: the m̃
    re-set (and O/l rescale) fires repeatedly at moderate jumps, never at the first tile only."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(13)
    B, S, H = 1, 1536, 2
    C = H * 64
    q = torch.randn(B, S, C, device=DEV, generator=g).half()
    ramp = torch.linspace(0.2, 3.0, S, device=DEV)[None, :, None]
    k = (torch.randn(B, S, C, device=DEV, generator=g) * ramp).half()
    v = torch.randn(B, S, C, device=DEV, generator=g).half()
    o = K_.attention(q, k, v, H)
    ref = _sdpa_ref(q, k, v, H)
    assert (o.float() - ref).abs().max().item() < 5e-3


def test_attention_smallkv():
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(9)
    B, S, H, L = 2, 999, 5, 2
    C = H * 64
    q = torch.randn(B, S, C, device=DEV, generator=g).half()
    k = torch.randn(1, L, C, device=DEV, generator=g).half()
    v = torch.randn(1, L, C, device=DEV, generator=g).half()
    o = K_.attention_smallkv(q, k, v, H)
    ref = _sdpa_ref(q, k.expand(B, -1, -1), v.expand(B, -1, -1), H)
    assert (o.float() - ref).abs().max().item() < 3e-3


@pytest.mark.parametrize("M,C,H", [(999, 320, 5), (517, 640, 10), (64, 128, 2)])
def test_cross_attn_pair(M, C, H, monkeypatch):
    """norm2 → attn2 (two-token context) → +residual as one row pass (rdmi_cross_attn_pair, exact
    fold of the two-key softmax) against the unfolded fp32 computation of the reference block; the
    head-unrolled kernel (H = 5 / 10) bitwise the per-head loop (RDMI_PAIR_HC=0)."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(31)
    x = torch.randn(M, C, device=DEV, generator=g).half()
    lg = 1 + 0.1 * torch.randn(C, device=DEV, generator=g)
    lb = 0.1 * torch.randn(C, device=DEV, generator=g)
    wq, wk, wv, wo = (torch.randn(C, C, device=DEV, generator=g) / math.sqrt(C) for _ in range(4))
    wq, wo = wq.half().float(), wo.half().float()
    bo = 0.1 * torch.randn(C, device=DEV, generator=g)
    ctx = torch.randn(2, C, device=DEV, generator=g).half()
    k2 = (ctx.float() @ wk.half().float().t()).half()
    v2 = (ctx.float() @ wv.half().float().t()).half()
    fold = K_.fold_attn2_pair(wq, wo, bo, k2, v2, H)
    y = K_.cross_attn_pair(x, lg, lb, 1e-5, *fold)
    monkeypatch.setenv("RDMI_PAIR_HC", "0")
    assert torch.equal(K_.cross_attn_pair(x, lg, lb, 1e-5, *fold), y)
    monkeypatch.delenv("RDMI_PAIR_HC")
    n2 = F.layer_norm(x.float(), (C,), lg, lb, 1e-5)
    q = n2 @ wq.t()
    o = _sdpa_ref(q.half()[None], k2[None], v2[None], H)[0]
    ref = x.float() + o.float() @ wo.t() + bo
    assert _rel(y, ref) < 4e-3


@pytest.mark.parametrize("cols,pad", [(9216, 0), (5000, 8), (20000, 0), (1024, 0), (234, 6), (36, 4)])
def test_softmax_rows(cols, pad):
    """Row softmax (single-pass register kernel for cols % 4 == 0 and ≤ 16384, three-pass
    otherwise) against torch.softmax; the padding columns are written as zeros."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(13)
    s = torch.randn(37, cols, device=DEV, generator=g) * 8
    out = torch.full((37, cols + pad), 7.0, device=DEV, dtype=torch.float16)
    p = K_.softmax_rows(s, 0.3, out=out)
    ref = torch.softmax(s * 0.3, dim=-1)
    assert (p[:, :cols].float() - ref).abs().max().item() < 2e-3
    assert torch.all(p[:, cols:] == 0)


@pytest.mark.parametrize("S", [256, 234, 97])
def test_vae_style_attention_via_gemm(S):
    """GEMM(f32 scores) → softmax_rows → GEMM with Vᵀ, the d=C single-head path (attention_1head);
    key counts that are not multiples of 8 run the PV GEMM on zero-padded K."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(10)
    B, D = 2, 128
    q = torch.randn(B, S, D, device=DEV, generator=g).half()
    k = torch.randn(B, S, D, device=DEV, generator=g).half()
    v = torch.randn(B, S, D, device=DEV, generator=g).half()
    o = K_.attention_1head(q, k, v, 1.0 / math.sqrt(D))
    ref = F.scaled_dot_product_attention(q.float()[:, None], k.float()[:, None], v.float()[:, None])[:, 0]
    assert (o.float() - ref).abs().max().item() < 5e-3
    if S % 8 == 0:
        s = K_.gemm(q, k, D, out_f32=True)
        p = K_.softmax_rows(s, 1.0 / math.sqrt(D))
        assert torch.equal(K_.gemm(p, K_.transpose(v), S), o)


@pytest.fixture(params=["w4", "w8"])
def d512_kernel(request, monkeypatch):
    """w4: the 32-query pass (fixed running max) + fix-up; w8: the 16-query kernel alone."""
    monkeypatch.setenv("RDMI_D512_W4", "1" if request.param == "w4" else "0")
    return request.param


@pytest.mark.parametrize("B,Sq,Sk", [(2, 576, 576), (1, 2304, 2304), (2, 100, 100), (1, 300, 77), (1, 9216, 9216)])
def test_attention_d512(B, Sq, Sk, d512_kernel):
    """Flash attention at head dim 512 (the VAE mid-block, rdmi_attention_d512) against an f64
    softmax reference on the same f16 inputs (rows sampled at the full 768² size), and against the
    GEMM → softmax → GEMM path; keys that are not a multiple of 32 are masked."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(41)
    D = 512
    qkv = torch.randn(B, max(Sq, Sk), 3 * D, device=DEV, generator=g).half()
    q, k, v = qkv[:, :Sq, :D], qkv[:, :Sk, D:2 * D], qkv[:, :Sk, 2 * D:]
    sc = 1.0 / math.sqrt(D)
    o = K_.attention_d512(q, k, v, sc)
    rows = torch.arange(Sq, device=DEV) if Sq <= 2304 else torch.randint(0, Sq, (256,), device=DEV, generator=g)
    s = torch.einsum("bqd,bkd->bqk", q[:, rows].double(), k.double()) * sc
    ref = torch.softmax(s, -1) @ v.double()
    err = (o[:, rows].double() - ref).abs().max().item()
    print(f"d512 B={B} Sq={Sq} Sk={Sk}: max |d| {err:.2e} (|ref| {ref.abs().max().item():.2f})")
    assert err < 4e-3
    if Sq <= 2304:
        import os
        os.environ["RDMI_VAE_FLASH"] = "0"
        try:
            o_gemm = K_.attention_1head(q.contiguous(), k.contiguous(), v.contiguous(), sc)
        finally:
            os.environ.pop("RDMI_VAE_FLASH")
        assert (o.float() - o_gemm.float()).abs().max().item() < 4e-3


@pytest.mark.parametrize("mixed", [False, True])
def test_attention_d512_rescale(d512_kernel, mixed):
    """Scores that grow along the keys (the running max re-set several times, O / l rescaled; for
    the 32-query pass: its blocks flagged and recomputed by the fix-up) and large scores (P at the
    edge of the f16 range before a rescale).  mixed: only the odd 128-query blocks grow past the
    f16 range, so flagged and unflagged blocks share one launch."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(42)
    B, S, D = 1, 640, 512
    qs = torch.full((S, 1), 1.5, device=DEV)
    if mixed:
        qs[(torch.arange(S, device=DEV) // 128) % 2 == 0] = 0.05
    q = (torch.randn(B, S, D, device=DEV, generator=g) * qs).half()
    growth = torch.linspace(0.2, 4.0, S, device=DEV)[None, :, None]
    k = (torch.randn(B, S, D, device=DEV, generator=g) * growth).half()
    v = torch.randn(B, S, D, device=DEV, generator=g).half()
    sc = 1.0 / math.sqrt(D)
    o = K_.attention_d512(q, k, v, sc)
    s = torch.einsum("bqd,bkd->bqk", q.double(), k.double()) * sc
    ref = torch.softmax(s, -1) @ v.double()
    err = (o.double() - ref).abs().max().item()
    print(f"d512 rescale: max |d| {err:.2e}, score range {s.min().item():.1f}..{s.max().item():.1f}")
    assert torch.isfinite(o).all()
    assert err < 8e-3


def test_layout_and_elementwise():
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(2, 3, 5, 7, device=DEV, generator=g)
    n = K_.nchw_to_nhwc(x, 8, scale=2.0)
    assert torch.allclose(n[..., :3].float(), (x * 2).permute(0, 2, 3, 1), atol=1e-2)
    assert n[..., 3:].abs().max().item() == 0
    back = K_.nhwc_to_nchw_f32(n, 3, scale=0.5, shift=1.0)
    assert torch.allclose(back, x + 1.0, atol=1e-2)
    a = torch.randn(10, 16, device=DEV, generator=g).half()
    b = torch.randn(10, 24, device=DEV, generator=g).half()
    assert torch.equal(K_.concat_channels(a, b), torch.cat([a, b], -1))
    t = torch.randn(3, 70, 130, device=DEV, generator=g).half()
    assert torch.equal(K_.transpose(t), t.transpose(1, 2).contiguous())
    rgb = torch.randn(6, 4, 4, 8, device=DEV, generator=g).half()
    dep = torch.randn(1, 4, 4, 8, device=DEV, generator=g).half()
    idx = torch.tensor([0, 2, 4, 1, 3, 5], dtype=torch.int32, device=DEV)
    u = K_.gather_unet_input(rgb, dep, idx, True)
    assert torch.equal(u[..., :4], rgb[idx.long(), ..., :4])
    assert torch.equal(u[..., 4:], dep[..., :4].expand(6, -1, -1, -1))
    e = torch.randn(6, 4, 4, 4, device=DEV, generator=g).half()
    y = K_.ddim_combine(u[..., 4:], e, 0.3, -0.7, 2.0, 4, 8)
    ref = (0.3 * u[..., 4:].float() - 0.7 * e.float()) * 2.0
    assert torch.allclose(y[..., :4].float(), ref, atol=1e-2) and y[..., 4:].abs().max().item() == 0
    z = torch.randn(100003, device=DEV, generator=g)
    mm = K_.minmax(z)
    assert mm[0].item() == z.min().item() and mm[1].item() == z.max().item()
    zr = z.clone()
    K_.renormalize_(zr, mm)
    ref = z - z.min()
    ref = ref / ref.max()
    ref = ref * 2.0 - 1.0
    assert torch.equal(zr, ref)


@pytest.mark.parametrize("H,W,Ho,Wo", [(7, 7, 13, 14), (14, 27, 27, 54), (12, 12, 24, 24), (5, 9, 11, 10)])
def test_resize_nearest(H, W, Ho, Wo):
    """rdmi_resize_nearest == F.interpolate(size=..., mode="nearest") bitwise (Upsample2D output_size)."""
    K_ = _k()
    x = torch.randn(2, H, W, 16, device=DEV).half()
    y = K_.resize_nearest(x, (Ho, Wo))
    ref = F.interpolate(x.permute(0, 3, 1, 2).float(), size=(Ho, Wo), mode="nearest").half().permute(0, 2, 3, 1)
    assert torch.equal(y, ref)



@pytest.mark.parametrize("B,H,W,Cin,Cout,up,gn", [(2, 32, 32, 128, 128, False, True), (1, 16, 32, 256, 256, False, True),
                                                  (1, 16, 16, 512, 128, False, False), (1, 8, 16, 256, 128, True, False),
                                                  (2, 16, 16, 64, 128, False, True)])
def test_conv_halo_prefetch_bitwise(B, H, W, Cin, Cout, up, gn, monkeypatch):
    """RDMI_HALO_PREF (the occ2 halo conv's L2 prefetch of the next channel block's halo) only adds loads
    into a scratch LDS area: outputs bitwise equal with and without it (one channel block included)."""
    K_ = _k()
    g = torch.Generator(device=DEV).manual_seed(33)
    x = torch.randn(B, H, W, Cin, device=DEV, generator=g).half()
    wp = K_.pack_conv(torch.randn(Cout, Cin, 3, 3) / math.sqrt(Cin * 9), DEV)
    bias = torch.randn(Cout, device=DEV, generator=g)
    ig = None
    if gn:
        gm = 1 + 0.2 * torch.randn(Cin, device=DEV, generator=g)
        bt = 0.2 * torch.randn(Cin, device=DEV, generator=g)
        ig = (K_.groupnorm_stats(x, 32, 1e-6), gm, bt, 32, True)
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("RDMI_HALO_PREF", v)
        outs.append(K_.conv2d(x, wp, Cout, 3, upsample=up, bias=bias, in_gn=ig))
    assert torch.equal(outs[0], outs[1])
