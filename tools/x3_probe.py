"""A/B of the f32 engine's two product forms (gemm_f32.hip): exact f32 products (v_mfma_f32_16x16x4_f32)
vs the bf16 split (RDMI_F32_X3: three v_mfma_f32_16x16x32_bf16).  Per shape: max error relative to
the output's max and mean error relative to its mean |value|, both against f64, and the kernel time.

    python tools/x3_probe.py"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

DEV, F32 = "cuda", torch.float32


def _time(fn, n=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def _err(y, ref):
    d = (y.double() - ref).abs()
    return d.max().item() / ref.abs().max().item(), d.mean().item() / ref.abs().mean().item()


def _packs(fn):
    out = {}
    for x3 in ("0", "1"):
        os.environ["RDMI_F32_X3"] = x3
        out[x3] = fn()
    return out


g = torch.Generator(device=DEV).manual_seed(0)
# UNet / VAE launch shapes of the paper preset at 768² (96² latents, 3-frame snippets)
for M, N, Kd in ((3 * 9216, 960, 320), (3 * 9216, 2560, 320), (3 * 9216, 320, 1280), (3 * 2304, 1920, 640),
                 (3 * 576, 3840, 1280), (1000, 256, 2880)):
    a = torch.randn(M, Kd, device=DEV, generator=g)
    w = torch.randn(N, Kd, device=DEV, generator=g) / math.sqrt(Kd)
    ref = a.double() @ w.double().t()
    ws = _packs(lambda: K.pack_linear(w, DEV, F32))
    line = f"gemm M={M} N={N} K={Kd}:"
    for x3, wp in ws.items():
        y = K.gemm(a, wp, Kd)
        ms = _time(lambda: K.gemm(a, wp, Kd, out=y))
        tf = 2.0 * M * N * Kd / ms / 1e9
        e = _err(y, ref)
        line += f" | {'x3' if x3 == '1' else 'f32'} {ms:.3f} ms {tf:.0f} TF/s max {e[0]:.1e} mean {e[1]:.1e}"
    print(line, flush=True)
    del a, ref

for B, H, W, Cin, Cout, up in ((3, 96, 96, 320, 320, False), (3, 48, 48, 640, 640, False), (3, 24, 24, 1280, 1280, False),
                               (3, 96, 96, 640, 320, False), (1, 384, 384, 256, 256, False),
                               (1, 192, 192, 512, 512, True), (2, 768, 768, 128, 128, False)):
    x = torch.randn(B, Cin, H, W, device=DEV, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, device=DEV, generator=g) / math.sqrt(Cin * 9)
    xin = F.interpolate(x.double(), scale_factor=2.0, mode="nearest") if up else x.double()
    ref = F.conv2d(xin, w.double(), padding=1).permute(0, 2, 3, 1)
    del xin
    xn = K.nchw_to_nhwc(x, Cin, dtype=F32)
    ws = _packs(lambda: K.pack_conv(w.cpu(), DEV, Cin, F32))
    line = f"conv B={B} {H}x{W} {Cin}->{Cout}{' up' if up else ''}:"
    Ho = 2 * H if up else H
    for x3, wp in ws.items():
        y = K.conv2d(xn, wp, Cout, 3, upsample=up)
        ms = _time(lambda: K.conv2d(xn, wp, Cout, 3, upsample=up, out=y), n=5)
        tf = 2.0 * B * Ho * Ho * Cout * 9 * Cin / ms / 1e9
        e = _err(y, ref)
        line += f" | {'x3' if x3 == '1' else 'f32'} {ms:.3f} ms {tf:.0f} TF/s max {e[0]:.1e} mean {e[1]:.1e}"
    print(line, flush=True)
    del x, ref, xn
    torch.cuda.empty_cache()

# cross-frame attention of the 768² snippet (3 frames): L0 S = 27648 (5 heads), L1 6912 (10), L2 1728 (20)
for B, S, H in ((1, 27648, 5), (2, 6912, 10), (4, 1728, 20)):
    C = H * 64
    qkv = torch.randn(B, S, 3 * C, device=DEV, generator=g)
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    rows = torch.randint(0, S, (256,), device=DEV, generator=g)
    qh = q.double()[:, rows].view(B, 256, H, 64).transpose(1, 2)
    ref = F.scaled_dot_product_attention(qh, k.double().view(B, S, H, 64).transpose(1, 2),
                                         v.double().view(B, S, H, 64).transpose(1, 2)).transpose(1, 2).reshape(B, 256, C)
    line = f"attention B={B} S={S} H={H}:"
    for x3 in ("0", "1"):
        os.environ["RDMI_F32_X3"] = x3
        o = K.attention(q, k, v, H)
        ms = _time(lambda: K.attention(q, k, v, H, out=o), n=3)
        tf = 4.0 * B * H * S * S * 64 / ms / 1e9
        err = (o[:, rows].double() - ref).abs().max().item()
        line += f" | {'x3' if x3 == '1' else 'f32'} {ms:.3f} ms {tf:.0f} TF/s max|Δ| {err:.1e}"
    print(line, flush=True)
