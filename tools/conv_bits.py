"""Bit fingerprints of the implicit-GEMM engines' outputs at the pipeline's shapes, for A/B builds that
must be bitwise equal (addressing-only changes): run once per library (RDMI_LIB=...) and diff.

    python tools/conv_bits.py > a.txt; RDMI_LIB=old.so python tools/conv_bits.py > b.txt; diff a.txt b.txt
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kbench import conv_cases  # noqa: E402


def fp(t: torch.Tensor) -> str:
    t = t.contiguous()
    v = (t.view(torch.int16) if t.element_size() == 2 else t.view(torch.int32)).flatten().to(torch.int64)
    w = torch.arange(v.numel(), device=v.device, dtype=torch.int64) % 65521 + 1
    return f"{int(v.sum())} {int((v * w).sum() % (1 << 61))}"


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    for lab, B, H, W, ci, co, up in conv_cases():
        B = min(B, 4)
        x = torch.randn(B, H, W, ci, device="cuda", generator=g).half()
        w = K.pack_conv(torch.randn(co, ci, 3, 3, generator=torch.Generator().manual_seed(1)) / math.sqrt(ci * 9),
                        "cuda", ci)
        Ho, Wo = (2 * H, 2 * W) if up else (H, W)
        out = K.conv2d(x, w, co, 3, upsample=up)
        print(f"conv   {lab:32s} {fp(out)}")
        gm, bt = torch.rand(ci, device="cuda", generator=g) + 0.5, torch.randn(ci, device="cuda", generator=g) * 0.1
        if K.conv2d_in_gn_supported(x, w, co, 3, 32, upsample=up):
            mr = K.groupnorm_stats(x, 32, 1e-6)
            res = torch.randn(B, Ho, Wo, co, device="cuda", generator=g).half()
            o2 = K.conv2d(x, w, co, 3, upsample=up, in_gn=(mr, gm, bt, 32, True), residual=res, gn=True)
            o2 = o2[0] if isinstance(o2, tuple) else o2
            print(f"gnconv {lab:32s} {fp(o2)}")
            print(f"gnmom  {lab:32s} {fp(getattr(o2, K._GN_ATTR))}")
        # epilogue operand combinations: bias, per-image row bias (the resnets' time embedding),
        # residual, output moments
        bias = torch.randn(co, device="cuda", generator=g) * 0.1
        rowb = torch.randn(B, co, device="cuda", generator=g) * 0.1
        res = torch.randn(B, Ho, Wo, co, device="cuda", generator=g).half()
        for tag, kw in (("b", dict(bias=bias)), ("br", dict(bias=bias, rowbias=rowb)),
                        ("brRm", dict(bias=bias, rowbias=rowb, residual=res, gn=True)),
                        ("bm", dict(bias=bias, gn=True))):
            o3 = K.conv2d(x, w, co, 3, upsample=up, **kw)
            mom = getattr(o3, K._GN_ATTR, None)
            # GroupNorm statistics from the emitted moments (gn_from_partials) where they exist
            st = f" {fp(K.groupnorm_stats(o3, 32, 1e-6))}" if mom is not None else ""
            print(f"ep{tag:5s} {lab:32s} {fp(o3)}" + (f" {fp(mom)}" if mom is not None else "") + st)
    # implicit-GEMM (non-halo) conv modes: nearest-x2 upsample at 12 -> 24 (Ho % 16 != 0), stride 2
    for lab, B, H, ci, co, kw in [("up 1280 12->24", 4, 12, 1280, 1280, dict(upsample=True)),
                                  ("s2 320 96->48", 4, 96, 320, 320, dict(stride=2)),
                                  ("s2 128 768->384", 1, 768, 128, 128, dict(stride=2))]:
        x = torch.randn(B, H, H, ci, device="cuda", generator=g).half()
        w = K.pack_conv(torch.randn(co, ci, 3, 3, generator=torch.Generator().manual_seed(2)) / math.sqrt(ci * 9),
                        "cuda", ci)
        print(f"conv   {lab:32s} {fp(K.conv2d(x, w, co, 3, **kw))}")
    for M, N, Kd in [(4096, 320, 320), (4096, 2560, 320), (2048, 1280, 1280), (4096, 960, 320), (1024, 10240, 1280),
                     (3000, 5120, 640)]:
        a = torch.randn(M, Kd, device="cuda", generator=g).half()
        wl = (torch.randn(N, Kd, device="cuda", generator=g) / math.sqrt(Kd)).half()
        print(f"gemm   M={M} N={N} K={Kd}{'':12s} {fp(K.gemm(a, wl, Kd))}")
        bias = torch.randn(N, device="cuda", generator=g) * 0.1
        res = torch.randn(M, N, device="cuda", generator=g).half()
        og = K.gemm(a, wl, Kd, bias=bias, residual=res, gn=True)
        mom = getattr(og, K._GN_ATTR, None)
        print(f"gemmep M={M} N={N} K={Kd}{'':12s} {fp(og)}" + (f" {fp(mom)}" if mom is not None else ""))
        if N % 128 == 0:  # GEGLU epilogue (value / gate halves interleaved per 64-column slab)
            print(f"geglu  M={M} N={N} K={Kd}{'':12s} {fp(K.gemm(a, wl, Kd, bias=bias, geglu=True))}")
    # GroupNorm(+SiLU) apply pass at the UNet / VAE shapes that run it unfused
    for B, H, C in [(6, 96, 320), (6, 48, 640), (6, 24, 1280), (5, 12, 2560), (3, 96, 512)]:
        x = torch.randn(B, H, H, C, device="cuda", generator=g).half()
        gm, bt = torch.rand(C, device="cuda", generator=g) + 0.5, torch.randn(C, device="cuda", generator=g) * 0.1
        for silu in (True, False):
            print(f"gnapp  B={B} {H}^2 C={C} silu={int(silu)}{'':10s} {fp(K.groupnorm(x, gm, bt, 32, 1e-5, silu))}")
    # decoder head (GroupNorm+SiLU -> 3x3 conv to one channel): f16 / f32 input, f16 / f32 output,
    # a ragged pixel count per workgroup (HW % 1024 != 0)
    for B, H, W, xdt, odt in [(3, 768, 768, torch.float16, torch.float32), (2, 96, 100, torch.float16, torch.float16),
                              (2, 64, 72, torch.float32, torch.float32)]:
        x = (torch.randn(B, H, W, 128, device="cuda", generator=g) * 2 + 0.3).to(xdt)
        gm, bt = torch.rand(128, device="cuda", generator=g) + 0.5, torch.randn(128, device="cuda", generator=g) * 0.1
        w9 = torch.randn(9, 128, device="cuda", generator=g) / 30
        for silu in (True, False):
            y = K.conv3x3_to1_gn(x, gm, bt, 32, 1e-6, silu, w9, 0.1, out_dtype=odt)
            print(f"head   B={B} {H}x{W} {str(xdt)[6:]}->{str(odt)[6:]} silu={int(silu)}{'':4s} {fp(y)}")
    # flash attention (attn_fwd_d64): a fused-QKV layout at the L0 / L1 shapes and ragged key counts
    for B, S, H in [(2, 27648, 5), (2, 6912, 10), (1, 1000, 5), (1, 31, 2)]:
        qkv = torch.randn(B, S, 3 * H * 64, device="cuda", generator=g).half()
        q, k, v = qkv[..., :H * 64], qkv[..., H * 64:2 * H * 64], qkv[..., 2 * H * 64:]
        print(f"attn   B={B} S={S} H={H}{'':18s} {fp(K.attention(q, k, v, H))}")
    # VAE mid-block attention at d = 512 (attn_fwd_d512): pipeline shape, ragged keys, growing scores
    for B, S, Sk, grow in [(2, 9216, 9216, False), (1, 300, 77, False), (1, 640, 640, True)]:
        q = torch.randn(B, S, 512, device="cuda", generator=g).half()
        gk = torch.linspace(0.2, 4.0, Sk, device="cuda")[None, :, None] if grow else 1.0
        k = (torch.randn(B, Sk, 512, device="cuda", generator=g) * gk).half()
        v = torch.randn(B, Sk, 512, device="cuda", generator=g).half()
        print(f"attn512 B={B} S={S} Sk={Sk} grow={int(grow)}{'':8s} {fp(K.attention_d512(q, k, v, 512 ** -0.5))}")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
