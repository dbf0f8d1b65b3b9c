"""Kernel micro-benchmarks at the metric configuration's shapes (768², snippet batch 8, VAE batch 8).

    python tools/kbench.py [--only conv,gemm,attn,gn] [--iters 20]

Prints achieved TFLOP/s (MFMA kernels) or GB/s (streaming kernels) per shape, timed with HIP
events on the launch stream, random data (zeros inflate clocks, guide §5.4 rule 25)."""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def conv_cases():
    # (label, B, H, W, Cin, Cout, up)
    return [
        ("unet L0 320->320 96^2 x24", 24, 96, 96, 320, 320, False),
        ("unet L1 640->640 48^2 x24", 24, 48, 48, 640, 640, False),
        ("unet L2 1280->1280 24^2 x24", 24, 24, 24, 1280, 1280, False),
        ("unet L3 1280->1280 12^2 x24", 24, 12, 12, 1280, 1280, False),
        # the pipeline's UNet launch shape: a 25-snippet batch = 75 frames (pipeline._snippet_batches)
        ("unet L2 1280->1280 24^2 x75", 75, 24, 24, 1280, 1280, False),
        ("unet L3 1280->1280 12^2 x75", 75, 12, 12, 1280, 1280, False),
        ("unet up 960->320 96^2 x24", 24, 96, 96, 960, 320, False),
        ("vae 512->512 96^2 x8", 8, 96, 96, 512, 512, False),
        ("vae 512->512 192^2 x8", 8, 192, 192, 512, 512, False),
        ("vae 256->256 384^2 x8", 8, 384, 384, 256, 256, False),
        ("vae 128->128 768^2 x8", 8, 768, 768, 128, 128, False),
        ("vae up 256 192->384 x8", 8, 192, 192, 256, 256, True),
    ]


def bench_conv(iters):
    for lab, B, H, W, ci, co, up in conv_cases():
        x = torch.randn(B, H, W, ci, device="cuda").half()
        w = K.pack_conv(torch.randn(co, ci, 3, 3) / math.sqrt(ci * 9), "cuda", ci)
        Ho, Wo = (2 * H, 2 * W) if up else (H, W)
        out = torch.empty(B, Ho, Wo, co, device="cuda", dtype=torch.float16)
        ms = timeit(lambda: K.conv2d(x, w, co, 3, upsample=up, out=out), iters)
        fl = 2.0 * B * Ho * Wo * co * ci * 9
        print(f"conv  {lab:32s} {ms * 1e3:9.1f} us  {fl / ms / 1e9:8.1f} TFLOP/s")


def bench_conv1(iters):
    """1×1 convs (ResnetBlock2D shortcuts) at the pipeline's launch shapes: dense GEMMs over pixels."""
    for lab, B, H, ci, co in [("vae sc 256->128 768^2 x5", 5, 768, 256, 128), ("vae sc 512->256 384^2 x9", 9, 384, 512, 256),
                              ("unet sc 640->320 96^2 x75", 75, 96, 640, 320), ("unet sc 960->320 96^2 x75", 75, 96, 960, 320),
                              ("unet sc 1280->640 48^2 x75", 75, 48, 1280, 640)]:
        x = torch.randn(B, H, H, ci, device="cuda").half()
        w = K.pack_conv(torch.randn(co, ci, 1, 1) / math.sqrt(ci), "cuda", ci)
        out = torch.empty(B, H, H, co, device="cuda", dtype=torch.float16)
        ms = timeit(lambda: K.conv2d(x, w, co, 1, pad=0, out=out), iters)
        fl = 2.0 * B * H * H * co * ci
        by = 2.0 * B * H * H * (ci + co)
        print(f"conv1 {lab:32s} {ms * 1e3:9.1f} us  {fl / ms / 1e9:8.1f} TFLOP/s {by / ms / 1e6:7.0f} GB/s")


def bench_gnpart(iters):
    """GroupNorm statistics from a producer's emitted moments (gn_from_partials) at the VAE / UNet shapes."""
    for lab, B, H, C in [("vae 128 768^2 x9", 9, 768, 128), ("vae 256 384^2 x18", 18, 384, 256),
                         ("vae 512 192^2 x36", 36, 192, 512), ("unet 640 48^2 x75", 75, 48, 640)]:
        x = torch.randn(B, H, H, C, device="cuda").half()
        w = K.pack_conv(torch.randn(C, C, 1, 1) / math.sqrt(C), "cuda", C)
        o = K.conv2d(x, w, C, 1, pad=0, gn=True)
        if getattr(o, K._GN_ATTR, None) is None:
            print(f"gnpart {lab:30s} (no moments)")
            continue
        ms = timeit(lambda: K.groupnorm_stats(o, 32, 1e-6), iters)
        print(f"gnpart {lab:30s} {ms * 1e3:9.1f} us")


def bench_head(iters):
    """Decoder head: GroupNorm+SiLU+3x3 conv to one channel (rdmi_conv3x3_to1_gn)."""
    for B, H, C in [(16, 768, 128), (8, 768, 128)]:
        x = torch.randn(B, H, H, C, device="cuda").half()
        g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        w9 = torch.randn(9, C, device="cuda") / 30
        out = torch.empty(B, H, H, 1, device="cuda", dtype=torch.float16)
        ms = timeit(lambda: K.conv3x3_to1_gn(x, g, b, 32, 1e-6, True, w9, 0.1, out=out), iters)
        print(f"head  B={B} {H}^2 C={C}                {ms * 1e3:9.1f} us  {x.numel() * 2 / ms / 1e6:8.0f} GB/s (input)")


def bench_gnconv(iters):
    """GroupNorm+SiLU → conv: apply pass + conv vs the norm fused into the halo conv's input."""
    from rollingdepth_amd._native import lib
    cases = conv_cases()[5:] + [("unet L0 320->320 96^2 x48", 48, 96, 96, 320, 320, False),
                                ("unet L1 640->640 48^2 x48", 48, 48, 48, 640, 640, False),
                                ("unet L0 640->320 96^2 x48", 48, 96, 96, 640, 320, False),
                                ("unet L1 320->640 48^2 x48", 48, 48, 48, 320, 640, False)]
    for lab, B, H, W, ci, co, up in cases:
        x = torch.randn(B, H, W, ci, device="cuda").half()
        w = K.pack_conv(torch.randn(co, ci, 3, 3) / math.sqrt(ci * 9), "cuda", ci)
        g, b = torch.ones(ci, device="cuda"), torch.zeros(ci, device="cuda")
        Ho, Wo = (2 * H, 2 * W) if up else (H, W)
        out = torch.empty(B, Ho, Wo, co, device="cuda", dtype=torch.float16)
        h = torch.empty_like(x)
        mr = K.groupnorm_stats(x, 32, 1e-6)
        if not K.conv2d_in_gn_supported(x, w, co, 3, 32, upsample=up):
            continue

        def unfused():
            lib.rdmi_groupnorm_apply(x.data_ptr(), h.data_ptr(), 0, B, H * W, ci, 32, mr.data_ptr(), g.data_ptr(),
                                     b.data_ptr(), 1, K._stream())
            K.conv2d(h, w, co, 3, upsample=up, out=out)

        ms_u = timeit(unfused, iters)
        ms_f = timeit(lambda: K.conv2d(x, w, co, 3, upsample=up, out=out, in_gn=(mr, g, b, 32, True)), iters)
        fl = 2.0 * B * Ho * Wo * co * ci * 9
        res = torch.randn(B, Ho, Wo, co, device="cuda").half()
        # as ResnetBlock2D.conv2 runs it: + residual, GroupNorm moments of the output for the next norm
        ms_r = timeit(lambda: K.conv2d(x, w, co, 3, upsample=up, out=out, in_gn=(mr, g, b, 32, True), residual=res,
                                       gn=True), iters)
        ms_r1 = timeit(lambda: K.conv2d(x, w, co, 3, upsample=up, out=out, in_gn=(mr, g, b, 32, True), residual=res),
                       iters)
        ms_m1 = timeit(lambda: K.conv2d(x, w, co, 3, upsample=up, out=out, in_gn=(mr, g, b, 32, True), gn=True), iters)
        print(f"gnconv {lab:31s} apply+conv {ms_u * 1e3:9.1f} us | fused {ms_f * 1e3:9.1f} us "
              f"{fl / ms_f / 1e9:8.1f} TFLOP/s | +res+moments {ms_r * 1e3:9.1f} us {fl / ms_r / 1e9:8.1f} TFLOP/s"
              f" | +res {ms_r1 * 1e3:9.1f} | +moments {ms_m1 * 1e3:9.1f}")


def bench_cinsweep(iters):
    """Fixed tile count, growing K: time = per-tile fixed cost + per-K-tile cost (halo engine)."""
    for co in (128, 256):
        for ci in (64, 128, 256, 512):
            B, H = 4, 768 if co == 128 else 384
            x = torch.randn(B, H, H, ci, device="cuda").half()
            w = K.pack_conv(torch.randn(co, ci, 3, 3) / math.sqrt(ci * 9), "cuda", ci)
            out = torch.empty(B, H, H, co, device="cuda", dtype=torch.float16)
            ms = timeit(lambda: K.conv2d(x, w, co, 3, out=out), iters)
            fl = 2.0 * B * H * H * co * ci * 9
            tiles = B * H * H // 256 * (co // 128 if co == 128 else co // 256)
            print(f"sweep {H}^2 x{B} {ci:4d}->{co:4d} {ms * 1e3:9.1f} us {fl / ms / 1e9:8.1f} TFLOP/s "
                  f"{ms * 1e3 / (tiles / 256):7.2f} us per tile-round ({ci // 64 * 9} K-tiles)")


def bench_gemm(iters):
    for lab, M, N, Kd, geglu in [("L0 qkv 221k x 960 x 320", 221184, 960, 320, False),
                                 ("L0 ff1 geglu 221k x 2560 x 320", 221184, 2560, 320, True),
                                 ("L0 proj 221k x 320 x 320 +res", 221184, 320, 320, False),
                                 ("L0 proj 691k x 320 x 320 +res (x75)", 691200, 320, 320, False),
                                 ("L0 qkv 691k x 960 x 320 (x75)", 691200, 960, 320, False),
                                 ("L0 ff1 geglu 691k x 2560 x 320 (x75)", 691200, 2560, 320, True),
                                 ("L0 ff2 691k x 320 x 1280 +res (x75)", 691200, 320, 1280, False),
                                 ("L1 proj 173k x 640 x 640 +res (x75)", 172800, 640, 640, False),
                                 ("L1 ff1 geglu 173k x 5120 x 640 (x75)", 172800, 5120, 640, True),
                                 ("L2 proj 43k x 1280 x 1280 +res (x75)", 43200, 1280, 1280, False),
                                 ("L1 proj 55k x 640 x 640 +res", 55296, 640, 640, False),
                                 ("L1 ff1 geglu 55k x 5120 x 640", 55296, 5120, 640, True),
                                 ("L0 ff2 221k x 320 x 1280", 221184, 320, 1280, False),
                                 ("L2 ff1 geglu 13.8k x 10240 x 1280", 13824, 10240, 1280, True),
                                 ("L2 ff2 13.8k x 1280 x 5120", 13824, 1280, 5120, False),
                                 ("L1 qkv 55k x 1920 x 640", 55296, 1920, 640, False),
                                 ("L2 qkv 13.8k x 3840 x 1280", 13824, 3840, 1280, False),
                                 ("vae qkv 73.7k x 1536 x 512", 73728, 1536, 512, False),
                                 ("vae scores b8 9216 x 9216 x 512 f32", 9216, 9216, 512, False),
                                 ("vae pv b8 9216 x 512 x 9216", 9216, 512, 9216, False)]:
        if " b8 " in lab:  # batched, operands as the VAE attention has them
            a = torch.randn(8, M, Kd, device="cuda").half()
            w = torch.randn(8, N, Kd, device="cuda").half()
            f32 = "f32" in lab
            ms = timeit(lambda: K.gemm(a, w, Kd, out_f32=f32), iters)
            fl = 2.0 * 8 * M * N * Kd
            print(f"gemm  {lab:32s} {ms * 1e3:9.1f} us  {fl / ms / 1e9:8.1f} TFLOP/s")
            continue
        a = torch.randn(M, Kd, device="cuda").half()
        w = K.pack_linear(torch.randn(N, Kd) / math.sqrt(Kd), "cuda")
        r = torch.randn(M, N, device="cuda").half() if "+res" in lab else None
        ms = timeit(lambda: K.gemm(a, w, Kd, geglu=geglu, residual=r), iters)
        fl = 2.0 * M * N * Kd
        print(f"gemm  {lab:32s} {ms * 1e3:9.1f} us  {fl / ms / 1e9:8.1f} TFLOP/s")


def bench_square(iters):
    """Dense square GEMMs: the engine against a plain-GEMM yardstick (guide §5 256² template)."""
    for n in (4096, 8192):
        a = (torch.rand(n, n, device="cuda") * 2 - 1).half()
        w = (torch.rand(n, n, device="cuda") * 2 - 1).half()
        out = torch.empty(n, n, device="cuda", dtype=torch.float16)
        ms = timeit(lambda: K.gemm(a, w, n, out=out), iters)
        print(f"gemm  square {n}^3{'':22s} {ms * 1e3:9.1f} us  {2.0 * n ** 3 / ms / 1e9:8.1f} TFLOP/s")
        ms = timeit(lambda: torch.matmul(a, w.t(), out=out), iters)
        print(f"torch square {n}^3{'':22s} {ms * 1e3:9.1f} us  {2.0 * n ** 3 / ms / 1e9:8.1f} TFLOP/s")


def bench_shapes(iters):
    """Dense GEMM scaling probe over M, N, K (fixed-overhead vs K-loop rate)."""
    print("CUs:", torch.cuda.get_device_properties(0).multi_processor_count)
    for m, n, k in [(4096, 4096, 4096), (4096, 4096, 8192), (4096, 4096, 16384), (8192, 4096, 4096),
                    (16384, 4096, 4096), (8192, 8192, 4096), (8192, 8192, 8192)]:
        a = (torch.rand(m, k, device="cuda") * 2 - 1).half()
        w = (torch.rand(n, k, device="cuda") * 2 - 1).half()
        out = torch.empty(m, n, device="cuda", dtype=torch.float16)
        ms = timeit(lambda: K.gemm(a, w, k, out=out), iters)
        print(f"gemm  {m}x{n}x{k}{'':18s} {ms * 1e3:9.1f} us  {2.0 * m * n * k / ms / 1e9:8.1f} TFLOP/s")


def bench_host(iters):
    """Host-side cost of one wrapper call (tiny problem: the GPU finishes first)."""
    import time
    a = torch.randn(16, 64, device="cuda").half()
    w = K.pack_linear(torch.randn(128, 64), "cuda")
    x = torch.randn(1, 8, 8, 64, device="cuda").half()
    wc = K.pack_conv(torch.randn(64, 64, 3, 3), "cuda")
    for lab, fn in (("gemm", lambda: K.gemm(a, w, 64)), ("conv2d", lambda: K.conv2d(x, wc, 64, 3)),
                    ("empty launch", lambda: torch.empty(1, device="cuda").zero_())):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            fn()
        dt = (time.perf_counter() - t0) / 200
        torch.cuda.synchronize()
        print(f"host  {lab:32s} {dt * 1e6:9.1f} us per call")


def bench_aligner(iters):
    """DepthAligner.run at the fast preset (N=100, dilations [1, 25], 768², 2000 iterations)."""
    from rollingdepth_amd import DepthAligner
    g = torch.Generator(device="cuda").manual_seed(0)
    sn = [(torch.rand(n, 3, 1, 768, 768, device="cuda", generator=g) * 0.8 + 0.1).half() for n in (98, 50)]
    al = DepthAligner("cuda")
    al.run(sn, [1, 25])
    torch.cuda.synchronize()
    ms = timeit(lambda: al.run(sn, [1, 25]), max(1, iters // 10))
    print(f"aligner fast preset N=100 2000 it        {ms * 1e3:9.1f} us")


def bench_pair(iters):
    """norm2 → attn2 (two-token context) → +residual: fused row pass vs LN + q GEMM + attention + out GEMM."""
    for lab, M, C, H in [("L0 25 snippets", 691200, 320, 5), ("L1 25 snippets", 172800, 640, 10)]:
        x = torch.randn(M, C, device="cuda").half()
        lg, lb = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        wq, wo = (torch.randn(C, C, device="cuda") / math.sqrt(C) for _ in range(2))
        bo = torch.zeros(C, device="cuda")
        k2, v2 = torch.randn(2, C, device="cuda").half(), torch.randn(2, C, device="cuda").half()
        fold = K.fold_attn2_pair(wq, wo, bo, k2, v2, H)
        out = torch.empty_like(x)
        ms_f = timeit(lambda: K.cross_attn_pair(x, lg, lb, 1e-5, *fold, out=out), iters)
        wqp, wop = K.pack_linear(wq, "cuda"), K.pack_linear(wo, "cuda")

        def unfused():
            n2 = K.layernorm(x, lg, lb, 1e-5)
            q = K.gemm(n2, wqp, C)
            o = K.attention_smallkv(q.view(1, M, C), k2[None], v2[None], H)
            K.gemm(o.view(M, C), wop, C, bias=bo, residual=x, out=out)

        ms_u = timeit(unfused, iters)
        print(f"pair  {lab:32s} fused {ms_f * 1e3:9.1f} us  unfused {ms_u * 1e3:9.1f} us  "
              f"({4 * M * C / ms_f / 1e6:6.0f} GB/s row traffic)")


def bench_attn(iters):
    for lab, B, S, H in [("L0 S=27648 H=5 b=8", 8, 27648, 5), ("L1 S=6912 H=10 b=8", 8, 6912, 10),
                         ("L2 S=1728 H=20 b=8", 8, 1728, 20), ("mid S=432 H=20 b=8", 8, 432, 20),
                         # the pipeline's launch shapes (25-snippet UNet batches)
                         ("L0 S=27648 H=5 b=25", 25, 27648, 5), ("L1 S=6912 H=10 b=25", 25, 6912, 10),
                         ("L2 S=1728 H=20 b=25", 25, 1728, 20)]:
        C = H * 64
        qkv = torch.randn(B, S, 3 * C, device="cuda").half()
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        out = torch.empty(B, S, C, device="cuda", dtype=torch.float16)
        ms = timeit(lambda: K.attention(q, k, v, H, out=out), max(2, iters // 4))
        fl = 4.0 * B * H * S * S * 64
        print(f"attn  {lab:32s} {ms * 1e3:9.1f} us  {fl / ms / 1e9:8.1f} TFLOP/s")


def bench_attn512(iters):
    """VAE mid-block attention (1 head, d = 512): flash kernel vs GEMM → softmax → GEMM."""
    for B, S in [(16, 9216), (75, 9216), (16, 2304)]:
        qkv = torch.randn(B, S, 1536, device="cuda").half()
        q, k, v = qkv[..., :512], qkv[..., 512:1024], qkv[..., 1024:]
        sc = 1.0 / math.sqrt(512)
        fl = 4.0 * B * S * S * 512
        ms_f = timeit(lambda: K.attention_d512(q, k, v, sc), iters)
        os.environ["RDMI_VAE_FLASH"] = "0"
        ms_g = timeit(lambda: K.attention_1head(q, k, v, sc), iters)
        os.environ.pop("RDMI_VAE_FLASH")
        print(f"attn512 B={B} S={S}: flash {ms_f * 1e3:9.1f} us {fl / ms_f / 1e9:7.1f} TF/s | gemm-softmax-gemm "
              f"{ms_g * 1e3:9.1f} us {fl / ms_g / 1e9:7.1f} TF/s", flush=True)


def bench_gn(iters):
    for lab, B, HW, C in [("unet 320 96^2 x24", 24, 9216, 320), ("vae 128 768^2 x8", 8, 589824, 128),
                          ("vae 256 384^2 x8", 8, 147456, 256), ("vae 512 96^2 x15", 15, 9216, 512),
                          ("vae 512 192^2 x15", 15, 36864, 512), ("unet 320 96^2 x75", 75, 9216, 320),
                          ("unet 640 48^2 x75", 75, 2304, 640), ("unet 1280 24^2 x75", 75, 576, 1280),
                          ("unet 1280 12^2 x75", 75, 144, 1280)]:
        x = torch.randn(B, HW, C, device="cuda").half()
        g = torch.ones(C, device="cuda")
        b = torch.zeros(C, device="cuda")
        out = torch.empty_like(x)
        ms_s = timeit(lambda: K.groupnorm_stats(x, 32, 1e-5), iters)
        mr = K.groupnorm_stats(x, 32, 1e-5)
        from rollingdepth_amd._native import lib
        ms_a = timeit(lambda: lib.rdmi_groupnorm_apply(x.data_ptr(), out.data_ptr(), 0, B, HW, C, 32, mr.data_ptr(),
                                                       g.data_ptr(), b.data_ptr(), 1, K._stream()), iters)
        by = x.numel() * 2
        print(f"gn    {lab:32s} stats {ms_s * 1e3:8.1f} us {by / ms_s / 1e6:7.0f} GB/s | apply {ms_a * 1e3:8.1f} us "
              f"{2 * by / ms_a / 1e6:7.0f} GB/s")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="conv,gemm,attn,gn")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    torch.manual_seed(0)
    for part in a.only.split(","):
        {"attn512": bench_attn512, "conv": bench_conv, "gemm": bench_gemm, "attn": bench_attn, "gn": bench_gn, "gnconv": bench_gnconv, "head": bench_head, "conv1": bench_conv1, "gnpart": bench_gnpart, "sweep": bench_cinsweep, "sq": bench_square, "shapes": bench_shapes, "host": bench_host, "aligner": bench_aligner, "pair": bench_pair}[part](a.iters)
