"""Targets for rocprofv3 PMC passes (tools/pmc_round.sh): one shape, a few launches.

    python tools/traffic_probe.py --what copy|conv|attn [--iters 3]

copy: a 1 GiB f16 device copy (reads 1 GiB, writes 1 GiB) — the known-bytes calibration of
      FETCH_SIZE / WRITE_SIZE for 16-B-per-lane streaming (the guide's ½ correction is checked here);
conv: the dominant conv of the metric config — VAE decoder 768² 128→128, 3×3, with the fused
      GroupNorm+SiLU input, the residual add and the GroupNorm-moment epilogue (ResnetBlock2D.conv2 of
      up_blocks.3), batch 8 (algorithmic bytes printed);
attn: level-0 cross-frame attention at 768² (B = 8 snippets, S = 27 648, H = 5)."""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--what", default="conv")
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--res", type=int, default=768)
ap.add_argument("--cin", type=int, default=128)
ap.add_argument("--variant", default="full", choices=["full", "plain", "gn", "gnres"],
                help="conv: full = GN input + residual + moments; plain = conv only; gn = GN input only; "
                     "gnres = GN input + residual")
a = ap.parse_args()
torch.manual_seed(0)
if a.what == "copy":
    n = 1 << 29  # halves: 1 GiB
    x = torch.randn(n // 1024, 1024, device="cuda").half()
    y = torch.empty_like(x)
    fn = lambda: y.copy_(x)  # noqa: E731
    print(f"algorithmic: read {n * 2} B, write {n * 2} B per launch")
elif a.what == "conv":
    B, H, W, C = a.batch, a.res, a.res, a.cin
    x = torch.randn(B, H, W, C, device="cuda").half()
    res = torch.randn(B, H, W, C, device="cuda").half()
    gm = 1 + 0.1 * torch.randn(C, device="cuda")
    bt = 0.1 * torch.randn(C, device="cuda")
    w = K.pack_conv(torch.randn(C, C, 3, 3) / math.sqrt(C * 9), "cuda", C)
    b = 0.02 * torch.randn(C, device="cuda")
    mr = K.groupnorm_stats(x, 32, 1e-6)
    out = torch.empty(B, H, W, C, device="cuda", dtype=torch.float16)

    ig = None if a.variant == "plain" else (mr, gm, bt, 32, True)
    rr = res if a.variant in ("full", "gnres") else None
    if ig is not None and not K.conv2d_in_gn_supported(x, w, C, 3, 32):
        ig = None
        print("GroupNorm input fusion not supported at this shape: unfused input")

    def fn():
        K.conv2d(x, w, C, 3, bias=b, residual=rr, out=out, gn=a.variant == "full", in_gn=ig)

    act = B * H * W * C * 2
    print(f"algorithmic: read {2 * act + w.numel() * 2} B (input + residual + weights), write {act} B "
          f"(+ GroupNorm moments {C // 4 * B * H * W // 32 * 8} B); {2.0 * B * H * W * C * C * 9:.4e} FLOP")
elif a.what == "f32conv":  # the f32 path's conv (RDMI_F32_X3 picks the product form at packing)
    B, H, W, C = a.batch, a.res, a.res, a.cin
    x = torch.randn(B, H, W, C, device="cuda")
    w = K.pack_conv(torch.randn(C, C, 3, 3) / math.sqrt(C * 9), "cuda", C, torch.float32)
    out = torch.empty(B, H, W, C, device="cuda")
    fn = lambda: K.conv2d(x, w, C, 3, out=out)  # noqa: E731
    print(f"f32 conv {B}x{H}x{W} {C}->{C}: {2.0 * B * H * W * C * C * 9:.4e} FLOP")
elif a.what == "f32gemm":  # the f32 path's Linear (UNet L0 GEGLU-free projection shape by default)
    M, N, Kd = a.batch * 9216, 3 * a.cin, a.cin
    x = torch.randn(M, Kd, device="cuda")
    w = K.pack_linear(torch.randn(N, Kd) / math.sqrt(Kd), "cuda", torch.float32)
    out = torch.empty(M, N, device="cuda")
    fn = lambda: K.gemm(x, w, Kd, out=out)  # noqa: E731
    print(f"f32 gemm M={M} N={N} K={Kd}: {2.0 * M * N * Kd:.4e} FLOP")
elif a.what == "f32attn":  # the f32 path's cross-frame attention (RDMI_F32_X3 / X6 pick the product form)
    B, S, H = a.batch, 27648, 5
    C = H * 64
    qkv = torch.randn(B, S, 3 * C, device="cuda")
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    out = torch.empty(B, S, C, device="cuda")
    fn = lambda: K.attention(q, k, v, H, out=out)  # noqa: E731
    print(f"f32 attention: {4.0 * B * H * S * S * 64:.4e} FLOP")
else:
    B, S, H = a.batch, 27648, 5
    C = H * 64
    qkv = torch.randn(B, S, 3 * C, device="cuda").half()
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    out = torch.empty(B, S, C, device="cuda", dtype=torch.float16)
    fn = lambda: K.attention(q, k, v, H, out=out)  # noqa: E731
    print(f"algorithmic: {4.0 * B * H * S * S * 64:.4e} FLOP; read {3 * B * S * C * 2} B, write {B * S * C * 2} B")
for _ in range(a.iters):
    fn()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
fn()
e.record()
torch.cuda.synchronize()
print(f"done: {s.elapsed_time(e) * 1e3:.1f} us per launch (event-timed, last launch)")
