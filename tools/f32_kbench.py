"""Kernel times of the f32 path's engines at the paper preset's shapes (768², 3-frame snippets), per
product mode (RDMI_F32_X3 = 0 exact / 1 bf16x3 / 6 bf16x6), against an f64 reference on a sample.
For A/B of two library builds run it once per library (RDMI_LIB=...).

    python tools/f32_kbench.py [--modes 1,6,0]"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--modes", default="1,6")
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
DEV, F32 = "cuda", torch.float32


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / a.iters)
    return best


CONVS = [("vae 768^2 128->128 x2", 2, 768, 128, 128, False), ("vae 384^2 256->256 x4", 4, 384, 256, 256, False),
         ("vae 192^2 512->512 x8", 8, 192, 512, 512, False), ("vae up 384->768 256 x2", 2, 384, 256, 256, True),
         ("unet 96^2 320->320 x15", 15, 96, 320, 320, False), ("unet 48^2 640->640 x15", 15, 48, 640, 640, False),
         ("vae 768^2 8->128 x4", 4, 768, 8, 128, False)]
GEMMS = [("L0 qkv", 15 * 9216, 960, 320), ("L0 geglu-width", 15 * 9216, 2560, 320), ("L0 ff2", 15 * 9216, 320, 1280),
         ("L2 proj", 15 * 576, 1280, 1280)]
g = torch.Generator(device=DEV).manual_seed(0)
for mode in a.modes.split(","):
    os.environ["RDMI_F32_X3"] = mode
    for lab, B, H, ci, co, up in CONVS:
        x = torch.randn(B, H, H, ci, device=DEV, generator=g)
        w0 = torch.randn(co, ci, 3, 3, generator=torch.Generator().manual_seed(1)) / math.sqrt(ci * 9)
        cp = K.pad_channels(ci)
        xn = K.nchw_to_nhwc(x.permute(0, 3, 1, 2).contiguous(), cp, dtype=F32)
        wp = K.pack_conv(w0, DEV, cp, F32)
        Ho = 2 * H if up else H
        out = torch.empty(B, Ho, Ho, co, device=DEV)
        ms = timeit(lambda: K.conv2d(xn, wp, co, 3, upsample=up, out=out))
        xs = x[:1].double().permute(0, 3, 1, 2)
        if up:
            xs = F.interpolate(xs, scale_factor=2.0, mode="nearest")
        ref = F.conv2d(xs, w0.double().to(DEV), padding=1)
        err = ((out[:1].permute(0, 3, 1, 2).double() - ref).abs().max() / ref.abs().max()).item()
        print(f"mode {mode} conv {lab:26s} {ms * 1e3:9.1f} us {2.0 * B * Ho * Ho * co * ci * 9 / ms / 1e9:7.1f} TF/s "
              f"rel {err:.1e}", flush=True)
        del x, xn, out
    for lab, M, N, Kd in GEMMS:
        x = torch.randn(M, Kd, device=DEV, generator=g)
        w0 = torch.randn(N, Kd, device=DEV, generator=g) / math.sqrt(Kd)
        wp = K.pack_linear(w0, DEV, F32)
        out = torch.empty(M, N, device=DEV)
        ms = timeit(lambda: K.gemm(x, wp, Kd, out=out))
        ref = x[:512].double() @ w0.double().t()
        err = ((out[:512].double() - ref).abs().max() / ref.abs().max()).item()
        print(f"mode {mode} gemm {lab:26s} {ms * 1e3:9.1f} us {2.0 * M * N * Kd / ms / 1e9:7.1f} TF/s rel {err:.1e}",
              flush=True)
