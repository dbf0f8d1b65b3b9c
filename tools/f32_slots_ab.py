"""A/B of the f32 engine's LDS ring (gemm_f32.hip, RDMI_F32_SLOTS read per launch): 3 slots, one
workgroup per CU (96 KiB) vs 2 slots, two workgroups per CU (64 KiB), for both product forms
(RDMI_F32_X3), at the paper preset's launch shapes (15-snippet UNet batch = 45 frames, 768²).
The K order is the same, so the outputs must be bitwise equal.

    python tools/f32_slots_ab.py"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

DEV, F32 = "cuda", torch.float32


def _time(fn, n=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


g = torch.Generator(device=DEV).manual_seed(0)
cases = [("gemm", 45 * 9216, 960, 320), ("gemm", 45 * 9216, 2560, 320), ("gemm", 45 * 9216, 320, 1280),
         ("gemm", 45 * 2304, 1920, 640), ("conv", 45, 96, 320, 320, False), ("conv", 45, 48, 640, 640, False),
         ("conv", 45, 24, 1280, 1280, False), ("conv", 8, 384, 256, 256, False), ("conv", 8, 192, 512, 512, True),
         ("conv", 4, 768, 128, 128, False)]
for x3 in ("1", "0"):
    os.environ["RDMI_F32_X3"] = x3
    for cs in cases:
        if cs[0] == "gemm":
            _, M, N, Kd = cs
            a = torch.randn(M, Kd, device=DEV, generator=g)
            w = K.pack_linear(torch.randn(N, Kd, device=DEV, generator=g) / math.sqrt(Kd), DEV, F32)
            fl = 2.0 * M * N * Kd
            run = lambda o: K.gemm(a, w, Kd, out=o)  # noqa: E731
            lab = f"gemm M={M} N={N} K={Kd}"
        else:
            _, B, H, Cin, Cout, up = cs
            x = torch.randn(B, H, H, Cin, device=DEV, generator=g)
            w = K.pack_conv(torch.randn(Cout, Cin, 3, 3) / math.sqrt(Cin * 9), DEV, Cin, F32)
            Ho = 2 * H if up else H
            fl = 2.0 * B * Ho * Ho * Cout * 9 * Cin
            run = lambda o: K.conv2d(x, w, Cout, 3, upsample=up, out=o)  # noqa: E731
            lab = f"conv B={B} {H}^2 {Cin}->{Cout}{' up' if up else ''}"
        outs, best = {}, {}
        for _ in range(3):
            for ns in ("3", "2"):
                os.environ["RDMI_F32_SLOTS"] = ns
                if ns not in outs:
                    outs[ns] = run(None)
                best[ns] = min(best.get(ns, 1e9), _time(lambda: run(outs[ns])))
        same = torch.equal(outs["3"], outs["2"])
        print(f"{'x3 ' if x3 == '1' else 'f32'} {lab:34s} " +
              "  ".join(f"slots={ns}: {best[ns]:8.3f} ms {fl / best[ns] / 1e9:6.1f} TF/s" for ns in ("3", "2")) +
              f"  bitwise-equal={same}", flush=True)
        del outs
        torch.cuda.empty_cache()
os.environ.pop("RDMI_F32_SLOTS", None)
