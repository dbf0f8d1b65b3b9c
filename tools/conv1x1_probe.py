"""The VAE conv_shortcut 1×1 convs at the bench's launch shapes: streaming kernel (conv1x1.hip) vs the
GEMM engines (RDMI_CONV1X1=0) — HIP-event time per launch, HBM rate of the algorithmic bytes, and
bitwise equality of the outputs.

    python tools/conv1x1_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
for lab, B, H, Cin, Cout in (("dec 768^2 256->128 B=5", 5, 768, 256, 128), ("dec 768^2 256->128 B=4", 4, 768, 256, 128),
                             ("enc 384^2 128->256 B=50", 25, 384, 128, 256)):
    x = torch.randn(B, H, H, Cin, device="cuda", generator=g).half()
    w = torch.randn(Cout, Cin, 1, 1, generator=torch.Generator().manual_seed(1)) / Cin ** 0.5
    wp = K.pack_conv(w, "cuda", Cin)
    b = torch.randn(Cout, device="cuda", generator=g)
    y = {}
    for mode in ("0", "1", "0", "1"):
        os.environ["RDMI_CONV1X1"] = mode
        out = K.conv2d(x, wp, Cout, 1, pad=0, bias=b)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            K.conv2d(x, wp, Cout, 1, pad=0, bias=b, out=out)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        by = B * H * H * (Cin + Cout) * 2
        print(f"{lab:26s} RDMI_CONV1X1={mode} {ms * 1e3:8.1f} us {by / ms / 1e9:6.2f} TB/s", flush=True)
        y[mode] = out
    print(f"{lab:26s} bitwise equal: {torch.equal(y['0'].view(torch.int16), y['1'].view(torch.int16))}", flush=True)
