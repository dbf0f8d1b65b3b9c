"""The UNet's 24² / 12² 3×3 convs (off the halo engine: Ho % 16 != 0) at the bench's launch shapes on the
ping-pong engine (default policy) and the classic 3-slot engine (RDMI_GEMM_PP=0): HIP-event time per
launch, TF/s and bitwise equality — a tile-count-quantisation check (845 256×256 tiles = 3.3 rounds of
256 CUs at 24², 1 690 256×128 tiles = 6.6 rounds).

    python tools/small_conv_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
for B, H, Cin, Cout in ((75, 24, 1280, 1280), (75, 12, 1280, 1280), (75, 24, 2560, 1280), (75, 12, 2560, 1280),
                        (75, 24, 1920, 1280), (75, 24, 640, 1280)):
    x = torch.randn(B, H, H, Cin, device="cuda", generator=g).half()
    w = torch.randn(Cout, Cin, 3, 3, generator=torch.Generator().manual_seed(1)) / (9 * Cin) ** 0.5
    wp = K.pack_conv(w, "cuda", Cin)
    b = torch.randn(Cout, device="cuda", generator=g)
    outs = {}
    for name, pp in (("pp", "1"), ("classic", "0"), ("pp", "1"), ("classic", "0")):
        os.environ["RDMI_GEMM_PP"] = pp
        y = K.conv2d(x, wp, Cout, 3, bias=b)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            K.conv2d(x, wp, Cout, 3, bias=b, out=y)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        fl = 2.0 * B * H * H * Cout * 9 * Cin
        print(f"B={B} {H}x{H} {Cin}->{Cout} {name:8s} {ms * 1e3:8.1f} us {fl / ms / 1e9:7.1f} TF/s", flush=True)
        outs[name] = y
    print(f"  bitwise equal: {torch.equal(outs['pp'].view(torch.int16), outs['classic'].view(torch.int16))}", flush=True)
