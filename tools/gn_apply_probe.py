"""Unfused GroupNorm(+SiLU) apply (rdmi_groupnorm_apply) at the pipeline's shapes — the VAE's 512-channel
norms and the UNet Transformer2DModel norm — per launch (HIP events) for the row-unrolled form (default)
and the one-row-per-trip form (RDMI_GN_APPLY_U=1), with the HBM rate of the algorithmic bytes (read + write
of x) and bitwise equality.

    python tools/gn_apply_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402
from rollingdepth_amd._native import lib  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
for lab, B, H, C, silu in (("vae 96^2 512 silu B=75", 75, 96, 512, 1), ("vae 192^2 512 silu B=37", 37, 192, 512, 1),
                           ("vae 384^2 512 silu B=9", 9, 384, 512, 1), ("unet 96^2 320 B=75", 75, 96, 320, 0),
                           ("vae 768^2 128 silu B=5", 5, 768, 128, 1)):
    x = torch.randn(B, H, H, C, device="cuda", generator=g).half()
    gam = torch.rand(C, device="cuda", generator=g) + 0.5
    bet = torch.randn(C, device="cuda", generator=g) * 0.1
    mr = K.groupnorm_stats(x, 32, 1e-6)
    y = torch.empty_like(x)
    outs = {}
    for u in ("4", "1", "4", "1"):
        os.environ["RDMI_GN_APPLY_U"] = u

        def run():
            K.check(lib.rdmi_groupnorm_apply(x.data_ptr(), y.data_ptr(), 0, B, H * H, C, 32, mr.data_ptr(),
                                             gam.data_ptr(), bet.data_ptr(), silu, K._stream()), "apply")
        run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            run()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        print(f"{lab:26s} U={u} {ms * 1e3:8.1f} us {4 * x.numel() / ms / 1e9:6.2f} TB/s", flush=True)
        outs[u] = y.clone()
    print(f"{lab:26s} bitwise equal: {torch.equal(outs['1'].view(torch.int16), outs['4'].view(torch.int16))}", flush=True)
