"""A/B of a halo-conv build switch inside one process (the switch is read from the environment at
every launch): per shape, time both settings alternately over several rounds and check that the
outputs are bitwise identical (the switches change the schedule, not the K order).

    python tools/conv_ab.py [--env RDMI_CONV_PIPE] [--rounds 3] [--iters 10]
TF/s: the 9-tap algorithmic FLOPs (for RDMI_UP2 = 1 an effective rate: the phase form executes 7/9)."""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--env", default="RDMI_CONV_PIPE")
ap.add_argument("--values", default="0,1")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--only", default="")
a = ap.parse_args()

# (label, B, H, Cin, Cout, up, variant): variant plain | gn (input GroupNorm+SiLU) | full (+ residual + moments)
CASES = [
    ("vae 128 768^2 x8 full", 8, 768, 128, 128, False, "full"),
    ("vae 128 768^2 x8 gn", 8, 768, 128, 128, False, "gn"),
    ("vae 128 768^2 x8 plain", 8, 768, 128, 128, False, "plain"),
    ("vae 256->128 768^2 x4 gn", 4, 768, 256, 128, False, "gn"),
    ("vae 256->128 768^2 x8 full", 8, 768, 256, 128, False, "full"),
    ("vae 256 384^2 x8 full", 8, 384, 256, 256, False, "full"),
    ("vae 256 384^2 x18 gn", 18, 384, 256, 256, False, "gn"),
    ("vae 256 384^2 x18 full", 18, 384, 256, 256, False, "full"),
    ("vae 512 192^2 x8 plain", 8, 192, 512, 512, False, "plain"),
    ("vae 512 192^2 x37 plain", 37, 192, 512, 512, False, "plain"),
    ("vae 512 96^2 x75 plain", 75, 96, 512, 512, False, "plain"),
    ("vae up 256 384->768 x8", 8, 384, 256, 256, True, "plain"),
    ("vae up 512 192->384 x8", 8, 192, 512, 512, True, "plain"),
    ("vae up 512 96->192 x8", 8, 96, 512, 512, True, "plain"),
    ("unet up 640 48->96 x75", 75, 48, 640, 640, True, "plain"),
    ("unet 320 96^2 x48 full", 48, 96, 320, 320, False, "full"),
    ("unet 640 48^2 x48 full", 48, 48, 640, 640, False, "full"),
]


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


torch.manual_seed(0)
vals = a.values.split(",")
for lab, B, H, ci, co, up, var in CASES:
    if a.only and a.only not in lab:
        continue
    x = torch.randn(B, H, H, ci, device="cuda").half()
    w0 = torch.randn(co, ci, 3, 3) / math.sqrt(ci * 9)
    w = K.pack_conv(w0, "cuda", ci)
    wu = K.pack_conv_up2(w0, "cuda", ci) if up else None  # phase weights (RDMI_UP2 A/B)
    Ho = 2 * H if up else H
    res = torch.randn(B, Ho, Ho, co, device="cuda").half()
    gm, bt = 1 + 0.1 * torch.randn(ci, device="cuda"), 0.1 * torch.randn(ci, device="cuda")
    bias = 0.02 * torch.randn(co, device="cuda")
    mr = K.groupnorm_stats(x, 32, 1e-6)
    ig = (mr, gm, bt, 32, True) if var != "plain" else None
    if ig is not None and not K.conv2d_in_gn_supported(x, w, co, 3, 32, upsample=up):
        ig = None
    outs = {v: torch.empty(B, Ho, Ho, co, device="cuda", dtype=torch.float16) for v in vals}

    def run(v):
        os.environ[a.env] = v
        K.conv2d(x, w, co, 3, upsample=up, bias=bias, residual=res if var == "full" else None, out=outs[v],
                 gn=var == "full", in_gn=ig, w_up2=wu)

    fl = 2.0 * B * Ho * Ho * co * ci * 9
    best = {v: 1e9 for v in vals}
    for _ in range(a.rounds):
        for v in vals:
            best[v] = min(best[v], timeit(lambda: run(v), a.iters))
    same = all(torch.equal(outs[vals[0]], outs[v]) for v in vals[1:])
    print(f"{lab:28s} " + "  ".join(f"{a.env}={v}: {best[v] * 1e3:8.1f} us {fl / best[v] / 1e9:7.1f} TF/s" for v in vals)
          + f"  bitwise-equal={same}", flush=True)
    os.environ.pop(a.env, None)
