"""GroupNorm(+SiLU) → 3×3 conv, fused into the halo conv's input path vs the apply pass + plain conv, at the
pipeline's own batch sizes for every halo-eligible conv the default policy (kernels.gn_conv2d, RDMI_GN_FUSE=1)
leaves unfused (Cin > 256).  Both forms carry the epilogue the pipeline gives that conv (conv1: GroupNorm
moments of the output; conv2: residual + moments).  The two forms compute the same values bitwise
(tests/test_kernels_gpu.py::test_conv2d_fused_input_groupnorm), so the choice is a pure speed policy.

    python tools/gn_fuse_probe.py [--rounds 3] [--iters 10]"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402
from rollingdepth_amd._native import lib  # noqa: E402

# (label, B, H, Cin, Cout, residual) — B as the fast preset runs them (UNet: 25-snippet batches = 75 frames;
# VAE encoder: 50-frame chunks; decoder: 75-frame groups at 96², 37-frame chunks at 192², 9 at 384²)
CASES = [
    ("unet 96^2 320->320 conv2", 75, 96, 320, 320, True),
    ("unet 96^2 640->320 conv1", 75, 96, 640, 320, False),
    ("unet 96^2 960->320 conv1", 75, 96, 960, 320, False),
    ("unet 48^2 320->640 conv1", 75, 48, 320, 640, False),
    ("unet 48^2 640->640 conv2", 75, 48, 640, 640, True),
    ("unet 48^2 1280->640 conv1", 75, 48, 1280, 640, False),
    ("unet 48^2 1920->640 conv1", 75, 48, 1920, 640, False),
    ("vae enc 192^2 512->512 conv2", 50, 192, 512, 512, True),
    ("vae enc 96^2 512->512 conv2", 50, 96, 512, 512, True),
    ("vae dec 96^2 512->512 conv2", 75, 96, 512, 512, True),
    ("vae dec 192^2 512->512 conv2", 37, 192, 512, 512, True),
    ("vae dec 384^2 512->256 conv1", 9, 384, 512, 256, False),
]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    os.environ["RDMI_GN_FUSE"] = "1"
    for r in range(a.rounds):
        for lab, B, H, ci, co, has_res in CASES:
            x = torch.randn(B, H, H, ci, device="cuda").half()
            w = K.pack_conv(torch.randn(co, ci, 3, 3) / math.sqrt(ci * 9), "cuda", ci)
            g, b = torch.rand(ci, device="cuda") + 0.5, torch.randn(ci, device="cuda") * 0.1
            if not K.conv2d_in_gn_supported(x, w, co, 3, 32):
                print(f"{lab:32s} B={B:3d}: not halo-eligible", flush=True)
                continue
            mr = K.groupnorm_stats(x, 32, 1e-6)
            res = torch.randn(B, H, H, co, device="cuda").half() if has_res else None
            h = torch.empty_like(x)
            out = torch.empty(B, H, H, co, device="cuda", dtype=torch.float16)

            def unfused():
                lib.rdmi_groupnorm_apply(x.data_ptr(), h.data_ptr(), 0, B, H * H, ci, 32, mr.data_ptr(), g.data_ptr(),
                                         b.data_ptr(), 1, K._stream())
                K.conv2d(h, w, co, 3, out=out, residual=res, gn=True)

            def fused():
                K.conv2d(x, w, co, 3, out=out, residual=res, gn=True, in_gn=(mr, g, b, 32, True))

            if r == 0:  # same values either way
                unfused()
                u = out.clone()
                fused()
                assert torch.equal(u, out), lab
            mu, mf = timeit(unfused, a.iters), timeit(fused, a.iters)
            print(f"round {r} {lab:32s} B={B:3d}: apply+conv {mu * 1e3:8.1f} us  fused {mf * 1e3:8.1f} us  "
                  f"fused/unfused {mf / mu:6.3f}", flush=True)
            del x, w, res, h, out


if __name__ == "__main__":
    main()
