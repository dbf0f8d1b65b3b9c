"""Phase-decomposed ×2 upsample conv (RDMI_UP2) vs the 9-tap form at the VAE decoder's shapes,
including the batch split at 2^30 input elements and the epilogue's GroupNorm moments; then a whole
VAE decode (SD2 shapes, 768²) with and without it.

    python tools/up2_probe.py"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

torch.manual_seed(0)
for B, H, ci in [(12, 96, 512), (12, 192, 512), (12, 384, 256), (75, 192, 512)]:
    x = (torch.randn(B, H, H, ci, device="cuda") * 2).half()
    w0 = torch.randn(ci, ci, 3, 3) / math.sqrt(ci * 9)
    w, wu = K.pack_conv(w0, "cuda", ci), K.pack_conv_up2(w0, "cuda", ci)
    b = 0.1 * torch.randn(ci, device="cuda")
    y2 = K.conv2d(x, w, ci, 3, upsample=True, bias=b, gn=True, w_up2=wu)
    y9 = K.conv2d(x, w, ci, 3, upsample=True, bias=b, gn=True)
    m2, m9 = K.groupnorm_stats(y2, 32, 1e-6), K.groupnorm_stats(y9, 32, 1e-6)
    ms = K.groupnorm_stats(y2.clone(), 32, 1e-6)  # standalone pass over the up2 output
    d = (y2.float() - y9.float()).abs()
    print(f"B={B} {H}->{2 * H} C={ci}: |y2-y9| mean {d.mean().item():.2e} max {d.max().item():.2e} "
          f"(|y| mean {y9.float().abs().mean().item():.2e}); moments fused-vs-standalone "
          f"{(m2 - ms).abs().max().item():.2e}, up2-vs-9tap {(m2 - m9).abs().max().item():.2e}", flush=True)
    del x, y2, y9

from rollingdepth_amd import config as C  # noqa: E402
from rollingdepth_amd.pipeline import RollingDepthPipeline  # noqa: E402

pipe = RollingDepthPipeline.from_synthetic(C.SD2_UNET, C.SD2_VAE, C.RD_SCHEDULER, device="cuda")
lat = torch.randn(6, 96, 96, 8, device="cuda").half()
outs = {}
for v in ("0", "1"):
    os.environ["RDMI_UP2"] = v
    outs[v] = pipe.vae.decode_depth(lat) if hasattr(pipe.vae, "decode_depth") else pipe.vae.decode(lat)
    torch.cuda.synchronize()
d = (outs["0"].float() - outs["1"].float()).abs()
print(f"VAE decode 6x768^2: |up2 - 9tap| mean {d.mean().item():.2e} max {d.max().item():.2e}", flush=True)
