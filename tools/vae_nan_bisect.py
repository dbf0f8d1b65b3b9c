"""Probe: first VAE encoder stage that turns non-finite at a large chunk (bisects the overflow)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import config as C  # noqa: E402
from rollingdepth_amd import kernels as K  # noqa: E402
from rollingdepth_amd import weights as W  # noqa: E402
from rollingdepth_amd.pipeline import RollingDepthPipeline  # noqa: E402

pipe = RollingDepthPipeline.from_synthetic(C.SD2_UNET, C.SD2_VAE, C.RD_SCHEDULER, device="cuda")
v = pipe.vae
B = int(sys.argv[1]) if len(sys.argv) > 1 else 30
frames = W.synth_frames(B, 768, 768, seed=0).to("cuda", torch.float16)
x = K.nchw_to_nhwc(frames, v.in_pad)


def chk(tag, t):
    bad = (~torch.isfinite(t.float())).flatten(1).any(1)
    print(f"{tag:40s} shape {tuple(t.shape)} nonfinite frames {bad.nonzero().flatten().tolist()[:8]}", flush=True)
    return bool(bad.any())


chk("input", x)
h = v.e_in(x, gn=True)
chk("e_in", h)
for bi, (res, ds) in enumerate(v.e_down):
    for ri, r in enumerate(res):
        h = r(h)
        if chk(f"down{bi} res{ri}", h):
            sys.exit(0)
    if ds is not None:
        h = ds(h, pad_tl=0, out_hw=v._down(h.shape[1], h.shape[2]), gn=True)
        if chk(f"down{bi} ds", h):
            sys.exit(0)
