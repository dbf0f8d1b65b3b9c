"""Probe: VAE encode/decode results must not depend on the chunk size (per-frame arithmetic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import config as C  # noqa: E402
from rollingdepth_amd import weights as W  # noqa: E402
from rollingdepth_amd.pipeline import RollingDepthPipeline  # noqa: E402

pipe = RollingDepthPipeline.from_synthetic(C.SD2_UNET, C.SD2_VAE, C.RD_SCHEDULER, device="cuda")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
frames = W.synth_frames(N, 768, 768, seed=0).to("cuda", torch.float16)
res = {}
for vb in (16, 75):
    pipe.vae_batch = vb
    lat = pipe.encode_rgb(frames)
    z = (lat[:75] / 0.18215).contiguous()
    out = torch.empty((75, 768, 768, 1), dtype=torch.float16, device="cuda")
    pipe.decode_depth(z, out)
    torch.cuda.synchronize()
    res[vb] = (lat.float().cpu(), out.float().cpu())
    print(f"vb={vb}: latent mean {lat.float().mean().item():.6f} absmax {lat.float().abs().max().item():.4f}", flush=True)
dl = (res[16][0] - res[75][0]).abs()
dd = (res[16][1] - res[75][1]).abs()
print(f"latent diff max {dl.max().item():.3e} (frames differing: {(dl.flatten(1).amax(1) > 0).sum().item()})")
print(f"decode diff max {dd.max().item():.3e} (frames differing: {(dd.flatten(1).amax(1) > 0).sum().item()})")
