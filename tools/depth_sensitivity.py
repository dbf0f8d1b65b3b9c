"""Sensitivity of the end-to-end depth error to rounding-level changes (sd2_768 reference fixture):
the same forward under build switches that only change f16 rounding (phase-decomposed upsample
conv, flash vs GEMM VAE mid attention, 32×32×16 conv form), reporting the decoded-snippet error
(before the aligner) and the co-aligned depth error (after the aligner's 2000 sign-driven Adam steps
and the min/max renormalisation) against the reference.  The decoded depth is kept in f32 unless
RDMI_DEPTH_F32=0 is set for the run (pipeline.depth_f32).  (Round 2's 16-variant study also toggled
an exact-erf GEGLU, RDMI_GELU_EXACT, since removed: profiles/r02_v28_depth_sens3.log.)

    python tools/depth_sensitivity.py [fixture]"""
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from safetensors.torch import load_file  # noqa: E402

from rollingdepth_amd import weights as W  # noqa: E402
from rollingdepth_amd.pipeline import RollingDepthPipeline  # noqa: E402

G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
name = sys.argv[1] if len(sys.argv) > 1 else "sd2_768"
t = load_file(os.path.join(G, name + ".safetensors"))
meta = json.load(open(os.path.join(G, name + ".json")))
frames = W.synth_frames(meta["n_frames"], meta["res"], meta["res"], seed=meta["frames_seed"])
pipe = RollingDepthPipeline.from_synthetic(meta["unet"], meta["vae"], meta["scheduler"], device="cuda")
pipe.snippet_batch = 25
pipe.empty_text_embed = t["context"]
s = meta["depth_stride"]
base = None
print(f"{name}: decoded depth dtype {pipe.depth_dtype}", flush=True)
# rounding-only switches (each variant an equally valid f16 evaluation order): phase upsample, VAE
# flash attention, the 32×32×16 conv form
for up2, fl, h32 in itertools.product("01", "10", "01"):
    os.environ.update(RDMI_UP2=up2, RDMI_VAE_FLASH=fl, RDMI_CONV_H32=h32)
    dil = list(meta["dilations_in"])
    out = pipe.forward(frames[None].half(), dil, meta["cap_dilation"], [3], [1], [1], None, meta["refine_step"], 3,
                       meta["refine_start_dilation"], None, False, 4, False, init_noise=t["init_noise"])
    sn = [(out.snippet_ls[i][0, :, 0, ::s, ::s].float() - t[f"snippet_{i}_first_sub"].float()).abs().mean().item()
          for i in range(len(dil))]
    d = out.depth_pred[..., ::s, ::s].float() - t["depth_pred_sub"].float()
    snips = torch.cat([x.float().flatten() for x in out.snippet_ls])
    dep = out.depth_pred.float()
    rel = ""
    if base is None:
        base = (snips, dep)
    else:
        ds, dd = (snips - base[0]).abs(), (dep - base[1]).abs()
        rel = (f" | vs first variant: all snippets mean {ds.mean().item():.2e} max {ds.max().item():.2e}, "
               f"depth mean {dd.mean().item():.2e}")
    print(f"UP2={up2} VAE_FLASH={fl} H32={h32}: snippet[0] L1 {' '.join(f'{v:.2e}' for v in sn)} | depth L1 "
          f"{d.abs().mean().item():.2e} mean(d) {d.mean().item():+.2e} max {d.abs().max().item():.2e}{rel}", flush=True)
