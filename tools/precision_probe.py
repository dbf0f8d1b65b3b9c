"""Where the f16 path's depth error comes from, at the metric resolution (sd2_768 reference fixture).

Runs the f16 and the f32 pipelines on the fixture's inputs and crosses their stages: the decoded
first snippet from {f16, f32} UNet latents × {f16, f32} VAE decoders, each against the reference's
decoded snippet (lattice L1), plus the full forward's depth L1 of both dtypes.

    python tools/precision_probe.py [sd2_768]
"""
import json
import os
import sys

import torch
from safetensors.torch import load_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from rollingdepth_amd import kernels as K  # noqa: E402
from rollingdepth_amd import weights as W  # noqa: E402
from rollingdepth_amd.pipeline import RollingDepthPipeline  # noqa: E402


def main(name="sd2_768"):
    G = os.path.join(ROOT, "tests", "golden")
    t = load_file(os.path.join(G, name + ".safetensors"))
    meta = json.load(open(os.path.join(G, name + ".json")))
    s = meta["depth_stride"]
    frames = W.synth_frames(meta["n_frames"], meta["res"], meta["res"], seed=0)
    pipes, recs, outs = {}, {}, {}
    for dt in (torch.float16, torch.float32):
        p = RollingDepthPipeline.from_synthetic(meta["unet"], meta["vae"], meta["scheduler"], device="cuda",
                                                torch_dtype=dt)
        p.empty_text_embed = t["context"]
        rec = {}
        out = p.forward(frames[None], list(meta["dilations_in"]), meta["cap_dilation"], [3], [1], [1], None, 0, 3,
                        6, None, False, 4, False, init_noise=t["init_noise"], record=rec)
        pipes[dt], recs[dt], outs[dt] = p, rec, out
        d = (out.depth_pred[..., ::s, ::s].float() - t["depth_pred_sub"].float()).abs().mean().item()
        sn = (out.snippet_ls[0][0, :, 0, ::s, ::s].float() - t["snippet_0_first_sub"].float()).abs().mean().item()
        print(f"{dt}: depth L1 {d:.3e}  decoded snippet L1 {sn:.3e}", flush=True)
    ref = t["snippet_0_first_sub"].float()
    H = W_ = meta["res"]
    for ldt in (torch.float16, torch.float32):
        lat = recs[ldt]["snippet_latent"][0][:3]  # NHWC [3, h, w, 8] channels 0..3
        for vdt in (torch.float16, torch.float32):
            z = K.ddim_combine(lat[..., :4].to(vdt), lat[..., :4].to(vdt), 1.0 / 0.18215, 0.0, 1.0, 4, 8)
            dec = torch.empty((3, H, W_, 1), dtype=vdt, device="cuda")
            pipes[vdt].decode_depth(z, dec)
            e = (dec[:, ::s, ::s, 0].float().cpu() - ref).abs().mean().item()
            print(f"latent {ldt} → decoder {vdt}: decoded snippet L1 {e:.3e}", flush=True)
    # encoder precision: rgb latent vs the reference
    for dt in (torch.float16, torch.float32):
        rl = recs[dt]["rgb_latent"][..., :4].permute(0, 3, 1, 2).float().cpu()
        e = (rl - t["rgb_latent"].float()).abs()
        print(f"{dt}: rgb latent mean {e.mean().item():.3e} max {e.max().item():.3e}", flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
