"""Error budget of the f16 path: where in the f16 forward does the depth error
against the reference come from?  One stage at a time runs on the f32 engines (x6 products:
f32-equivalent, RDMI_F32_X3=6) while everything else stays f16; reported per stage: the decoded-snippet
L1 (before the aligner) and the co-aligned depth L1 (after the aligner + min/max renormalisation)
against the reference fixture — the same lattice statistics as tests/test_pipeline_gpu.py::_run_compact.

    python tools/error_budget.py [sd2_768 [sd2_1024 ...]] [--stages enc,unet_down,...]

Stages: enc (whole encoder), unet_down / unet_mid / unet_up (UNet levels, the skips converted at the
boundary), dec_in (post_quant + conv_in), dec_mid (mid resnets + attention), dec_up0..3 (decoder up
blocks incl. their upsample conv), dec_head (conv_norm_out + SiLU + conv_out), and unions (unet, dec,
all).  The f32 modules hold the same synthetic weights (from_synthetic, same seed); activations cross a
stage boundary by one rounding to the other dtype."""
import json
import os
import sys
import time

os.environ.setdefault("RDMI_F32_X3", "6")  # x6 everywhere: f32-equivalent products
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from safetensors.torch import load_file  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402
from rollingdepth_amd import weights as W  # noqa: E402
from rollingdepth_amd.pipeline import RollingDepthPipeline  # noqa: E402

G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
F16, F32 = torch.float16, torch.float32
UNET_STAGES = ("unet_down", "unet_mid", "unet_up")
DEC_STAGES = ("dec_in", "dec_mid", "dec_up0", "dec_up1", "dec_up2", "dec_up3", "dec_head")
UNIONS = {"unet": UNET_STAGES, "dec": DEC_STAGES, "all": ("enc",) + UNET_STAGES + DEC_STAGES}


def _to(x, dt):
    return x if x.dtype == dt else x.to(dt).contiguous()


def hybrid_unet(u16, u32, on):
    """UNet.forward (unet.py) with the levels in `on` run by the f32 UNet."""
    def fwd(sample, t, num_view):
        def mod(stage):
            return (u32, F32) if stage in on else (u16, F16)

        u, dt = mod("unet_down")
        temb = u.time_embedding(t)
        x = u.conv_in(_to(sample, dt), gn=True)
        skips = [x]
        for bi, blk in enumerate(u.down):
            for j, r in enumerate(blk["res"]):
                x = r(x, temb)
                if blk["attn"]:
                    x = blk["attn"][j](x, num_view)
                skips.append(x)
            if blk["ds"] is not None:
                x = blk["ds"](x, gn=True)
                skips.append(x)
        u, dt = mod("unet_mid")
        temb = u.time_embedding(t)
        x = _to(x, dt)
        x = u.mid_res[0](x, temb)
        x = u.mid_attn(x, num_view)
        x = u.mid_res[1](x, temb)
        u, dt = mod("unet_up")
        temb = u.time_embedding(t)
        x = _to(x, dt)
        for blk in u.up:
            for j, r in enumerate(blk["res"]):
                x = K.concat_channels(x, _to(skips.pop(), dt))
                x = r(x, temb)
                if blk["attn"]:
                    x = blk["attn"][j](x, num_view)
            if blk["us"] is not None:
                x = blk["us"](x, upsample=True, gn=True)
        x = K.groupnorm(x, u.norm_out.g, u.norm_out.b, u.groups, u.eps, silu=True)
        return _to(u.conv_out(x), F16)
    return fwd


def hybrid_decode(v16, v32, on):
    """VAE.decode_depth (vae.py) with the stages in `on` run by the f32 VAE."""
    def dec(z, out=None):
        def mod(stage):
            return (v32, F32) if stage in on else (v16, F16)

        B, hh, ww, _ = z.shape
        v, dt = mod("dec_in")
        h = torch.zeros((B, hh, ww, v.d_in.cin_pad), dtype=dt, device=z.device)
        v.post_quant(_to(z, dt), out=h)
        h = v.d_in(h, gn=True)
        v, dt = mod("dec_mid")
        h = _to(h, dt)
        h = v.d_mid[0](h)
        h = v.d_attn(h)
        h = v.d_mid[1](h)
        for i in range(len(v16.d_up)):
            v, dt = mod(f"dec_up{i}")
            h = _to(h, dt)
            res, us = v.d_up[i]
            for r in res:
                h = r(h)
            if us is not None:
                h = us(h, upsample=True, gn=True)
        v, dt = mod("dec_head")
        h = _to(h, dt)
        o = torch.empty(out.shape, dtype=F32, device=z.device)
        K.conv3x3_to1_gn(h, v.d_norm.g, v.d_norm.b, v.groups, 1e-6, True, v.d_w9, v.d_b, out=o)
        out.copy_(o)
        return out
    return dec


def hybrid_encode(v16, v32, on):
    def enc(x, out=None):
        if "enc" not in on:
            return v16.encode(x, out=out)
        o = v32.encode(_to(x, F32))
        out.copy_(o.to(out.dtype))
        return out
    return enc


def run(name, stages):
    t = load_file(os.path.join(G, name + ".safetensors"))
    meta = json.load(open(os.path.join(G, name + ".json")))
    frames = W.synth_frames(meta["n_frames"], meta["res"], meta["res"], seed=meta["frames_seed"])
    p16 = RollingDepthPipeline.from_synthetic(meta["unet"], meta["vae"], meta["scheduler"], device="cuda")
    p32 = RollingDepthPipeline.from_synthetic(meta["unet"], meta["vae"], meta["scheduler"], device="cuda",
                                              torch_dtype=F32)
    p16.snippet_batch = 25
    p16.empty_text_embed = t["context"]
    p32.empty_text_embed = t["context"]
    p32._context()
    s = meta["depth_stride"]
    orig = (p16.unet.forward, p16.vae.decode_depth, p16.vae.encode)
    print(f"{name}: {meta['n_frames']} frames {meta['res']}², dilations {meta['dilations_in']}, decoded depth "
          f"{p16.depth_dtype}, f32 engines {K.f32_precision_label()}", flush=True)
    for st in stages:
        on = set(UNIONS.get(st, (st,))) if st != "none" else set()
        p16.unet.forward, p16.vae.decode_depth, p16.vae.encode = orig
        if on & set(UNET_STAGES):
            p16.unet.forward = hybrid_unet(p16.unet, p32.unet, on)
        if on & set(DEC_STAGES):
            p16.vae.decode_depth = hybrid_decode(p16.vae, p32.vae, on)
        if "enc" in on:
            p16.vae.encode = hybrid_encode(p16.vae, p32.vae, on)
        dil = list(meta["dilations_in"])
        t0 = time.perf_counter()
        out = p16.forward(frames[None].half(), dil, meta["cap_dilation"], [3], [1], [1], None, meta["refine_step"], 3,
                          meta["refine_start_dilation"], None, False, 4, False, init_noise=t["init_noise"])
        torch.cuda.synchronize()
        sn = [(out.snippet_ls[i][0, :, 0, ::s, ::s].float() - t[f"snippet_{i}_first_sub"].float()).abs().mean().item()
              for i in range(len(dil))]
        d = out.depth_pred[..., ::s, ::s].float() - t["depth_pred_sub"].float()
        print(f"  {st:10s}: snippet[0] L1 {' '.join(f'{v:.2e}' for v in sn)} | depth L1 {d.abs().mean().item():.2e} "
              f"mean(d) {d.mean().item():+.2e} max {d.abs().max().item():.2e}  ({time.perf_counter() - t0:.1f} s)",
              flush=True)
    p16.unet.forward, p16.vae.decode_depth, p16.vae.encode = orig
    del p16, p32
    torch.cuda.empty_cache()


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    stages = ["none", "enc", *UNET_STAGES, "unet", *DEC_STAGES, "dec", "all"]
    if "--stages" in sys.argv:
        stages = sys.argv[sys.argv.index("--stages") + 1].split(",")
        args = [a for a in args if a != sys.argv[sys.argv.index("--stages") + 1]]
    for name in args or ["sd2_768"]:
        run(name, stages)
