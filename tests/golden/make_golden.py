"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Build-container only (needs /root/reference, read-only; see _refload.py).  The GPU box never
runs this; it only reads the committed .safetensors / .json outputs.

    python tests/golden/make_golden.py [--skip-sd2]

Fixtures (all inputs synthesised deterministically, rollingdepth_amd/weights.py):
  keys_sd2_unet.json / keys_sd2_vae.json    state-dict key→shape of the reference modules
  tiny_pipeline.safetensors (+ .json)       RollingDepthPipeline.forward, tiny UNet/VAE, 9 frames
                                            32², dilations [1,3] (capped by the reference), fp32
  sd2_256.safetensors (+ .json)             config 1: 3 frames 256², SD2-shaped, dil [1], fp32,
                                            cap_dilation=False, aligner 2000 it
  attn_processor.safetensors                modified AttnProcessor2_0 (num_view=3 self / cross,
                                            VAE-style 4-D group_norm+residual), fp32
  aligner.safetensors (+ .json)             DepthAligner.run on synthetic snippets, dil [1,4]
  aligner_mixed.safetensors (+ .json)       DepthAligner.run with snippet lengths [3, 2] (rows of the
                                            two dilations coincide: the reference's overwrite)
  tiny_mixed.safetensors (+ .json)          RollingDepthPipeline.forward, tiny, snippet_lengths [3, 2]
  tiny_steps2 / tiny_steps13 (+ .json)      RollingDepthPipeline.forward, tiny, init_infer_steps [2] and
                                            [1, 3] (per dilation): multi-step DDIM per snippet
  sd2_768_f32.safetensors (+ .json)         the sd2_768 run stored in f32 (paper-preset precision)
  ddim.json                                 DDIMScheduler timesteps / step / add_noise values
  snippet_indices.json                      get_snippet_indice / cap_max_dilation / aligner indices
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from safetensors.torch import save_file  # noqa: E402

import _refload  # noqa: E402
from rollingdepth_amd import config as C  # noqa: E402
from rollingdepth_amd import weights as W  # noqa: E402


def _c(t):
    return t.detach().to(torch.float32).contiguous().clone()


def build_pipe(P, ucfg, vcfg, scfg, seed=0):
    from diffusers import AutoencoderKL, DDIMScheduler, UNet2DConditionModel

    unet = UNet2DConditionModel(**ucfg)
    vae = AutoencoderKL(**vcfg)
    unet.load_state_dict(W.synth_state_dict(W.unet_param_shapes(ucfg), seed), strict=True)
    vae.load_state_dict(W.synth_state_dict(W.vae_param_shapes(vcfg), seed), strict=True)
    sched = DDIMScheduler(**scfg)
    pipe = P.RollingDepthPipeline(unet=unet, vae=vae, scheduler=sched, text_encoder=None, tokenizer=None)
    pipe.empty_text_embed = W.synth_context(ucfg["cross_attention_dim"], seed)
    return pipe


def run_pipe(pipe, frames, dilations, cap, noise_seed, coalign=None, refine_step=0, refine_start=6,
             snippet_lengths=(3,), init_infer_steps=(1,)):
    rec = {"unet_out": [], "snip_lat": []}
    orig_single = pipe.single_step
    orig_dec = pipe.decode_depth
    orig_enc = pipe.encode_rgb

    def single(**kw):
        out = orig_single(**kw)
        rec["unet_out"].append(_c(out[0]))
        return out

    def enc(x, **kw):
        out = orig_enc(x, **kw)
        rec.setdefault("rgb_latent", _c(out[0]))
        return out

    def dec(lat, **kw):
        rec["snip_lat"].append(_c(lat))
        return orig_dec(lat, **kw)

    pipe.single_step = single
    pipe.decode_depth = dec
    pipe.encode_rgb = enc
    dil = list(dilations)
    g = torch.Generator().manual_seed(noise_seed)
    with torch.no_grad():
        out = pipe.forward(
            input_frames=frames[None], dilations=dil, cap_dilation=cap, snippet_lengths=list(snippet_lengths),
            init_infer_steps=list(init_infer_steps), strides=[1], coalign_kwargs=coalign, refine_step=refine_step,
            refine_snippet_len=3, refine_start_dilation=refine_start, generator=g, verbose=False,
            max_vae_bs=4, unload_snippet=False)
    rec["dilations_used"] = dil  # forward mutates the caller's list in place (:246-252)
    return out, rec


TINY_CLIP = dict(vocab_size=30, hidden_size=96, intermediate_size=192, num_hidden_layers=2, num_attention_heads=4,
                 max_position_embeddings=77, hidden_act="gelu", layer_norm_eps=1e-5, bos_token_id=0, eos_token_id=1,
                 pad_token_id=1)
TINY_VOCAB = {"<|startoftext|>": 0, "<|endoftext|>": 1, **{c: 2 + i for i, c in enumerate("abcdefghijklmn")},
              **{c + "</w>": 16 + i for i, c in enumerate("abcdefghijklmn")}}


def attach_clip(P, pipe):
    """A transformers CLIPTokenizer + CLIPTextModel (tiny config, weights synthesised per key like the
    UNet/VAE) on the reference pipeline, so forward() runs the reference's encode_empty_text."""
    import tempfile

    from transformers import CLIPTextConfig, CLIPTextModel, CLIPTokenizer

    from rollingdepth_amd import text_encoder as TE

    d = tempfile.mkdtemp()
    json.dump(TINY_VOCAB, open(os.path.join(d, "vocab.json"), "w"))
    open(os.path.join(d, "merges.txt"), "w").write("#version: 0.2\n")
    tk = CLIPTokenizer(os.path.join(d, "vocab.json"), os.path.join(d, "merges.txt"), model_max_length=77)
    cfg = CLIPTextConfig(**TINY_CLIP)
    te = CLIPTextModel(cfg).eval()
    syn = W.synth_state_dict(TE.text_encoder_param_shapes(TINY_CLIP), 0)
    own = set(te.state_dict())
    te.load_state_dict({(k if k in own else k[len("text_model."):]): v for k, v in syn.items()}, strict=True)
    pipe.register_modules(text_encoder=te, tokenizer=tk)
    pipe.empty_text_embed = None
    return pipe


def pipeline_fixture(P, name, ucfg, vcfg, frames, dilations, cap, coalign=None, refine_step=0, refine_start=6,
                     clip=False, snippet_lengths=(3,), init_infer_steps=(1,)):
    pipe = build_pipe(P, ucfg, vcfg, C.RD_SCHEDULER)
    if clip:
        attach_clip(P, pipe)
    h, w = frames.shape[-2] // C.vae_downscale(vcfg), frames.shape[-1] // C.vae_downscale(vcfg)
    noise = torch.randn((1, 4, h, w), generator=torch.Generator().manual_seed(1))
    out, rec = run_pipe(pipe, frames, dilations, cap, 1, coalign, refine_step, refine_start, snippet_lengths,
                        init_infer_steps)
    t = {
        "frames": _c(frames), "init_noise": _c(noise), "context": _c(pipe.empty_text_embed),
        "rgb_latent": rec["rgb_latent"], "depth_pred": _c(out.depth_pred),
        "depth_coaligned": _c(out.depth_coaligned),
        "unet_out_first": rec["unet_out"][0].clone(), "unet_out_last": rec["unet_out"][-1].clone(),
    }
    if refine_step > 0:
        t["refined_latent"] = rec["snip_lat"][-1][0].clone()  # decode_depth's input after refine
    for i, (lat, sn) in enumerate(zip(rec["snip_lat"], out.snippet_ls)):
        t[f"snippet_latent_{i}"] = lat
        t[f"snippet_{i}"] = _c(sn)
    save_file(t, os.path.join(HERE, name + ".safetensors"))
    meta = {"dilations_in": list(dilations), "dilations_used": rec["dilations_used"], "cap_dilation": cap,
            "unet": ucfg, "vae": vcfg, "scheduler": C.RD_SCHEDULER, "coalign": coalign or {},
            "refine_step": refine_step, "refine_start_dilation": refine_start,
            "snippet_lengths": list(snippet_lengths), "init_infer_steps": list(init_infer_steps),
            "n_unet_calls": len(rec["unet_out"])}
    if clip:  # the context above is the reference's encode_empty_text output
        meta.update(text_encoder=TINY_CLIP, tokenizer_vocab=TINY_VOCAB, text_encoder_seed=0)
    json.dump(meta, open(os.path.join(HERE, name + ".json"), "w"), indent=1)
    print(name, {k: tuple(v.shape) for k, v in t.items()})


def _h16(t):
    return t.detach().to(torch.float16).contiguous().clone()


def compact_fixture(P, name, ucfg, vcfg, n, res, dilations, cap, depth_stride, refine_step=0, refine_start=6,
                    store=None):
    """Large-resolution fixture (768² / 1024²) kept small enough to commit: the frames are NOT
    stored (the GPU test re-synthesises them with weights.synth_frames(n, res, res, seed=0), bitwise
    the same tensor), latents are stored in f16 (the HIP path stores f16), only the first snippet of
    each dilation is stored, and depth maps are stored f16 on a [::s, ::s] pixel lattice plus the
    full-map mean / mean-|x| (size-independent checksums of the whole map).  store=_c keeps every
    stored tensor in f32 (the f32 path's fixture: f16 storage would hide its 1e-6-level error)."""
    h16 = store or _h16
    pipe = build_pipe(P, ucfg, vcfg, C.RD_SCHEDULER)
    frames = W.synth_frames(n, res, res, seed=0)
    h = w = res // C.vae_downscale(vcfg)
    noise = torch.randn((1, 4, h, w), generator=torch.Generator().manual_seed(1))
    out, rec = run_pipe(pipe, frames, dilations, cap, 1, None, refine_step, refine_start)
    s = depth_stride
    t = {
        "init_noise": _c(noise), "context": _c(pipe.empty_text_embed),
        "frames_checksum": torch.tensor([frames.double().sum().item(), frames.double().abs().sum().item()]),
        "rgb_latent": h16(rec["rgb_latent"]),
        "unet_out_first": h16(rec["unet_out"][0]), "unet_out_last": h16(rec["unet_out"][-1]),
        "depth_pred_sub": h16(out.depth_pred[..., ::s, ::s]),
        "depth_coaligned_sub": h16(out.depth_coaligned[..., ::s, ::s]),
        "depth_pred_stats": torch.tensor([out.depth_pred.double().mean().item(),
                                          out.depth_pred.double().abs().mean().item()]),
    }
    if refine_step > 0:
        t["refined_latent"] = h16(rec["snip_lat"][-1][0])
    for i, sn in enumerate(out.snippet_ls):
        t[f"snippet_latent_{i}_first"] = h16(rec["snip_lat"][i][0])
        t[f"snippet_{i}_first_sub"] = h16(sn[0, :, 0, ::s, ::s])
        t[f"snippet_{i}_stats"] = torch.tensor([sn.double().mean().item(), sn.double().abs().mean().item()])
    save_file(t, os.path.join(HERE, name + ".safetensors"))
    meta = {"n_frames": n, "res": res, "frames_seed": 0, "depth_stride": s, "dilations_in": list(dilations),
            "dilations_used": rec["dilations_used"], "cap_dilation": cap, "unet": ucfg, "vae": vcfg,
            "scheduler": C.RD_SCHEDULER, "coalign": {}, "refine_step": refine_step,
            "refine_start_dilation": refine_start, "n_unet_calls": len(rec["unet_out"]),
            "storage": "f32" if store is not None else "f16"}
    json.dump(meta, open(os.path.join(HERE, name + ".json"), "w"), indent=1)
    print(name, {k: tuple(v.shape) for k, v in t.items()}, flush=True)


def colorize_fixture():
    """src/util/colorize.py (the reference's visualisation) on random depth maps, f16 and f32, with and
    without a valid mask; output uint8 / float bytes are the golden."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("ref_colorize", "/root/reference/src/util/colorize.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    g = torch.Generator().manual_seed(11)
    out = {}
    d32 = (torch.randn(5, 1, 24, 32, generator=g) * 0.6).clamp(-1, 1)
    d32[0, 0, 0, :4] = torch.tensor([-1.0, 1.0, 0.0, 0.5])
    d16 = d32.half()
    mask = (torch.rand(5, 1, 24, 32, generator=g) > 0.2)
    for nm, d in (("f32", d32), ("f16", d16)):
        out[f"depth_{nm}"] = d.clone()
        out[f"rgb_{nm}"] = torch.from_numpy(mod.colorize_depth_multi_thread(d.numpy(), color_map="Spectral"))
        out[f"rgb_{nm}_masked"] = torch.from_numpy(
            mod.colorize_depth_multi_thread(d.numpy(), valid_mask=mask[:, 0].numpy(), color_map="Spectral"))
        dn = d.numpy()[:, 0]
        out[f"float_{nm}_Spectral_r"] = torch.from_numpy(
            mod.colorize_depth(dn, float(dn.min()) * 0.9, float(dn.max()) * 0.8, cmap="Spectral_r").copy())
    out["mask"] = mask
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "colorize.safetensors"))
    print("colorize", {k: tuple(v.shape) for k, v in out.items()})


def attn_fixture():
    from diffusers.models.attention_processor import Attention, AttnProcessor2_0

    torch.manual_seed(0)
    out = {}
    # UNet self-attention (attn1) with the num_view fold; L0-like width, reduced hw.
    a = Attention(query_dim=320, heads=5, dim_head=64, bias=False, out_bias=True)
    a.set_processor(AttnProcessor2_0())
    sd = W.synth_state_dict({k: tuple(v.shape) for k, v in a.state_dict().items()}, 7)
    a.load_state_dict(sd)
    x = torch.randn(3, 64, 320)
    with torch.no_grad():
        y = a(x, num_view=3)
        y1 = a(x)  # num_view=None: per-frame attention
    out.update({"self_x": x, "self_y_nv3": _c(y), "self_y_nv_none": _c(y1)})
    shapes = {"self": {k: list(t.shape) for k, t in sd.items()}}
    # cross-attention (attn2) against a 2-token context, num_view folded.
    c = Attention(query_dim=320, cross_attention_dim=1024, heads=5, dim_head=64, bias=False, out_bias=True)
    c.set_processor(AttnProcessor2_0())
    sdc = W.synth_state_dict({k: tuple(v.shape) for k, v in c.state_dict().items()}, 8)
    c.load_state_dict(sdc)
    ctx = torch.randn(1, 2, 1024)
    with torch.no_grad():
        yc = c(x, encoder_hidden_states=ctx, num_view=3)
    out.update({"cross_ctx": ctx, "cross_y_nv3": _c(yc)})
    shapes["cross"] = {k: list(t.shape) for k, t in sdc.items()}
    # VAE mid-block attention: group_norm, 1 head d=C, biased, residual, 4-D input.
    v = Attention(query_dim=128, heads=1, dim_head=128, rescale_output_factor=1.0, eps=1e-6,
                  norm_num_groups=32, spatial_norm_dim=None, residual_connection=True, bias=True,
                  upcast_softmax=True, _from_deprecated_attn_block=True)
    v.set_processor(AttnProcessor2_0())
    sdv = W.synth_state_dict({k: tuple(t.shape) for k, t in v.state_dict().items()}, 9)
    v.load_state_dict(sdv)
    xv = torch.randn(2, 128, 8, 8)
    with torch.no_grad():
        yv = v(xv)
    out.update({"vae_x": xv, "vae_y": _c(yv)})
    shapes["vae"] = {k: list(t.shape) for k, t in sdv.items()}
    shapes["seeds"] = {"self": 7, "cross": 8, "vae": 9}
    json.dump(shapes, open(os.path.join(HERE, "attn_processor.json"), "w"), indent=1)
    save_file({k: t.contiguous() for k, t in out.items()}, os.path.join(HERE, "attn_processor.safetensors"))
    print("attn_processor", len(out))


def aligner_fixture(A, name="aligner", lengths=(3, 3), dil=(1, 4)):
    g = torch.Generator().manual_seed(3)
    N, H, Wd = 20, 64, 64
    dil = list(dil)
    base = torch.rand((N, 1, H, Wd), generator=g) * 2 - 1
    snips = []
    for d, w in zip(dil, lengths):
        gap = d
        n = N - (w - 1) * gap
        s = torch.stack([torch.stack([base[i + j * gap] for j in range(w)]) for i in range(n)])
        sc = 0.5 + torch.rand((n, 1, 1, 1, 1), generator=g)
        sh = 0.3 * torch.randn((n, 1, 1, 1, 1), generator=g)
        snips.append((s * sc + sh + 0.01 * torch.randn(s.shape, generator=g)).float())
    al = A.DepthAligner(device=torch.device("cpu"), num_iterations=2000)
    merged, s, t, hist = al.run([x.clone() for x in snips], list(dil))
    out = {f"snippet_{i}": x for i, x in enumerate(snips)}
    out.update({"merged": _c(merged)})
    for i, (a, b) in enumerate(zip(s, t)):
        out[f"scale_{i}"] = _c(a)
        out[f"trans_{i}"] = _c(b)
    out["loss_hist"] = torch.tensor(np.array(hist, dtype=np.float64))
    save_file(out, os.path.join(HERE, name + ".safetensors"))
    json.dump({"dilations": dil, "N": N, "H": H, "W": Wd, "iterations": 2000, "snippet_lengths": list(lengths)},
              open(os.path.join(HERE, name + ".json"), "w"))
    print(name, merged.shape)


def ddim_fixture():
    from diffusers import DDIMScheduler

    s = DDIMScheduler(**C.RD_SCHEDULER)
    res = {"alphas_cumprod_0": float(s.alphas_cumprod[0]), "alphas_cumprod_999": float(s.alphas_cumprod[999]),
           "final_alpha_cumprod": float(s.final_alpha_cumprod)}
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 4, 3, 3, generator=g)
    o = torch.randn(2, 4, 3, 3, generator=g)
    for n in (1, 4, 10, 20):
        s.set_timesteps(n)
        ts = [int(t) for t in s.timesteps]
        res[f"timesteps_{n}"] = ts
        res[f"step_{n}_t0"] = s.step(o, ts[0], x).prev_sample.flatten().tolist()
        res[f"step_{n}_tlast"] = s.step(o, ts[-1], x).prev_sample.flatten().tolist()
    res["add_noise_499"] = s.add_noise(x, o, torch.tensor([499])).flatten().tolist()
    res["x"] = x.flatten().tolist()
    res["o"] = o.flatten().tolist()
    json.dump(res, open(os.path.join(HERE, "ddim.json"), "w"))
    print("ddim", list(res)[:6])


def index_fixture(P, A):
    RDP = P.RollingDepthPipeline
    res = {"cap": [], "snippets": [], "aligner": []}
    for n in (3, 6, 9, 10, 25, 100, 500):
        for d in (1, 3, 10, 25):
            res["cap"].append([n, 3, d, RDP.cap_max_dilation(n, 3, d, False)])
    for n, d in ((9, 1), (9, 2), (100, 1), (100, 25), (500, 10), (500, 25), (12, 5)):
        ts = torch.tensor([999])
        res["snippets"].append([n, d, RDP.get_snippet_indice(0, ts, n, 3, d, d, 1)])
    for i_step, T in ((0, 5), (2, 5), (4, 5)):
        ts = torch.arange(T)
        res["snippets"].append([50, [6, 1, i_step, T], RDP.get_snippet_indice(i_step, ts, 50, 3, 6, 1, 1)])
    al = A.DepthAligner(device=torch.device("cpu"))
    for n, gap in ((9, 0), (9, 1), (100, 24), (500, 9)):
        res["aligner"].append([n, gap, al.create_triplet_indices(n, gap, 3).tolist()])
    json.dump(res, open(os.path.join(HERE, "snippet_indices.json"), "w"))
    print("indices ok")


def keys_fixture():
    from diffusers import AutoencoderKL, UNet2DConditionModel

    with torch.device("meta"):
        u = UNet2DConditionModel(**C.SD2_UNET)
        v = AutoencoderKL(**C.SD2_VAE)
    json.dump({k: list(t.shape) for k, t in u.state_dict().items()}, open(os.path.join(HERE, "keys_sd2_unet.json"), "w"))
    json.dump({k: list(t.shape) for k, t in v.state_dict().items()}, open(os.path.join(HERE, "keys_sd2_vae.json"), "w"))
    print("keys ok")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-sd2", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", os.cpu_count() or 8)))
    P, A = _refload.load_reference()
    todo = a.only.split(",") if a.only else ["keys", "idx", "ddim", "attn", "aligner", "aligner_mixed", "tiny",
                                             "tiny_mixed", "refine", "clip", "colorize", "sd2", "steps"]
    if "keys" in todo:
        keys_fixture()
    if "idx" in todo:
        index_fixture(P, A)
    if "ddim" in todo:
        ddim_fixture()
    if "attn" in todo:
        attn_fixture()
    if "aligner" in todo:
        aligner_fixture(A)
    if "aligner_mixed" in todo:  # snippet lengths per dilation; rows 2 of both dilations coincide
        aligner_fixture(A, "aligner_mixed", (3, 2), (1, 3))
    if "tiny" in todo:
        frames = W.synth_frames(9, 32, 32, seed=0)
        pipeline_fixture(P, "tiny_pipeline", C.TINY_UNET, C.TINY_VAE, frames, [1, 3], True)
    if "refine" in todo:
        frames = W.synth_frames(9, 32, 32, seed=0)
        pipeline_fixture(P, "tiny_refine", C.TINY_UNET, C.TINY_VAE, frames, [1, 3], True, refine_step=2,
                         refine_start=6)
    if "tiny_mixed" in todo:  # snippet_lengths [3, 2] (rollingdepth_pipeline.py:221-226)
        frames = W.synth_frames(9, 32, 32, seed=0)
        pipeline_fixture(P, "tiny_mixed", C.TINY_UNET, C.TINY_VAE, frames, [1, 3], True, snippet_lengths=(3, 2))
    if "steps" in todo:  # init_infer_steps > 1: each snippet denoised over several DDIM steps
        # (rollingdepth_pipeline.py:421-445; scheduling_ddim.py:342-468, prev_timestep = t - T/n)
        frames = W.synth_frames(9, 32, 32, seed=0)
        pipeline_fixture(P, "tiny_steps2", C.TINY_UNET, C.TINY_VAE, frames, [1, 3], True, init_infer_steps=(2,))
        pipeline_fixture(P, "tiny_steps13", C.TINY_UNET, C.TINY_VAE, frames, [1, 3], True, init_infer_steps=(1, 3))
    if "colorize" in todo:
        colorize_fixture()
    if "clip" in todo:  # tiny pipeline whose empty-text context comes from the reference's CLIP path
        frames = W.synth_frames(9, 32, 32, seed=0)
        pipeline_fixture(P, "tiny_clip_pipeline", C.TINY_UNET, C.TINY_VAE, frames, [1, 3], True, clip=True)
    if "sd2" in todo and not a.skip_sd2:
        frames = W.synth_frames(3, 256, 256, seed=0)
        pipeline_fixture(P, "sd2_256", C.SD2_UNET, C.SD2_VAE, frames, [1], False)
    # large-resolution fixtures (opt-in: --only; tens of CPU-minutes each)
    if "sd2_768" in todo:  # fast preset arithmetic on one 3-frame 768² snippet (SURVEY §8c fixture 3)
        compact_fixture(P, "sd2_768", C.SD2_UNET, C.SD2_VAE, 3, 768, [1], False, 2)
    if "sd2_768_f32" in todo:  # the same run, stored f32: pins the f32 (paper preset) path at 768²
        compact_fixture(P, "sd2_768_f32", C.SD2_UNET, C.SD2_VAE, 3, 768, [1], False, 2, store=_c)
    if "sd2_1024" in todo:  # fast1024 preset arithmetic on one 3-frame 1024² snippet
        compact_fixture(P, "sd2_1024", C.SD2_UNET, C.SD2_VAE, 3, 1024, [1], False, 2)
    if "full1024" in todo:  # full preset: 1024², [1,10,25] capped as the reference caps, refine 10
        compact_fixture(P, "full1024", C.SD2_UNET, C.SD2_VAE, 6, 1024, [1, 10, 25], True, 4, refine_step=10,
                        refine_start=6)
    if "full1024_mix" in todo:  # full preset at 1024² on 12 frames: [1,10,25] capped to [1,3,3] by the
        # reference (max gap int(12/3)-1 = 3), so two distinct dilations are co-aligned and refined
        compact_fixture(P, "full1024_mix", C.SD2_UNET, C.SD2_VAE, 12, 1024, [1, 10, 25], True, 4, refine_step=10,
                        refine_start=6)
    if "paper256" in todo:  # paper preset semantics (fp32, cap_dilation False, refine 10) at 256², N=51
        compact_fixture(P, "paper256", C.SD2_UNET, C.SD2_VAE, 51, 256, [1, 10, 25], False, 2, refine_step=10,
                        refine_start=6)


if __name__ == "__main__":
    main()
