"""Parameter inventory (diffusers state-dict keys) and deterministic weight synthesis.

No checkpoint exists in the image, so every parity run and the benchmark use weights
synthesised per key: w = N(0,1)·1/√fan_in for conv/linear weights, 1 + 0.1·N(0,1) for norm
scales, 0.02·N(0,1) for biases, drawn from a CPU torch.Generator seeded by crc32(key) ^ seed.
The generator is deterministic for a given torch build, so the fixture tool (reference modules,
build container) and the GPU box (same image) see bit-identical weights without committing
the 866 M-parameter SD2 state dict.  The key sets are checked against the reference modules'
own state dicts (tests/golden/*_keys.json, written by make_golden.py).
"""
from __future__ import annotations

import math
import zlib
from collections import OrderedDict
from typing import Dict, Tuple

import torch

from .config import unet_heads

Shapes = "OrderedDict[str, Tuple[int, ...]]"


def _conv(d, p, cin, cout, k=3, bias=True):
    d[p + ".weight"] = (cout, cin, k, k)
    if bias:
        d[p + ".bias"] = (cout,)


def _lin(d, p, cin, cout, bias=True):
    d[p + ".weight"] = (cout, cin)
    if bias:
        d[p + ".bias"] = (cout,)


def _norm(d, p, c):
    d[p + ".weight"] = (c,)
    d[p + ".bias"] = (c,)


def _resnet(d, p, cin, cout, temb):
    _norm(d, p + ".norm1", cin)
    _conv(d, p + ".conv1", cin, cout)
    if temb:
        _lin(d, p + ".time_emb_proj", temb, cout)
    _norm(d, p + ".norm2", cout)
    _conv(d, p + ".conv2", cout, cout)
    if cin != cout:
        _conv(d, p + ".conv_shortcut", cin, cout, k=1)


def _transformer(d, p, c, ctx):
    _norm(d, p + ".norm", c)
    _lin(d, p + ".proj_in", c, c)
    q = p + ".transformer_blocks.0"
    _norm(d, q + ".norm1", c)
    for n in ("q", "k", "v"):
        _lin(d, f"{q}.attn1.to_{n}", c, c, bias=False)
    _lin(d, q + ".attn1.to_out.0", c, c)
    _norm(d, q + ".norm2", c)
    _lin(d, q + ".attn2.to_q", c, c, bias=False)
    _lin(d, q + ".attn2.to_k", ctx, c, bias=False)
    _lin(d, q + ".attn2.to_v", ctx, c, bias=False)
    _lin(d, q + ".attn2.to_out.0", c, c)
    _norm(d, q + ".norm3", c)
    _lin(d, q + ".ff.net.0.proj", c, 8 * c)
    _lin(d, q + ".ff.net.2", 4 * c, c)
    _lin(d, p + ".proj_out", c, c)


def unet_param_shapes(cfg) -> Shapes:
    """Key → shape of UNet2DConditionModel's state dict for the SD2-family layout
    (unet_2d_condition.py:71, unet_2d_blocks.py CrossAttnDown/Down/Mid/Up/CrossAttnUp)."""
    d: Dict = OrderedDict()
    ch = cfg["block_out_channels"]
    L = cfg["layers_per_block"]
    ctx = cfg["cross_attention_dim"]
    temb = ch[0] * 4
    _conv(d, "conv_in", cfg["in_channels"], ch[0])
    _lin(d, "time_embedding.linear_1", ch[0], temb)
    _lin(d, "time_embedding.linear_2", temb, temb)
    cin = ch[0]
    for i, bt in enumerate(cfg["down_block_types"]):
        cout = ch[i]
        for j in range(L):
            _resnet(d, f"down_blocks.{i}.resnets.{j}", cin if j == 0 else cout, cout, temb)
            if bt == "CrossAttnDownBlock2D":
                _transformer(d, f"down_blocks.{i}.attentions.{j}", cout, ctx)
        if i < len(ch) - 1:
            _conv(d, f"down_blocks.{i}.downsamplers.0.conv", cout, cout)
        cin = cout
    rch = list(reversed(ch))
    for i, bt in enumerate(cfg["up_block_types"]):
        prev = rch[i - 1] if i > 0 else rch[0]
        out = rch[i]
        inp = rch[min(i + 1, len(ch) - 1)]
        for j in range(L + 1):
            skip = inp if j == L else out
            rin = prev if j == 0 else out
            _resnet(d, f"up_blocks.{i}.resnets.{j}", rin + skip, out, temb)
            if bt == "CrossAttnUpBlock2D":
                _transformer(d, f"up_blocks.{i}.attentions.{j}", out, ctx)
        if i < len(ch) - 1:
            _conv(d, f"up_blocks.{i}.upsamplers.0.conv", out, out)
    _resnet(d, "mid_block.resnets.0", ch[-1], ch[-1], temb)
    _transformer(d, "mid_block.attentions.0", ch[-1], ctx)
    _resnet(d, "mid_block.resnets.1", ch[-1], ch[-1], temb)
    _norm(d, "conv_norm_out", ch[0])
    _conv(d, "conv_out", ch[0], cfg["out_channels"])
    return d


def _vae_attn(d, p, c):
    _norm(d, p + ".group_norm", c)
    for n in ("q", "k", "v"):
        _lin(d, f"{p}.to_{n}", c, c)
    _lin(d, p + ".to_out.0", c, c)


def vae_param_shapes(cfg) -> Shapes:
    """Key → shape of AutoencoderKL's state dict (autoencoder_kl.py:36, vae.py:47/185)."""
    d: Dict = OrderedDict()
    ch = cfg["block_out_channels"]
    L = cfg["layers_per_block"]
    lat = cfg["latent_channels"]
    _conv(d, "encoder.conv_in", cfg["in_channels"], ch[0])
    cin = ch[0]
    for i, cout in enumerate(ch):
        for j in range(L):
            _resnet(d, f"encoder.down_blocks.{i}.resnets.{j}", cin if j == 0 else cout, cout, 0)
        if i < len(ch) - 1:
            _conv(d, f"encoder.down_blocks.{i}.downsamplers.0.conv", cout, cout)
        cin = cout
    _resnet(d, "encoder.mid_block.resnets.0", ch[-1], ch[-1], 0)
    _vae_attn(d, "encoder.mid_block.attentions.0", ch[-1])
    _resnet(d, "encoder.mid_block.resnets.1", ch[-1], ch[-1], 0)
    _norm(d, "encoder.conv_norm_out", ch[-1])
    _conv(d, "encoder.conv_out", ch[-1], 2 * lat)
    _conv(d, "decoder.conv_in", lat, ch[-1])
    _resnet(d, "decoder.mid_block.resnets.0", ch[-1], ch[-1], 0)
    _vae_attn(d, "decoder.mid_block.attentions.0", ch[-1])
    _resnet(d, "decoder.mid_block.resnets.1", ch[-1], ch[-1], 0)
    rch = list(reversed(ch))
    prev = rch[0]
    for i, cout in enumerate(rch):
        for j in range(L + 1):
            _resnet(d, f"decoder.up_blocks.{i}.resnets.{j}", prev if j == 0 else cout, cout, 0)
        if i < len(ch) - 1:
            _conv(d, f"decoder.up_blocks.{i}.upsamplers.0.conv", cout, cout)
        prev = cout
    _norm(d, "decoder.conv_norm_out", ch[0])
    _conv(d, "decoder.conv_out", ch[0], cfg["out_channels"])
    _conv(d, "quant_conv", 2 * lat, 2 * lat, k=1)
    _conv(d, "post_quant_conv", lat, lat, k=1)
    return d


def _is_norm(key: str) -> bool:
    leaf = key.rsplit(".", 2)[-2]
    return "norm" in leaf


def synth_tensor(key: str, shape, seed: int = 0) -> torch.Tensor:
    g = torch.Generator().manual_seed((zlib.crc32(key.encode()) ^ (seed * 0x9E3779B1)) & 0x7FFFFFFF)
    x = torch.randn(shape, generator=g, dtype=torch.float32)
    if key.endswith(".bias"):
        return x * 0.02
    if len(shape) == 1 and _is_norm(key):
        return 1.0 + 0.1 * x
    fan_in = int(math.prod(shape[1:]))
    return x / math.sqrt(fan_in)


def synth_state_dict(shapes: Shapes, seed: int = 0) -> Dict[str, torch.Tensor]:
    return OrderedDict((k, synth_tensor(k, s, seed)) for k, s in shapes.items())


def synth_context(cross_dim: int, seed: int = 0, tokens: int = 2) -> torch.Tensor:
    """Stand-in for the empty-prompt CLIP embedding [1, 2, cross_dim]
    (encode_empty_text, rollingdepth_pipeline.py:178-191; BOS+EOS tokens)."""
    g = torch.Generator().manual_seed(1234 + seed)
    return torch.randn((1, tokens, cross_dim), generator=g, dtype=torch.float32)


def synth_frames(n: int, h: int, w: int, seed: int = 0, first: int = 0, count: int = None) -> torch.Tensor:
    """Synthetic video [n,3,h,w] in [-1,1]: smooth moving sinusoids + noise,
    clipped to [0,1] then mapped as video_io.py:123.  `first`/`count` return frames
    [first, first+count) of the same n-frame video (per-frame noise streams), so a rank can
    materialise only its own chunk."""
    count = n - first if count is None else count
    u = torch.arange(w, dtype=torch.float32)[None, None, :] / w
    v = torch.arange(h, dtype=torch.float32)[None, :, None] / h
    f = torch.tensor([1.3, 2.1, 0.7], dtype=torch.float32)[:, None, None]
    out = torch.empty((count, 3, h, w), dtype=torch.float32)
    for i in range(count):
        k = (first + i) / max(n, 1)
        x = 0.5 + 0.35 * torch.sin(2 * math.pi * (u * f + v * (3.0 - f) + k * 1.5 + f))
        g = torch.Generator().manual_seed(seed * 1000003 + first + i)
        x = x + 0.05 * torch.randn((3, h, w), generator=g)
        out[i] = x.clamp(0, 1) * 2.0 - 1.0
    return out


def synth_noise(h: int, w: int, seed: int = 1, c: int = 4) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randn((1, c, h, w), generator=g, dtype=torch.float32)
