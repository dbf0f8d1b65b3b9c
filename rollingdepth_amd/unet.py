"""UNet2DConditionModel forward on librdmi (NHWC f16 activations, f32 accumulation).

Mirrors diffusers/models/unets/unet_2d_condition.py:1039-1324 with RollingDepth's `num_view`
threading (:1226-1301 → Transformer2DModel → BasicTransformerBlock → Attention with the
cross-frame fold, attention_processor.py:2208-2266).  Weights come from a diffusers state dict
(same keys as the reference) and are packed once at construction:
  * convs → [Cout][kh][kw][Cin_pad] f16 (implicit-GEMM K order), biases f32;
  * attn1 to_q/to_k/to_v fused into one [3C, C] projection (one GEMM, one read of the input);
  * attn2 K/V of the constant empty-text context are projected once per context
    (rollingdepth_pipeline.py:271-272,376: the context never changes);
  * GEGLU proj rows interleaved for the fused GEGLU epilogue;
  * all ResnetBlock2D.time_emb_proj rows concatenated: the time embedding of a timestep is one
    GEMM chain, cached per timestep (every 1-step snippet uses t = 999).
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional

import numpy as np
import torch

from . import kernels as K
from .config import unet_heads, validate_unet_config

F16, F32 = torch.float16, torch.float32


def _sinusoid(t: int, dim: int, flip: bool, shift: float) -> np.ndarray:
    """Timesteps projection (embeddings.py:591 / get_timestep_embedding) for one integer t —
    a constant table lookup computed once per timestep value, like a positional table."""
    half = dim // 2
    ex = -math.log(10000) * np.arange(half, dtype=np.float32) / (half - shift)
    e = np.float32(t) * np.exp(ex.astype(np.float32)).astype(np.float32)
    e = np.concatenate([np.sin(e), np.cos(e)]).astype(np.float32)
    if flip:
        e = np.concatenate([e[half:], e[:half]])
    return e


class _Lin:
    def __init__(self, sd, key, dev, bias=True, dtype=F16):
        w = sd[key + ".weight"]
        if w.dim() == 4 and tuple(w.shape[2:]) == (1, 1):
            # Transformer2DModel with use_linear_projection=False (the diffusers default): proj_in /
            # proj_out are 1×1 convs, the same per-pixel linear map on the NHWC tokens
            w = w[:, :, 0, 0]
        self.n, self.k = w.shape
        self.w = K.pack_linear(w, dev, dtype)
        self.b = sd[key + ".bias"].to(dev, F32) if bias and key + ".bias" in sd else None

    def __call__(self, x, out=None, residual=None, silu=False, gn=False):
        return K.gemm(x, self.w, self.k, out=out, bias=self.b, residual=residual, silu=silu, gn=gn)


class _Conv:
    def __init__(self, sd, key, dev, stride=1, pad=1, dtype=F16, up2=False):
        """up2: the conv of an Upsample2D — also pack the phase-decomposed weights (K.pack_conv_up2)."""
        w = sd[key + ".weight"]
        self.cout, self.cin, self.k, _ = w.shape
        self.cin_pad = K.pad_channels(self.cin)
        self.w = K.pack_conv(w, dev, self.cin_pad, dtype)
        self.w_up2 = K.pack_conv_up2(w, dev, self.cin_pad) if up2 and dtype == F16 else None
        self.b = sd[key + ".bias"].to(dev, F32) if key + ".bias" in sd else None
        self.stride, self.pad = stride, pad

    def __call__(self, x, upsample=False, residual=None, rowbias=None, out=None, pad_tl=None, out_hw=None, gn=False):
        """gn=True when a GroupNorm consumes the output (its moments come from this epilogue)."""
        return K.conv2d(x, self.w, self.cout, self.k, stride=self.stride, pad=self.pad, pad_tl=pad_tl,
                        upsample=upsample, bias=self.b, residual=residual, rowbias=rowbias, out=out, out_hw=out_hw,
                        gn=gn, w_up2=self.w_up2 if upsample else None)

    def normed(self, x, norm, groups, eps, silu=True, residual=None, rowbias=None, gn=False):
        """self(silu?(GroupNorm(x))), the norm fused into the conv's input path where supported."""
        return K.gn_conv2d(x, norm.g, norm.b, groups, eps, silu, self.w, self.cout, self.k, stride=self.stride,
                           pad=self.pad, bias=self.b, residual=residual, rowbias=rowbias, gn=gn)


class _Norm:
    def __init__(self, sd, key, dev):
        self.g = sd[key + ".weight"].to(dev, F32)
        self.b = sd[key + ".bias"].to(dev, F32)


class Resnet:
    """ResnetBlock2D (resnet.py:189, forward :320-373)."""

    def __init__(self, sd, p, dev, groups, eps, temb_slot=None, dtype=F16):
        self.n1 = _Norm(sd, p + ".norm1", dev)
        self.c1 = _Conv(sd, p + ".conv1", dev, dtype=dtype)
        self.n2 = _Norm(sd, p + ".norm2", dev)
        self.c2 = _Conv(sd, p + ".conv2", dev, dtype=dtype)
        self.sc = _Conv(sd, p + ".conv_shortcut", dev, pad=0, dtype=dtype) if p + ".conv_shortcut.weight" in sd \
            else None
        self.groups, self.eps = groups, eps
        self.temb_slot = temb_slot  # (offset, width) into the concatenated time projections

    def __call__(self, x, temb_all=None):
        rb = None
        if self.temb_slot is not None and temb_all is not None:
            o, w = self.temb_slot
            rb = temb_all[o:o + w]
        h = self.c1.normed(x, self.n1, self.groups, self.eps, rowbias=rb, gn=True)
        res = self.sc(x) if self.sc is not None else x
        return self.c2.normed(h, self.n2, self.groups, self.eps, residual=res, gn=True)


class Transformer:
    """Transformer2DModel (use_linear_projection) + BasicTransformerBlock with the modified
    cross-frame attn1 (num_view fold) and attn2 against the constant context."""

    def __init__(self, sd, p, dev, heads, groups, dtype=F16):
        self.heads, self.groups = heads, groups
        self.norm = _Norm(sd, p + ".norm", dev)
        self.proj_in = _Lin(sd, p + ".proj_in", dev, dtype=dtype)
        self.proj_out = _Lin(sd, p + ".proj_out", dev, dtype=dtype)
        q = p + ".transformer_blocks.0"
        self.ln1 = _Norm(sd, q + ".norm1", dev)
        self.ln2 = _Norm(sd, q + ".norm2", dev)
        self.ln3 = _Norm(sd, q + ".norm3", dev)
        wqkv = torch.cat([sd[f"{q}.attn1.to_{n}.weight"] for n in ("q", "k", "v")], 0)
        self.c = wqkv.shape[1]
        self.qkv = K.pack_linear(wqkv, dev, dtype)
        self.o1 = _Lin(sd, q + ".attn1.to_out.0", dev, dtype=dtype)
        self.q2 = _Lin(sd, q + ".attn2.to_q", dev, bias=False, dtype=dtype)
        self.k2 = _Lin(sd, q + ".attn2.to_k", dev, bias=False, dtype=dtype)
        self.v2 = _Lin(sd, q + ".attn2.to_v", dev, bias=False, dtype=dtype)
        self.o2 = _Lin(sd, q + ".attn2.to_out.0", dev, dtype=dtype)
        wp, bp = K.geglu_permute(sd[q + ".ff.net.0.proj.weight"], sd[q + ".ff.net.0.proj.bias"])
        self.ff1_w = K.pack_linear(wp, dev, dtype)
        self.ff1_b = bp.to(dev, F32)
        self.ff2 = _Lin(sd, q + ".ff.net.2", dev, dtype=dtype)
        self._ctx_key = None
        # f16-rounded to_q / to_out weights for the two-token attn2 fold (set_context), kept only where
        # the folded [H, C] w / u tables fit the kernel's LDS (2·H·C·4 B ≤ 64 KiB, H ≤ 16: C ≤ 640 at d = 64)
        # (f16 path only: the f32 path runs LN → q GEMM → attention → out GEMM in f32)
        self._pair = None
        self._pair_w = None
        if dtype == F16 and 2 * heads * self.c * 4 <= 64 * 1024 and heads <= 16 and \
                os.environ.get("RDMI_ATTN2_PAIR", "1") != "0":
            self._pair_w = (sd[q + ".attn2.to_q.weight"].half().float().to(dev),
                            sd[q + ".attn2.to_out.0.weight"].half().float().to(dev),
                            sd.get(q + ".attn2.to_out.0.bias", torch.zeros(self.c)).float().to(dev))

    def set_context(self, ctx16: torch.Tensor):
        """K/V of attn2 for the (constant) encoder_hidden_states [Bc, L, Dctx] f16."""
        if self._ctx_key is ctx16:
            return
        self.k2c = K.gemm(ctx16, self.k2.w, self.k2.k)
        self.v2c = K.gemm(ctx16, self.v2.w, self.v2.k)
        self._ctx_key = ctx16
        self._pair = None
        if self._pair_w is not None and self.k2c.shape[0] == 1 and self.k2c.shape[1] == 2:
            # exact fold of softmax over two keys (attention.hip attn2_pair_k): once per context
            self._pair = K.fold_attn2_pair(*self._pair_w, self.k2c[0], self.v2c[0], self.heads)

    def __call__(self, x, num_view: Optional[int]):
        B, H, W, C = x.shape
        HW = H * W
        t = K.groupnorm(x, self.norm.g, self.norm.b, self.groups, 1e-6, silu=False)
        t = self.proj_in(t.view(B * HW, C))
        # attn1: cross-frame self-attention over the snippet's n·h·w tokens
        n1 = K.layernorm(t, self.ln1.g, self.ln1.b, 1e-5)
        qkv = K.gemm(n1, self.qkv, C)
        nv = num_view or 1
        bb = B // nv
        qkv3 = qkv.view(bb, nv * HW, 3 * C)
        o = K.attention(qkv3[..., :C], qkv3[..., C:2 * C], qkv3[..., 2 * C:], self.heads)
        t = self.o1(o.view(B * HW, C), residual=t)
        # attn2: cross-attention to the context (the fold is a no-op for shared K/V)
        if self._pair is not None:  # two-token context: norm2 + attn2 + residual in one row pass
            t = K.cross_attn_pair(t, self.ln2.g, self.ln2.b, 1e-5, *self._pair)
        else:
            n2 = K.layernorm(t, self.ln2.g, self.ln2.b, 1e-5)
            q2 = self.q2(n2)
            kv_b = self.k2c.shape[0]
            if kv_b == 1:
                o2 = K.attention_smallkv(q2.view(1, B * HW, C), self.k2c, self.v2c, self.heads)
            else:
                o2 = K.attention_smallkv(q2.view(kv_b, -1, C), self.k2c, self.v2c, self.heads)
            t = self.o2(o2.view(B * HW, C), residual=t)
        # GEGLU feed-forward
        n3 = K.layernorm(t, self.ln3.g, self.ln3.b, 1e-5)
        f = K.gemm(n3, self.ff1_w, C, bias=self.ff1_b, geglu=True)
        t = self.ff2(f, residual=t)
        out = self.proj_out(t, residual=x.view(B * HW, C), gn=True)
        return K.gn_view(out, (B, H, W, C))


class UNet:
    """Native UNet2DConditionModel (SD2 family: CrossAttnDown* + Down, mid CrossAttn, Up + CrossAttnUp*)."""

    def __init__(self, cfg: dict, sd: Dict[str, torch.Tensor], device, dtype=F16):
        dev = torch.device(device)
        if dtype not in (F16, F32):
            raise NotImplementedError(f"UNet storage dtype {dtype} (f16 or f32)")
        validate_unet_config(cfg)
        self.cfg, self.dev, self.dtype = cfg, dev, dtype
        g, eps = cfg["norm_num_groups"], cfg["norm_eps"]
        heads = unet_heads(cfg)
        ch = cfg["block_out_channels"]
        L = cfg["layers_per_block"]
        self.ch, self.L = ch, L
        self.in_ch = cfg["in_channels"]
        self.out_ch = cfg["out_channels"]
        self.conv_in = _Conv(sd, "conv_in", dev, dtype=dtype)
        self.t1 = _Lin(sd, "time_embedding.linear_1", dev, dtype=dtype)
        self.t2 = _Lin(sd, "time_embedding.linear_2", dev, dtype=dtype)
        # concatenated time_emb_proj of every resnet
        tp_w, tp_b, off = [], [], 0
        slots = {}
        for k in sd:
            if k.endswith("time_emb_proj.weight"):
                p = k[: -len(".time_emb_proj.weight")]
                w = sd[k]
                tp_w.append(w)
                tp_b.append(sd[p + ".time_emb_proj.bias"])
                slots[p] = (off, w.shape[0])
                off += w.shape[0]
        self.tp_w = K.pack_linear(torch.cat(tp_w, 0), dev, dtype)
        self.tp_b = torch.cat(tp_b, 0).to(dev, F32)
        self.tp_k = tp_w[0].shape[1]
        self._temb_cache = {}

        def R(p):
            return Resnet(sd, p, dev, g, eps, slots.get(p), dtype=dtype)

        self.down = []
        for i, bt in enumerate(cfg["down_block_types"]):
            blk = {"res": [], "attn": [], "ds": None}
            for j in range(L):
                blk["res"].append(R(f"down_blocks.{i}.resnets.{j}"))
                if bt == "CrossAttnDownBlock2D":
                    blk["attn"].append(Transformer(sd, f"down_blocks.{i}.attentions.{j}", dev, heads[i], g, dtype))
            if i < len(ch) - 1:
                blk["ds"] = _Conv(sd, f"down_blocks.{i}.downsamplers.0.conv", dev, stride=2, pad=1, dtype=dtype)
            self.down.append(blk)
        self.mid_res = [R("mid_block.resnets.0"), R("mid_block.resnets.1")]
        self.mid_attn = Transformer(sd, "mid_block.attentions.0", dev, heads[-1], g, dtype)
        rheads = list(reversed(heads))
        self.up = []
        for i, bt in enumerate(cfg["up_block_types"]):
            blk = {"res": [], "attn": [], "us": None}
            for j in range(L + 1):
                blk["res"].append(R(f"up_blocks.{i}.resnets.{j}"))
                if bt == "CrossAttnUpBlock2D":
                    blk["attn"].append(Transformer(sd, f"up_blocks.{i}.attentions.{j}", dev, rheads[i], g, dtype))
            if i < len(ch) - 1:
                blk["us"] = _Conv(sd, f"up_blocks.{i}.upsamplers.0.conv", dev, dtype=dtype, up2=True)
            self.up.append(blk)
        self.norm_out = _Norm(sd, "conv_norm_out", dev)
        self.conv_out = _Conv(sd, "conv_out", dev, dtype=dtype)
        self.groups, self.eps = g, eps
        self.transformers = [t for b in self.down for t in b["attn"]] + [self.mid_attn] + \
                            [t for b in self.up for t in b["attn"]]

    # ------------------------------------------------------------------ time embedding
    def time_embedding(self, t: int) -> torch.Tensor:
        """silu(TimestepEmbedding(Timesteps(t))) projected through every resnet's time_emb_proj
        (resnet.py:338-343), cached per timestep value; [Σ Cout] f32 on device."""
        e = self._temb_cache.get(int(t))
        if e is not None:
            return e
        s = _sinusoid(int(t), self.ch[0], self.cfg.get("flip_sin_to_cos", True), self.cfg.get("freq_shift", 0))
        x = torch.from_numpy(s).to(self.dev, self.dtype).view(1, -1)
        h = K.gemm(x, self.t1.w, self.t1.k, bias=self.t1.b, silu=True)
        emb = K.gemm(h, self.t2.w, self.t2.k, bias=self.t2.b, silu=True)  # silu(temb) feeds every proj
        proj = K.gemm(emb, self.tp_w, self.tp_k, bias=self.tp_b, out_f32=True)
        e = proj.view(-1)
        self._temb_cache[int(t)] = e
        return e

    def set_context(self, ctx16: torch.Tensor):
        for tr in self.transformers:
            tr.set_context(ctx16)

    # ------------------------------------------------------------------ forward
    def forward(self, sample: torch.Tensor, t: int, num_view: Optional[int]) -> torch.Tensor:
        """sample: NHWC f16 [B, h, w, in_ch_pad]; one timestep value for the whole batch (the
        pipeline repeats a scalar t, rollingdepth_pipeline.py:434).  Returns NHWC [B, h, w, out]."""
        B, h, w, _ = sample.shape
        temb = self.time_embedding(t)
        x = self.conv_in(sample, gn=True)
        skips = [x]
        for blk in self.down:
            for j, r in enumerate(blk["res"]):
                x = r(x, temb)
                if blk["attn"]:
                    x = blk["attn"][j](x, num_view)
                skips.append(x)
            if blk["ds"] is not None:
                x = blk["ds"](x, gn=True)
                skips.append(x)
        x = self.mid_res[0](x, temb)
        x = self.mid_attn(x, num_view)
        x = self.mid_res[1](x, temb)
        for blk in self.up:
            for j, r in enumerate(blk["res"]):
                x = K.concat_channels(x, skips.pop())
                x = r(x, temb)
                if blk["attn"]:
                    x = blk["attn"][j](x, num_view)
            if blk["us"] is not None:
                # forward_upsample_size (unet_2d_condition.py): a latent that is not a multiple of
                # 2^levels upsamples to the next skip's size, not ×2 (Upsample2D with output_size)
                size = tuple(skips[-1].shape[1:3])
                if size == (2 * x.shape[1], 2 * x.shape[2]):
                    x = blk["us"](x, upsample=True, gn=True)
                else:
                    x = blk["us"](K.resize_nearest(x, size), gn=True)
        x = K.groupnorm(x, self.norm_out.g, self.norm_out.b, self.groups, self.eps, silu=True)
        return self.conv_out(x)
