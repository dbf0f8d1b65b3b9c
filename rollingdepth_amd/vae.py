"""AutoencoderKL encoder/decoder on librdmi (NHWC f16), as the depth pipeline uses it:
`vae.encoder → quant_conv → mean ×0.18215` (rollingdepth_pipeline.py:665-704) and
`z/0.18215 → post_quant_conv → vae.decoder → mean over RGB` (:706-740).  Like the reference, the
whole frame is processed at once (no tiling: AutoencoderKL.tiled_encode/decode blend tiles and
change results).

Exact algebraic folds done once at weight-packing time:
  * encoder conv_out → quant_conv (1×1) → channel slice [:4] → ×0.18215 is one 3×3 conv
    (W' = 0.18215·Wq[:4]·W_out, b' = 0.18215·(Wq[:4]·b_out + bq[:4]));
  * decoder conv_out → mean over the 3 output channels is one 3×3 conv with the channel-averaged
    weights (mean is linear), so the decoder writes the depth map directly.
"""
from __future__ import annotations

import math
from typing import Dict

import torch

from . import kernels as K
from .config import validate_vae_config
from .unet import _Conv, _Lin, _Norm, Resnet

F16, F32 = torch.float16, torch.float32
LATENT_SCALE = 0.18215


class _FoldedConv(_Conv):
    def __init__(self, w: torch.Tensor, b: torch.Tensor, dev, stride=1, pad=1, dtype=F16):
        self.cout, self.cin, self.k, _ = w.shape
        self.cin_pad = K.pad_channels(self.cin)
        self.w = K.pack_conv(w, dev, self.cin_pad, dtype)
        self.w_up2 = None
        self.b = b.to(dev, F32)
        self.stride, self.pad = stride, pad


class VaeAttention:
    """Mid-block Attention (unet_2d_blocks.py:680-697; AttnProcessor2_0 4-D path): GroupNorm →
    fused biased QKV GEMM → f32 scores GEMM → row softmax → GEMM with Vᵀ → to_out + residual."""

    def __init__(self, sd, p, dev, groups, dtype=F16):
        self.norm = _Norm(sd, p + ".group_norm", dev)
        self.c = sd[p + ".to_q.weight"].shape[0]
        w = torch.cat([sd[f"{p}.to_{n}.weight"] for n in ("q", "k", "v")], 0)
        b = torch.cat([sd[f"{p}.to_{n}.bias"] for n in ("q", "k", "v")], 0)
        self.qkv_w = K.pack_linear(w, dev, dtype)
        self.qkv_b = b.to(dev, F32)
        self.out = _Lin(sd, p + ".to_out.0", dev, dtype=dtype)
        self.groups = groups

    def __call__(self, x):
        B, H, W, C = x.shape
        S = H * W
        t = K.groupnorm(x, self.norm.g, self.norm.b, self.groups, 1e-6, silu=False)
        qkv = K.gemm(t.view(B * S, C), self.qkv_w, C, bias=self.qkv_b).view(B, S, 3 * C)
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        o = K.attention_1head(q, k, v, 1.0 / math.sqrt(C))
        out = self.out(o.view(B * S, C), residual=x.view(B * S, C), gn=True)
        return K.gn_view(out, (B, H, W, C))


class VAE:
    def __init__(self, cfg: dict, sd: Dict[str, torch.Tensor], device, dtype=F16):
        dev = torch.device(device)
        if dtype not in (F16, F32):
            raise NotImplementedError(f"VAE storage dtype {dtype} (f16 or f32)")
        validate_vae_config(cfg)
        self.cfg, self.dev, self.dtype = cfg, dev, dtype
        g = cfg["norm_num_groups"]
        eps = 1e-6
        ch = cfg["block_out_channels"]
        L = cfg["layers_per_block"]
        lat = cfg["latent_channels"]
        self.lat = lat
        self.factor = 2 ** (len(ch) - 1)
        self.in_pad = K.pad_channels(cfg["in_channels"])
        self.lat_pad = K.pad_channels(lat)

        def R(p):
            return Resnet(sd, p, dev, g, eps, dtype=dtype)

        # encoder
        self.e_in = _Conv(sd, "encoder.conv_in", dev, dtype=dtype)
        self.e_down = []
        for i in range(len(ch)):
            res = [R(f"encoder.down_blocks.{i}.resnets.{j}") for j in range(L)]
            ds = _Conv(sd, f"encoder.down_blocks.{i}.downsamplers.0.conv", dev, stride=2, pad=0, dtype=dtype) \
                if i < len(ch) - 1 else None
            self.e_down.append((res, ds))
        self.e_mid = [R("encoder.mid_block.resnets.0"), R("encoder.mid_block.resnets.1")]
        self.e_attn = VaeAttention(sd, "encoder.mid_block.attentions.0", dev, g, dtype)
        self.e_norm = _Norm(sd, "encoder.conv_norm_out", dev)
        wq = sd["quant_conv.weight"][:lat, :, 0, 0]
        bq = sd["quant_conv.bias"][:lat]
        wo, bo = sd["encoder.conv_out.weight"], sd["encoder.conv_out.bias"]
        wf = torch.einsum("oc,cikj->oikj", wq.double(), wo.double()).float()
        bf = (wq.double() @ bo.double() + bq.double()).float()
        self.e_out = _FoldedConv(wf * LATENT_SCALE, bf * LATENT_SCALE, dev, dtype=dtype)
        # decoder
        self.post_quant = _Conv(sd, "post_quant_conv", dev, pad=0, dtype=dtype)
        self.d_in = _Conv(sd, "decoder.conv_in", dev, dtype=dtype)
        self.d_mid = [R("decoder.mid_block.resnets.0"), R("decoder.mid_block.resnets.1")]
        self.d_attn = VaeAttention(sd, "decoder.mid_block.attentions.0", dev, g, dtype)
        self.d_up = []
        for i in range(len(ch)):
            res = [R(f"decoder.up_blocks.{i}.resnets.{j}") for j in range(L + 1)]
            us = _Conv(sd, f"decoder.up_blocks.{i}.upsamplers.0.conv", dev, dtype=dtype, up2=True) \
                if i < len(ch) - 1 else None
            self.d_up.append((res, us))
        self.d_norm = _Norm(sd, "decoder.conv_norm_out", dev)
        wd, bd = sd["decoder.conv_out.weight"], sd["decoder.conv_out.bias"]
        wm = wd.double().mean(0, keepdim=True).float()  # [1, C, 3, 3]
        bm = bd.double().mean(0, keepdim=True).float()
        self.d_out = _FoldedConv(wm, bm, dev, dtype=dtype)
        # the same folded conv as the fused GroupNorm+SiLU+conv head's [tap][C] f32 weights
        self.d_w9 = wm[0].permute(1, 2, 0).reshape(9, -1).contiguous().to(dev, F32)
        self.d_b = float(bm[0])
        self.groups = g

    # ------------------------------------------------------------------ encode
    @staticmethod
    def _down(H: int, W: int):
        """Downsample2D(padding=0) output size: F.pad(0,1,0,1) then 3×3 stride 2, ⌊(H+1−3)/2⌋+1."""
        return (H - 2) // 2 + 1, (W - 2) // 2 + 1

    def latent_hw(self, H: int, W: int):
        """Latent size of an H×W frame (H/8 for multiples of 8; odd sizes round up per level)."""
        for _ in range(len(self.cfg["block_out_channels"]) - 1):
            H, W = self._down(H, W)
        return H, W

    def encode(self, x: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
        """x: NHWC f16 [B, H, W, in_pad] in [-1, 1] → scaled latent mean NHWC [B, h, w, lat_pad]
        (channels ≥ latent_channels are zero)."""
        B, H, W, _ = x.shape
        h = self.e_in(x, gn=True)
        for res, ds in self.e_down:
            for r in res:
                h = r(h)
            if ds is not None:
                # Downsample2D(padding=0): F.pad(0,1,0,1) then 3×3 s2 (downsampling.py:141-146)
                h = ds(h, pad_tl=0, out_hw=self._down(h.shape[1], h.shape[2]), gn=True)
        h = self.e_mid[0](h)
        h = self.e_attn(h)
        h = self.e_mid[1](h)
        h = K.groupnorm(h, self.e_norm.g, self.e_norm.b, self.groups, 1e-6, silu=True)
        if out is None:
            out = torch.zeros((B, h.shape[1], h.shape[2], self.lat_pad), dtype=self.dtype, device=x.device)
        self.e_out(h, out=out)
        return out

    # ------------------------------------------------------------------ decode
    def decode_depth(self, z: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
        """z: NHWC [B, h, w, lat_pad] holding latent/0.18215 (zero padded) → depth [B, H, W, 1]
        = mean over the decoder's RGB outputs, in out's dtype (f16 / f32; default the VAE's)."""
        B, hh, ww, _ = z.shape
        h = torch.zeros((B, hh, ww, self.d_in.cin_pad), dtype=self.dtype, device=z.device)
        self.post_quant(z, out=h)
        h = self.d_in(h, gn=True)
        h = self.d_mid[0](h)
        h = self.d_attn(h)
        h = self.d_mid[1](h)
        for res, us in self.d_up:
            for r in res:
                h = r(h)
            if us is not None:
                h = us(h, upsample=True, gn=True)
        # conv_norm_out → SiLU → conv_out (RGB mean folded) as one HBM pass over h (convhead.hip)
        if out is not None and not out.is_contiguous():
            if out.dtype != self.dtype:
                raise ValueError("decode_depth: a strided out must have the VAE's dtype")
            h = K.groupnorm(h, self.d_norm.g, self.d_norm.b, self.groups, 1e-6, silu=True)
            return self.d_out(h, out=out)
        return K.conv3x3_to1_gn(h, self.d_norm.g, self.d_norm.b, self.groups, 1e-6, True, self.d_w9, self.d_b,
                                out=out)
