"""Drop-in diffusers attention processor running the modified (RollingDepth) AttnProcessor2_0
semantics on librdmi — diffusers/models/attention_processor.py:2172-2276.

Install into any diffusers UNet / VAE the reference builds:
    unet.set_attn_processor(CrossFrameAttnProcessor())        # unet_2d_condition.py:721-753
It keeps the exact processor signature, including the `num_view` parameter: `Attention.forward`
drops every kwarg the processor's __call__ does not declare (:483-492), so a processor without
`num_view` silently degrades to per-frame attention.

Semantics (b = batch of snippets, n = num_view frames per snippet):
  fold "(b n) hw c -> b (n hw) c" (:2208-2211) → [group_norm] → to_q/to_k/to_v → per-head
  softmax(q kᵀ/√d) v over all n·hw tokens of the snippet (cross-frame) → to_out[0] (+bias)
  → unfold (:2263-2266) → 4-D restore → (+ residual) / rescale_output_factor.
The reference supports only b = 1 per call (the cross-attention residual add
fails for b > 1); this processor is correct for any b.

Compute follows the input dtype: f32 inputs (the paper preset, run_video.py:444-449) run librdmi's
f32 kernels (f32-input MFMA, exact f32 products); f16 / bf16 inputs run the f16 kernels with f32
accumulation.  Layout changes of the 4-D (VAE) form and its residual add are librdmi transposes and
the output GEMM's residual epilogue; PyTorch only allocates.
"""
from __future__ import annotations

import math
import weakref
from typing import Optional

import torch

from . import kernels as K

F16, F32 = torch.float16, torch.float32


class _Packed:
    def __init__(self, attn, dev, dtype):
        def lin(m):
            w = m.weight.detach().float().cpu()
            b = m.bias.detach().float().to(dev) if m.bias is not None else None
            return K.pack_linear(w, dev, dtype), w.shape[1], b

        self.q = lin(attn.to_q)
        self.k = lin(attn.to_k)
        self.v = lin(attn.to_v)
        self.o = lin(attn.to_out[0])
        self.self_qkv = None
        if attn.to_k.weight.shape[1] == attn.to_q.weight.shape[1]:
            ws = [attn.to_q, attn.to_k, attn.to_v]
            w = torch.cat([m.weight.detach().float().cpu() for m in ws], 0)
            bs = [m.bias for m in ws]
            b = None
            if all(x is not None for x in bs):
                b = torch.cat([x.detach().float() for x in bs]).to(dev)
            self.self_qkv = (K.pack_linear(w, dev, dtype), w.shape[1], b)
        gn = attn.group_norm
        self.gn = None
        if gn is not None:
            self.gn = (gn.weight.detach().float().to(dev), gn.bias.detach().float().to(dev), gn.num_groups, gn.eps)


class CrossFrameAttnProcessor:
    """Modified AttnProcessor2_0 on MI355X (see module docstring)."""

    def __init__(self):
        self._cache = weakref.WeakKeyDictionary()

    def _packed(self, attn, dev, dtype) -> _Packed:
        per = self._cache.get(attn)
        if per is None:
            per = {}
            self._cache[attn] = per
        p = per.get(dtype)
        if p is None:
            p = _Packed(attn, dev, dtype)
            per[dtype] = p
        return p

    def __call__(self, attn, hidden_states: torch.Tensor, encoder_hidden_states: Optional[torch.Tensor] = None,
                 attention_mask: Optional[torch.Tensor] = None, temb: Optional[torch.Tensor] = None,
                 num_view: int = None, *args, **kwargs) -> torch.Tensor:
        if attention_mask is not None:
            raise NotImplementedError("attention_mask is not used on the RollingDepth path")
        if getattr(attn, "spatial_norm", None) is not None or getattr(attn, "norm_q", None) is not None \
                or getattr(attn, "norm_k", None) is not None or getattr(attn, "norm_cross", None):
            raise NotImplementedError("spatial_norm / qk-norm / norm_cross are not used on the RollingDepth path")
        in_dtype = hidden_states.dtype
        cdt = F32 if in_dtype == F32 else F16
        dev = hidden_states.device
        p = self._packed(attn, dev, cdt)
        residual = hidden_states
        x = hidden_states.to(cdt)
        input_ndim = x.dim()
        if input_ndim == 4:  # [b, c, h, w] → token-major [b, hw, c]
            bsz, channel, height, width = x.shape
            x = K.transpose(x.reshape(bsz, channel, height * width))
        x = x.contiguous()
        if num_view is not None:  # "(b n) hw c -> b (n hw) c"
            x = x.view(x.shape[0] // num_view, num_view * x.shape[1], x.shape[2])
        B, S, C = x.shape
        if p.gn is not None:
            g, b, ng, eps = p.gn
            x = K.groupnorm(x, g, b, ng, eps, silu=False)
        H = attn.heads
        flat = x.view(B * S, C)
        if encoder_hidden_states is None and p.self_qkv is not None:
            wq, kq, bq = p.self_qkv
            qkv = K.gemm(flat, wq, kq, bias=bq).view(B, S, -1)
            inner = qkv.shape[-1] // 3
            q, k, v = qkv[..., :inner], qkv[..., inner:2 * inner], qkv[..., 2 * inner:]
        else:
            ctx = x if encoder_hidden_states is None else encoder_hidden_states.to(dev, cdt).contiguous()
            q = K.gemm(flat, p.q[0], p.q[1], bias=p.q[2]).view(B, S, -1)
            cb, L, cd = ctx.shape
            k = K.gemm(ctx.view(cb * L, cd), p.k[0], p.k[1], bias=p.k[2]).view(cb, L, -1)
            v = K.gemm(ctx.view(cb * L, cd), p.v[0], p.v[1], bias=p.v[2]).view(cb, L, -1)
            if cb != B and cb != 1:
                raise ValueError(f"context batch {cb} incompatible with query batch {B}")
        inner = q.shape[-1]
        D = inner // H
        if D == 64 and k.shape[1] <= 16 and encoder_hidden_states is not None:
            o = K.attention_smallkv(q, k, v, H)
        elif D == 64:
            if k.shape[0] != B:
                k, v = k.expand(B, -1, -1), v.expand(B, -1, -1)
            o = K.attention(q, k, v, H)
        else:
            if H != 1:
                raise NotImplementedError(f"head_dim {D} with {H} heads")
            kk = k if k.shape[0] == B else k.expand(B, -1, -1).contiguous()
            vv = v if v.shape[0] == B else v.expand(B, -1, -1).contiguous()
            o = K.attention_1head(q, kk, vv, 1.0 / math.sqrt(D))
        res_tok = None
        if attn.residual_connection:  # the residual enters the output GEMM's epilogue, token-major
            if input_ndim == 4:
                res_tok = K.transpose(residual.to(cdt).reshape(bsz, channel, height * width)).view(B * S, C)
            else:
                res_tok = residual.to(cdt).reshape(B * S, C).contiguous()
        out = K.gemm(o.reshape(B * S, inner), p.o[0], p.o[1], bias=p.o[2], residual=res_tok)
        if num_view is not None:  # "b (n hw) c -> (b n) hw c"
            out = out.view(B * num_view, S // num_view, C)
        else:
            out = out.view(B, S, C)
        if input_ndim == 4:  # token-major → [b, c, h, w]
            out = K.transpose(out).view(bsz, channel, height, width)
        out = out.to(in_dtype)
        if attn.rescale_output_factor != 1.0:
            out = out / attn.rescale_output_factor
        return out
