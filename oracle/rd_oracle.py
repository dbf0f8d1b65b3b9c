"""CPU oracle for the RollingDepth snippet-denoise hot path — TEST INFRASTRUCTURE ONLY.

This module is a from-scratch restatement (PyTorch eager fp32 on the CPU for the network
arithmetic, numpy fp32 with explicit gradients for the DepthAligner) of what the reference
computes on the path named by BASELINE.json:north_star.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it, and only as the
checker / reported CPU baseline.  The product (`rollingdepth_amd`) never imports it and fails
loudly when its HIP library is missing.

Pinning: every function is checked against golden vectors produced by running the reference
itself in the build container (`tests/golden/make_golden.py`, which imports
/root/reference via tests/golden/_refload.py) — see tests/test_oracle_golden.py.

Weights are diffusers state dicts (same keys as the reference modules), so the oracle, the
reference and the HIP path all consume one synthesised state dict
(rollingdepth_amd/weights.py).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

SD = Dict[str, torch.Tensor]

LATENT_SCALE = 0.18215  # rollingdepth_pipeline.py:53-54


# ----------------------------------------------------------------------------- primitives
def _lin(x, sd, p, bias=True):
    return F.linear(x, sd[p + ".weight"], sd.get(p + ".bias") if bias else None)


def _conv(x, sd, p, stride=1, padding=1):
    return F.conv2d(x, sd[p + ".weight"], sd.get(p + ".bias"), stride=stride, padding=padding)


def _gn(x, sd, p, groups, eps):
    return F.group_norm(x, groups, sd[p + ".weight"], sd[p + ".bias"], eps)


def _ln(x, sd, p, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


def sdpa(q, k, v, chunk=4096):
    """softmax(q kᵀ/√d) v, fp32, query-chunked.  q/k/v: [B, H, S, d].
    Restates F.scaled_dot_product_attention (attention_processor.py:2251-2253): no mask, no
    dropout, non-causal, default scale 1/√d."""
    d = q.shape[-1]
    out = torch.empty_like(q)
    for s0 in range(0, q.shape[2], chunk):
        sc = torch.matmul(q[:, :, s0:s0 + chunk], k.transpose(-1, -2)) / math.sqrt(d)
        out[:, :, s0:s0 + chunk] = torch.matmul(torch.softmax(sc, dim=-1), v)
    return out


def timestep_embedding(t: torch.Tensor, dim: int, flip_sin_to_cos=True, shift=0.0, max_period=10000):
    """Sinusoidal projection (diffusers/models/embeddings.py get_timestep_embedding, used by
    `Timesteps` :591)."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=torch.float32) / (half - shift)
    emb = t[:, None].float() * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


# ----------------------------------------------------------------------------- attention
def attention(sd: SD, p: str, x: torch.Tensor, heads: int, context: Optional[torch.Tensor] = None,
              num_view: Optional[int] = None) -> torch.Tensor:
    """Modified AttnProcessor2_0 body for a UNet transformer Attention (3-D input, no
    group_norm, no residual), attention_processor.py:2181-2276.  `num_view` folds
    "(b n) hw c -> b (n hw) c" before the projections and unfolds after to_out (:2208-2211,
    :2263-2266): cross-frame attention over all n·hw tokens of the snippet."""
    bn, hw, c = x.shape
    if num_view is not None:
        x = x.reshape(bn // num_view, num_view * hw, c)
    b = x.shape[0]
    q = _lin(x, sd, p + ".to_q", bias=False)
    ctx = x if context is None else context
    k = _lin(ctx, sd, p + ".to_k", bias=False)
    v = _lin(ctx, sd, p + ".to_v", bias=False)
    d = q.shape[-1] // heads
    q = q.view(b, -1, heads, d).transpose(1, 2)
    k = k.view(ctx.shape[0], -1, heads, d).transpose(1, 2)
    v = v.view(ctx.shape[0], -1, heads, d).transpose(1, 2)
    o = sdpa(q, k, v).transpose(1, 2).reshape(b, -1, heads * d)
    o = _lin(o, sd, p + ".to_out.0")
    if num_view is not None:
        o = o.reshape(bn, hw, c)
    return o


def vae_mid_attention(sd: SD, p: str, x: torch.Tensor, groups=32, eps=1e-6) -> torch.Tensor:
    """VAE mid-block Attention (unet_2d_blocks.py:680-697): group_norm, 1 head of d=C, biased
    q/k/v/out, residual_connection=True, rescale 1 — through AttnProcessor2_0 with
    num_view=None (4-D input path, :2200-2202, :2268-2274)."""
    b, c, h, w = x.shape
    res = x
    t = x.view(b, c, h * w).transpose(1, 2)
    t = F.group_norm(t.transpose(1, 2), groups, sd[p + ".group_norm.weight"], sd[p + ".group_norm.bias"], eps).transpose(1, 2)
    q = _lin(t, sd, p + ".to_q")[:, None]
    k = _lin(t, sd, p + ".to_k")[:, None]
    v = _lin(t, sd, p + ".to_v")[:, None]
    o = sdpa(q, k, v)[:, 0]
    o = _lin(o, sd, p + ".to_out.0")
    o = o.transpose(1, 2).reshape(b, c, h, w)
    return o + res


# ----------------------------------------------------------------------------- blocks
def resnet(sd: SD, p: str, x, temb, groups, eps):
    """ResnetBlock2D.forward, resnet.py:320-373 (time_embedding_norm='default',
    output_scale_factor=1, dropout 0)."""
    h = F.silu(_gn(x, sd, p + ".norm1", groups, eps))
    h = _conv(h, sd, p + ".conv1")
    if temb is not None:
        h = h + _lin(F.silu(temb), sd, p + ".time_emb_proj")[:, :, None, None]
    h = F.silu(_gn(h, sd, p + ".norm2", groups, eps))
    h = _conv(h, sd, p + ".conv2")
    if p + ".conv_shortcut.weight" in sd:
        x = _conv(x, sd, p + ".conv_shortcut", padding=0)
    return x + h


def transformer2d(sd: SD, p: str, x, context, heads, groups, num_view):
    """Transformer2DModel (use_linear_projection=True) + one BasicTransformerBlock,
    transformer_2d.py:327-470 and attention.py:421-548."""
    b, c, h, w = x.shape
    res = x
    t = F.group_norm(x, groups, sd[p + ".norm.weight"], sd[p + ".norm.bias"], 1e-6)
    t = t.permute(0, 2, 3, 1).reshape(b, h * w, c)
    t = _lin(t, sd, p + ".proj_in")
    q = p + ".transformer_blocks.0"
    t = attention(sd, q + ".attn1", _ln(t, sd, q + ".norm1"), heads, None, num_view) + t
    t = attention(sd, q + ".attn2", _ln(t, sd, q + ".norm2"), heads, context, num_view) + t
    n3 = _ln(t, sd, q + ".norm3")
    hs, gate = _lin(n3, sd, q + ".ff.net.0.proj").chunk(2, dim=-1)  # GEGLU, activations.py:113-123
    t = _lin(hs * F.gelu(gate), sd, q + ".ff.net.2") + t
    t = _lin(t, sd, p + ".proj_out")
    t = t.reshape(b, h, w, c).permute(0, 3, 1, 2)
    return t + res


def _heads(cfg):
    ah = cfg["attention_head_dim"]
    nh = cfg.get("num_attention_heads") or ah
    n = len(cfg["block_out_channels"])
    return list(nh) if isinstance(nh, (list, tuple)) else [nh] * n


def unet_forward(sd: SD, cfg: dict, sample: torch.Tensor, timestep: torch.Tensor,
                 context: torch.Tensor, num_view: Optional[int]) -> torch.Tensor:
    """UNet2DConditionModel.forward restricted to the SD2-family layout the path uses
    (unet_2d_condition.py:1039-1324)."""
    groups, eps = cfg["norm_num_groups"], cfg["norm_eps"]
    heads = _heads(cfg)
    chans = cfg["block_out_channels"]
    L = cfg["layers_per_block"]
    t = timestep.expand(sample.shape[0]) if timestep.dim() == 1 else timestep
    temb = timestep_embedding(t, chans[0], cfg.get("flip_sin_to_cos", True), cfg.get("freq_shift", 0))
    temb = _lin(F.silu(_lin(temb, sd, "time_embedding.linear_1")), sd, "time_embedding.linear_2")

    x = _conv(sample, sd, "conv_in")
    skips = [x]
    for i, bt in enumerate(cfg["down_block_types"]):
        for j in range(L):
            x = resnet(sd, f"down_blocks.{i}.resnets.{j}", x, temb, groups, eps)
            if bt == "CrossAttnDownBlock2D":
                x = transformer2d(sd, f"down_blocks.{i}.attentions.{j}", x, context, heads[i], groups, num_view)
            skips.append(x)
        if i < len(chans) - 1:
            x = _conv(x, sd, f"down_blocks.{i}.downsamplers.0.conv", stride=2, padding=1)
            skips.append(x)
    x = resnet(sd, "mid_block.resnets.0", x, temb, groups, eps)
    x = transformer2d(sd, "mid_block.attentions.0", x, context, heads[-1], groups, num_view)
    x = resnet(sd, "mid_block.resnets.1", x, temb, groups, eps)
    rheads = list(reversed(heads))
    for i, bt in enumerate(cfg["up_block_types"]):
        for j in range(L + 1):
            x = torch.cat([x, skips.pop()], dim=1)
            x = resnet(sd, f"up_blocks.{i}.resnets.{j}", x, temb, groups, eps)
            if bt == "CrossAttnUpBlock2D":
                x = transformer2d(sd, f"up_blocks.{i}.attentions.{j}", x, context, rheads[i], groups, num_view)
        if i < len(chans) - 1:
            size = skips[-1].shape[-2:]
            x = F.interpolate(x, size=size, mode="nearest")
            x = _conv(x, sd, f"up_blocks.{i}.upsamplers.0.conv")
    x = F.silu(_gn(x, sd, "conv_norm_out", groups, eps))
    return _conv(x, sd, "conv_out")


def vae_encode(sd: SD, cfg: dict, x: torch.Tensor) -> torch.Tensor:
    """Encoder.forward (vae.py:140-182) → quant_conv → posterior mean (rollingdepth_pipeline.py
    :687-693).  Returns the UNSCALED mean [B, latent, h, w]."""
    g, eps = cfg["norm_num_groups"], 1e-6
    chans = cfg["block_out_channels"]
    L = cfg["layers_per_block"]
    h = _conv(x, sd, "encoder.conv_in")
    for i in range(len(chans)):
        for j in range(L):
            h = resnet(sd, f"encoder.down_blocks.{i}.resnets.{j}", h, None, g, eps)
        if i < len(chans) - 1:
            h = F.pad(h, (0, 1, 0, 1))
            h = _conv(h, sd, f"encoder.down_blocks.{i}.downsamplers.0.conv", stride=2, padding=0)
    h = resnet(sd, "encoder.mid_block.resnets.0", h, None, g, eps)
    h = vae_mid_attention(sd, "encoder.mid_block.attentions.0", h, g, eps)
    h = resnet(sd, "encoder.mid_block.resnets.1", h, None, g, eps)
    h = F.silu(_gn(h, sd, "encoder.conv_norm_out", g, eps))
    h = _conv(h, sd, "encoder.conv_out")
    m = _conv(h, sd, "quant_conv", padding=0)
    return m[:, : cfg["latent_channels"]]


def vae_decode(sd: SD, cfg: dict, z: torch.Tensor) -> torch.Tensor:
    """post_quant_conv → Decoder.forward (vae.py:284-347).  Returns [B, out_ch, H, W]."""
    g, eps = cfg["norm_num_groups"], 1e-6
    chans = list(reversed(cfg["block_out_channels"]))
    L = cfg["layers_per_block"]
    z = _conv(z, sd, "post_quant_conv", padding=0)
    h = _conv(z, sd, "decoder.conv_in")
    h = resnet(sd, "decoder.mid_block.resnets.0", h, None, g, eps)
    h = vae_mid_attention(sd, "decoder.mid_block.attentions.0", h, g, eps)
    h = resnet(sd, "decoder.mid_block.resnets.1", h, None, g, eps)
    for i in range(len(chans)):
        for j in range(L + 1):
            h = resnet(sd, f"decoder.up_blocks.{i}.resnets.{j}", h, None, g, eps)
        if i < len(chans) - 1:
            h = F.interpolate(h, scale_factor=2.0, mode="nearest")
            h = _conv(h, sd, f"decoder.up_blocks.{i}.upsamplers.0.conv")
    h = F.silu(_gn(h, sd, "decoder.conv_norm_out", g, eps))
    return _conv(h, sd, "decoder.conv_out")


# ----------------------------------------------------------------------------- DDIM
class DDIM:
    """DDIMScheduler arithmetic (scheduling_ddim.py:180-230 tables, :297-340 set_timesteps,
    :342-468 step with eta=0, :471-495 add_noise)."""

    def __init__(self, cfg: dict):
        self.cfg = cfg
        T = cfg.get("num_train_timesteps", 1000)
        sched = cfg.get("beta_schedule", "scaled_linear")
        b0, b1 = cfg.get("beta_start", 0.00085), cfg.get("beta_end", 0.012)
        if sched == "scaled_linear":
            betas = torch.linspace(b0 ** 0.5, b1 ** 0.5, T, dtype=torch.float32) ** 2
        elif sched == "linear":
            betas = torch.linspace(b0, b1, T, dtype=torch.float32)
        else:
            raise NotImplementedError(sched)
        if cfg.get("rescale_betas_zero_snr", False):
            a = torch.cumprod(1.0 - betas, 0).sqrt()
            a0, aT = a[0].clone(), a[-1].clone()
            a = (a - aT) * (a0 / (a0 - aT))
            ab = a ** 2
            al = torch.cat([ab[0:1], ab[1:] / ab[:-1]])
            betas = 1 - al
        self.alphas_cumprod = torch.cumprod(1.0 - betas, 0)
        self.final_alpha_cumprod = torch.tensor(1.0) if cfg.get("set_alpha_to_one", False) else self.alphas_cumprod[0]
        self.T = T

    def set_timesteps(self, n: int) -> List[int]:
        sp = self.cfg.get("timestep_spacing", "trailing")
        T = self.T
        if sp == "trailing":
            ts = np.round(np.arange(T, 0, -T / n)).astype(np.int64) - 1
        elif sp == "leading":
            ts = (np.arange(0, n) * (T // n)).round()[::-1].astype(np.int64) + self.cfg.get("steps_offset", 0)
        elif sp == "linspace":
            ts = np.linspace(0, T - 1, n).round()[::-1].astype(np.int64)
        else:
            raise ValueError(sp)
        self.n = n
        return [int(t) for t in ts]

    def coeffs(self, t: int) -> Tuple[float, float, float, float]:
        prev = t - self.T // self.n
        a = float(self.alphas_cumprod[t])
        ap = float(self.alphas_cumprod[prev]) if prev >= 0 else float(self.final_alpha_cumprod)
        return a, 1 - a, ap, 1 - ap

    def step(self, out: torch.Tensor, t: int, x: torch.Tensor) -> torch.Tensor:
        a, b, ap, bp = self.coeffs(t)
        pt = self.cfg.get("prediction_type", "v_prediction")
        if pt == "v_prediction":
            x0 = a ** 0.5 * x - b ** 0.5 * out
            eps = a ** 0.5 * out + b ** 0.5 * x
        elif pt == "epsilon":
            x0 = (x - b ** 0.5 * out) / a ** 0.5
            eps = out
        else:
            raise NotImplementedError(pt)
        return ap ** 0.5 * x0 + bp ** 0.5 * eps

    def add_noise(self, x0, noise, t: int):
        a = float(self.alphas_cumprod[t])
        return a ** 0.5 * x0 + (1 - a) ** 0.5 * noise


# ----------------------------------------------------------------------------- snippets
def cap_max_dilation(seq_len: int, snippet_len: int, dilation: int) -> int:
    """rollingdepth_pipeline.py:504-515 (compares a gap bound with the dilation, as the
    reference does)."""
    max_gap = int(seq_len / snippet_len) - 1
    return min(max_gap, dilation) if max_gap < dilation else dilation


def snippet_indices(i_step: int, total_step: int, seq_len: int, snippet_len: int,
                    dilation_start: int, dilation_end: int, stride: int = 1) -> List[List[int]]:
    """rollingdepth_pipeline.py:465-502."""
    gs, ge = dilation_start - 1, dilation_end - 1
    assert gs >= ge and gs >= 0 and ge >= 0
    g = int((1 - i_step / total_step) * (gs - ge) + ge)
    win = (snippet_len - 1) * (g + 1) + 1
    starts = list(range(0, seq_len - win + 1, stride))
    if starts[-1] < seq_len - win:
        starts.append(seq_len - win)
    return [list(range(s, s + win, g + 1)) for s in starts]


# ----------------------------------------------------------------------------- aligner
def _f32(x):
    return np.float32(x)


def aligner_optimize(xs: Sequence[np.ndarray], idx: Sequence[np.ndarray], seq_len: int,
                     lr=1e-3, iters=2000, lmda2=0.1, lmda3=10.0, depth_w=1.0, loss_scale=1.0,
                     betas=(0.5, 0.9), eps=1e-8, history=True):
    """DepthAligner.optimize (depth_aligner.py:123-229) restated with explicit gradients.

    xs[d]:  [n_d, w_d, P] float32 subsampled, min-shifted snippets of dilation d.
    idx[d]: [n_d, w_d] frame index of (snippet, slot).
    Row layout (depth_aligner.py:179-188): slot j of dilation d is row d·w_d + j of the [Σw, N, P]
    tensors; when snippet lengths differ, rows of different dilations can coincide and the later
    dilation's value overwrites the earlier one's at the frames both cover (`alive` below: an
    overwritten slot contributes neither to the frame means, the count B, the loss nor the gradient).
    Loss = loss_scale·(mean|M−T|·B/s + w_d·mean|M_d−T_d|·B/s_d) + Σ_d λ2·mean(relu(1−s)²) + λ3·mean(t²)
    where the means run over the FULL Σw×N×P tensors (zeros included, :200-201), T/T_d are the
    detached per-frame means (:190-198), M_d = 1/clip(A, 1e-3) (:182-184), A = x·s + t.
    Adam follows torch.optim.Adam's single-tensor update order exactly (lerp with weight 0.5,
    mul+addcmul, sqrt/bc2_sqrt + eps, addcdiv) in float32.
    """
    nd = len(xs)
    P = xs[0].shape[-1]
    ws = [x.shape[1] for x in xs]
    R = sum(ws)
    rb = [d * w for d, w in enumerate(ws)]
    denom = np.float32(R * seq_len * P)
    alive = [np.ones(ix.shape, bool) for ix in idx]
    for d in range(nd):
        for j in range(ws[d]):
            r = rb[d] + j
            for d2 in range(d + 1, nd):
                j2 = r - rb[d2]
                if 0 <= j2 < ws[d2]:
                    alive[d][:, j] &= ~np.isin(idx[d][:, j], idx[d2][:, j2])
    s = [np.ones(x.shape[0], np.float32) for x in xs]
    t = [np.zeros(x.shape[0], np.float32) for x in xs]
    params = s + t
    m = [np.zeros_like(p) for p in params]
    v = [np.zeros_like(p) for p in params]
    b1, b2 = _f32(betas[0]), _f32(betas[1])
    cnt = np.zeros(seq_len, np.float32)
    for ix, al in zip(idx, alive):
        np.add.at(cnt, ix[al], 1.0)
    hist = []
    for it in range(iters):
        A = [x * s[d][:, None, None] + t[d][:, None, None] for d, x in enumerate(xs)]  # mul then add
        Ac = [np.maximum(a, _f32(1e-3)) for a in A]
        Ad = [_f32(1.0) / a for a in Ac]
        summ = np.zeros((seq_len, P), np.float32)
        summd = np.zeros((seq_len, P), np.float32)
        for r in range(R):  # row order of M (depth_aligner.py:179-190)
            for d in range(nd):
                j = r - rb[d]
                if 0 <= j < ws[d]:
                    al = alive[d][:, j]
                    summ[idx[d][al, j]] += A[d][al, j]
                    summd[idx[d][al, j]] += Ad[d][al, j]
        summ = summ / cnt[:, None]
        summd = summd / cnt[:, None]
        sc = np.abs(summ).mean(-1)
        scd = np.abs(summd).mean(-1)
        g_s, g_t = [], []
        loss1 = 0.0
        loss2 = 0.0
        for d in range(nd):
            T = summ[idx[d]]
            Td = summd[idx[d]]
            S = sc[idx[d]][..., None]
            Sd = scd[idx[d]][..., None]
            live = alive[d][..., None].astype(np.float32)
            diff = A[d] - T
            diffd = Ad[d] - Td
            loss1 += float(np.sum(np.abs(diff / S) * live, dtype=np.float64))
            loss2 += float(np.sum(np.abs(diffd / Sd) * live, dtype=np.float64))
            gA = np.sign(diff) / S * live
            gAd = np.sign(diffd) / Sd * (-(Ad[d] * Ad[d])) * (A[d] >= _f32(1e-3)) * live
            g = (gA + _f32(depth_w) * gAd) * _f32(loss_scale) / denom
            g_s.append((g * xs[d]).sum(axis=(1, 2)).astype(np.float32))
            g_t.append(g.sum(axis=(1, 2)).astype(np.float32))
        soft = 0.0
        for d in range(nd):
            r = np.maximum(_f32(0.0), _f32(1.0) - s[d])
            n = np.float32(len(s[d]))
            soft += float(lmda2 * np.mean(r * r) + lmda3 * np.mean(t[d] * t[d]))
            g_s[d] = g_s[d] + _f32(lmda2) * _f32(2.0) * r * _f32(-1.0) / n
            g_t[d] = g_t[d] + _f32(lmda3) * _f32(2.0) * t[d] / n
        if history:
            loss = loss_scale * (loss1 / float(denom) + depth_w * loss2 / float(denom)) + soft
            hist.append((loss, float(summ.min()), float(summ.max())))
        grads = g_s + g_t
        step = it + 1
        bc1 = 1 - betas[0] ** step
        bc2 = 1 - betas[1] ** step
        step_size = _f32(lr / bc1)
        bc2s = _f32(bc2 ** 0.5)
        for k, p in enumerate(params):
            g = grads[k]
            diff = g - m[k]
            m[k] = g - diff * (_f32(1.0) - (_f32(1.0) - b1))  # torch lerp, weight>=0.5 branch
            v[k] = v[k] * b2 + (_f32(1.0 - betas[1]) * g) * g
            den = np.sqrt(v[k]) / bc2s + _f32(eps)
            p -= (step_size * m[k]) / den
    return s, t, hist


def aligner_indices(seq_len: int, gap: int, window: int) -> np.ndarray:
    """DepthAligner.create_triplet_indices (depth_aligner.py:57-66)."""
    g = gap + 1
    return np.array([[i + j * g for j in range(window)] for i in range(seq_len - (window - 1) * g)], np.int64)


def aligner_run(snippets: Sequence[np.ndarray], dilations: Sequence[int], factor=10, border=2,
                **kw):
    """DepthAligner.run (depth_aligner.py:68-120) + merge_scaled_triplets (:231-262).
    snippets[d]: [n_d, w_d, 1, H, W].  Returns (merged [N,1,H,W], scales, translations, hist).
    Rows past Σ w_d in the reference's layout raise its IndexError."""
    w0 = snippets[0].shape[1]
    ws = [s.shape[1] for s in snippets]
    for i, w in enumerate(ws):
        if (i + 1) * w > sum(ws):
            raise IndexError(f"index {(i + 1) * w - 1} is out of bounds for dimension 0 with size {sum(ws)}")
    gaps = [d - 1 for d in dilations]
    seq_len = snippets[0].shape[0] + (w0 - 1) * gaps[0] + (w0 - 1)
    mn = min(float(s.min()) for s in snippets)
    dt = snippets[0].dtype
    shifted = [(s - np.asarray(mn, dtype=dt)).astype(dt) for s in snippets]
    sub = [s[:, :, :, border:-border, border:-border][..., ::factor, ::factor] for s in shifted]
    xs = [s.reshape(s.shape[0], s.shape[1], -1).astype(np.float32) for s in sub]
    idx = [aligner_indices(seq_len, g, s.shape[1]) for g, s in zip(gaps, snippets)]
    sc, tr, hist = aligner_optimize(xs, idx, seq_len, **kw)
    merged = aligner_merge(shifted, idx, sc, tr, seq_len)
    return merged, sc, tr, hist


def aligner_merge(snippets, idx, sc, tr, seq_len):
    """merge_scaled_triplets (depth_aligner.py:231-262): s·x+t in the snippet dtype, then per
    frame the mean over every covering (snippet, slot) of every dilation."""
    dt = snippets[0].dtype
    out = []
    scaled = [x * sc[d].astype(dt)[:, None, None, None, None] + tr[d].astype(dt)[:, None, None, None, None]
              for d, x in enumerate(snippets)]
    for f in range(seq_len):
        parts = [scaled[d][idx[d] == f] for d in range(len(snippets))]
        cat = np.concatenate(parts, 0).astype(np.float32)
        out.append(cat.mean(0).astype(dt))
    return np.stack(out, 0)  # [N, 1, H, W]


# ----------------------------------------------------------------------------- pipeline
def encode_frames(sd, vcfg, frames: torch.Tensor, max_bs=4) -> torch.Tensor:
    """encode_rgb (rollingdepth_pipeline.py:665-704): [N,3,H,W] → [N,4,h,w]·0.18215."""
    outs = [vae_encode(sd, vcfg, frames[i:i + max_bs]) for i in range(0, frames.shape[0], max_bs)]
    return torch.cat(outs) * LATENT_SCALE


def decode_depth(sd, vcfg, lat: torch.Tensor, max_bs=4) -> torch.Tensor:
    """decode_depth (:706-740): z/0.18215 → decoder → mean over output channels."""
    lat = lat / LATENT_SCALE
    outs = [vae_decode(sd, vcfg, lat[i:i + max_bs]) for i in range(0, lat.shape[0], max_bs)]
    return torch.cat(outs).mean(dim=1, keepdim=True)


def snippet_denoise(usd, ucfg, sched: DDIM, rgb_lat, init_noise, idx_list, context, steps=1):
    """init_snippet_infer inner loop (:415-446) for one dilation: per snippet gather, then `steps`
    UNet (rgb latent first in the 8-channel input, :650-651) + DDIM steps over the set timesteps."""
    outs = []
    for ids in idx_list:
        r = rgb_lat[ids]
        dl = init_noise[ids]
        ts = sched.set_timesteps(steps)
        for t in ts:
            x = torch.cat([r, dl], dim=1)
            pred = unet_forward(usd, ucfg, x, torch.full((len(ids),), t, dtype=torch.long), context, len(ids))
            dl = sched.step(pred, t, dl)
        outs.append(dl)
    return torch.stack(outs)  # [n_d, w, 4, h, w]


def refine(usd, ucfg, sched: DDIM, rgb_lat, depth_lat, init_noise, refine_step, snippet_len, start_dilation,
           context, skip_t_ratio=0.5):
    """RollingDepthPipeline.refine (rollingdepth_pipeline.py:517-633): add noise at the middle
    timestep, then per step every snippet (gap shrinking start_dilation → 1) is denoised from the
    OLD latents and each frame takes the mean of its snippets' predictions."""
    N = rgb_lat.shape[0]
    T = int(refine_step / skip_t_ratio)
    ts = sched.set_timesteps(T)
    ts = ts[int(len(ts) * skip_t_ratio):]
    new = sched.add_noise(depth_lat, init_noise.expand_as(depth_lat), ts[0])
    for i, t in enumerate(ts):
        idx = snippet_indices(i, len(ts), N, snippet_len, start_dilation, 1)
        old = new.clone()
        acc = torch.zeros_like(new)
        cnt = torch.zeros(N)
        for ids in idx:
            x = torch.cat([rgb_lat[ids], old[ids]], dim=1)
            pred = unet_forward(usd, ucfg, x, torch.full((len(ids),), t, dtype=torch.long), context, len(ids))
            acc[ids] += sched.step(pred, t, old[ids])
            cnt[ids] += 1
        new = acc / cnt[:, None, None, None]
    return new


def pipeline_forward(usd, ucfg, vsd, vcfg, scfg, frames: torch.Tensor, init_noise: torch.Tensor,
                     context: torch.Tensor, dilations: List[int], cap_dilation=True, snippet_len=3,
                     coalign_kwargs=None, max_vae_bs=4, record=None, refine_step=0, refine_snippet_len=3,
                     refine_start_dilation=6, init_infer_steps=(1,)):
    """RollingDepthPipeline.forward (rollingdepth_pipeline.py:193-354), stride 1.
    frames [N,3,H,W] in [-1,1]; init_noise [1,4,h,w] (broadcast to all frames, :282-288).
    snippet_len: one length or one per dilation (:215-226); init_infer_steps likewise (:227-231)."""
    N = frames.shape[0]
    dil = list(dilations)
    slens = list(snippet_len) if isinstance(snippet_len, (list, tuple)) else [snippet_len]
    if len(slens) == 1:
        slens = slens * len(dil)  # rollingdepth_pipeline.py:220-223
    steps = list(init_infer_steps)
    if len(steps) == 1:
        steps = steps * len(dil)  # rollingdepth_pipeline.py:227-231
    if cap_dilation:
        dil = [cap_max_dilation(N, sl, d) for d, sl in zip(dil, slens)]
        refine_start_dilation = cap_max_dilation(N, refine_snippet_len, refine_start_dilation)
    rgb_lat = encode_frames(vsd, vcfg, frames, max_vae_bs)
    noise = init_noise.expand(N, *init_noise.shape[1:])
    sched = DDIM(scfg)
    snippets = []
    for d, sl, ns in zip(dil, slens, steps):
        ids = snippet_indices(0, 1, N, sl, d, d)
        lat = snippet_denoise(usd, ucfg, sched, rgb_lat, noise, ids, context, ns)
        nd, w = lat.shape[:2]
        dec = decode_depth(vsd, vcfg, lat.reshape(nd * w, *lat.shape[2:]), max_vae_bs)
        snippets.append(dec.reshape(nd, w, 1, *dec.shape[-2:]))
        if record is not None:
            record.setdefault("snippet_latents", []).append(lat)
    kw = dict(coalign_kwargs or {})
    merged, sc, tr, hist = aligner_run([s.numpy() for s in snippets], dil, **kw)
    d = torch.from_numpy(merged)
    d = d - d.min()
    d = d / d.max()
    d = d * 2.0 - 1.0
    if record is not None:
        record.update(rgb_latent=rgb_lat, snippets=snippets, scales=sc, translations=tr, hist=hist,
                      dilations=dil, depth_coaligned=d)
    if refine_step > 0:
        dlat = encode_frames(vsd, vcfg, d.expand(-1, 3, -1, -1), max_vae_bs)
        new = refine(usd, ucfg, sched, rgb_lat, dlat, init_noise, refine_step, refine_snippet_len,
                     refine_start_dilation, context)
        if record is not None:
            record.update(refined_latent=new)
        d = decode_depth(vsd, vcfg, new, max_vae_bs)
    return d


# ----------------------------------------------------------------------------- colourisation
def colorize_index(depth: np.ndarray, mn, mx, n: int) -> np.ndarray:
    """Colormap table index per pixel: colorize_depth's normalisation (src/util/colorize.py:26, numpy
    arithmetic in the depth's dtype) followed by matplotlib Colormap.__call__'s float → index rule
    (x·N, x == N → N−1, truncating cast; NaN → the 'bad' entry N + 2)."""
    dt = depth.dtype
    x = ((depth - dt.type(mn)) / (dt.type(mx) - dt.type(mn))).clip(0, 1)
    x = x * dt.type(n)
    x[x == n] = n - 1
    idx = x.astype(np.int64)
    idx[np.isnan(x)] = n + 2
    return idx


def colorize_depth_multi_thread(depth: np.ndarray, valid_mask=None, color_map: str = "Spectral") -> np.ndarray:
    """src/util/colorize.py:41-93 (single-threaded restatement): [N,1,H,W] → uint8 [N,H,W,3]."""
    import matplotlib

    d = depth.squeeze(1)
    v = d if valid_mask is None else d[valid_mask.reshape(d.shape).astype(bool)]
    cm = matplotlib.colormaps[color_map]
    if not cm._isinit:
        cm._init()
    lut = (cm._lut[:, :3] * 255).astype(np.uint8)
    return lut[colorize_index(d, v.min(), v.max(), cm.N)]
