"""Torch-tensor front end of librdmi: argument validation, output allocation (PyTorch caching
allocator owns every buffer) and the current HIP stream.  No arithmetic happens here."""
from __future__ import annotations

import ctypes as C
import math
import os
from typing import Optional, Sequence, Tuple

import torch

from . import _native as _N
from ._native import check, lib

F16 = torch.float16
F32 = torch.float32


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


# ----------------------------------------------------------------------------- live kernel timing
# bench.py brackets the hot kernels with HIP events on the launch stream (no host sync inside the
# timed region) to compute per-kernel achieved TFLOP/s.
_PROF = None


def profile_start():
    global _PROF
    _PROF = {}


def profile_stop():
    global _PROF
    prof, _PROF = _PROF, None
    if not prof:
        return {}
    torch.cuda.synchronize()
    out = {}
    for name, recs in prof.items():
        ms = sum(a.elapsed_time(b) for a, b, _, _ in recs)
        out[name] = {"ms": ms, "flop": float(sum(r[2] for r in recs)), "bytes": float(sum(r[3] for r in recs)),
                     "n": len(recs)}
    return out


_PROF_SHAPES = os.environ.get("RDMI_PROF_SHAPES") == "1"  # key the timings by launch shape too
# RDMI_PROF_SEQ=path (diagnostics, tools/traffic_split.py): every timed launch's (family, shape, FLOPs,
# algorithmic bytes) in launch order, written to `path` at exit — matched 1:1 against the dispatches of a
# rocprofv3 --pmc pass of the same process to split the fabric traffic per kernel and shape.
_PROF_SEQ_PATH = os.environ.get("RDMI_PROF_SEQ")
_PROF_SEQ = [] if _PROF_SEQ_PATH else None
if _PROF_SEQ_PATH:
    import atexit
    import json as _json

    atexit.register(lambda: _json.dump(_PROF_SEQ, open(_PROF_SEQ_PATH, "w")))


class _Timed:
    """nbytes: the launch's algorithmic HBM bytes (every operand read once, the output written once)."""
    __slots__ = ("name", "flop", "nbytes", "ev")

    def __init__(self, name, flop, shape=None, nbytes=0):
        self.name, self.flop, self.nbytes, self.ev = name, flop, nbytes, None
        if _PROF_SEQ is not None:
            _PROF_SEQ.append((name, shape, flop, nbytes))
        if _PROF_SHAPES and shape is not None:
            self.name = f"{name} {shape}"

    def __enter__(self):
        if _PROF is not None:
            self.ev = torch.cuda.Event(enable_timing=True)
            self.ev.record()
        return self

    def __exit__(self, *exc):
        if _PROF is not None and self.ev is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            _PROF.setdefault(self.name, []).append((self.ev, e, self.flop, self.nbytes))


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _need(t: torch.Tensor, dtype, name: str):
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a device tensor, got {t.device}")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")


def _need_act(t: torch.Tensor, name: str):
    """An activation of either storage dtype (f16 path, or the paper preset's f32 path)."""
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a device tensor, got {t.device}")
    if t.dtype not in (F16, F32):
        raise TypeError(f"{name}: expected f16 or f32, got {t.dtype}")


# ----------------------------------------------------------------------------- weight packing
BF16 = torch.bfloat16


def _f32_x3_mode() -> str:
    m = os.environ.get("RDMI_F32_X3", "conv")
    if m not in ("0", "1", "conv", "6"):
        raise ValueError(f"RDMI_F32_X3={m!r}: 0 (exact f32 products everywhere), conv (default: bf16-split "
                         f"products in the convolutions only), 1 (bf16-split products everywhere) or 6 "
                         f"(f32-equivalent three-way bf16 split everywhere)")
    return m


def f32_x3(kind: str = "conv") -> bool:
    """Whether the f32 path runs `kind` ("conv" | "linear" — Linear layers and the cross-frame
    attention) on the bf16-split engine (RDMI_F32_X3, rdmi.h): f32 activations and accumulation,
    three bf16 MFMA products per multiply-add (≈2^-16 relative per product, 2.2× the exact engine's
    speed on the paper preset's shapes: profiles/r03f_x3_probe.log).  Read when the weights are packed,
    and by attention() at each call for its own products.
    The default (RDMI_F32_X3=conv, round 5) follows the reference's fp32 preset precision layer by
    layer: its convolutions run through cuDNN under PyTorch's default allow_tf32 (run_video.py sets no
    precision flag), 2^-11 products on its Ampere+ GPUs — bf16x3 (2^-16) is finer — while its Linear
    layers (matmul: allow_tf32 off by default) and SDPA are exact f32, and so are ours (the exact-f32
    engines, v_mfma_f32_16x16x4_f32).  RDMI_F32_X3=1: bf16x3 everywhere (the round-3/4 default, a
    labelled faster variant); RDMI_F32_X3=0: exact f32 products everywhere."""
    m = _f32_x3_mode()
    return m == "1" or (m == "conv" and kind == "conv")


def f32_x6() -> bool:
    """Whether the f32 path's Linear layers and cross-frame attention (with RDMI_F32_X3=conv) run their
    products on the three-way bf16 split (RDMI_F32_X6, rdmi.h: six bf16 MFMA products per f32
    multiply-add, a few 2^-24 per product — f32's own product rounding) instead of the exact
    f32-input MFMA: the same precision class at ≈2× the speed.  RDMI_F32_X6=0 keeps the exact engine.
    Read when weights are packed, and per attention call."""
    m = _f32_x3_mode()
    return m == "6" or (m == "conv" and os.environ.get("RDMI_F32_X6", "1") != "0")


def _f32_parts(kind: str) -> int:
    """bf16 parts per f32 operand for `kind` ("conv" | "linear"): 1 exact f32, 2 bf16x3, 3 bf16x6."""
    if f32_x3(kind):
        return 2
    if _f32_x3_mode() == "6":
        return 3
    return 3 if kind == "linear" and f32_x6() else 1


def f32_precision_label() -> str:
    """The f32 path's product precision, for bench lines."""
    m = _f32_x3_mode()
    if m == "conv":
        return "bf16x3 conv products, " + \
            ("f32-equivalent bf16x6 Linear/attention products" if f32_x6() else "exact f32 Linear/attention")
    return {"0": "exact f32 products", "1": "bf16x3 products",
            "6": "f32-equivalent bf16x6 products everywhere"}[m]


def split_bf16(w: torch.Tensor) -> torch.Tensor:
    """f32 [N, Kp] (Kp % 32 == 0) → bf16 [N, 2·Kp]: per 32-deep K-tile, bf16(w) then bf16(w − bf16(w))
    (both round-to-nearest-even; the RDMI_F32_X3 weight layout of rdmi.h)."""
    n, kp = w.shape
    if kp % 32:
        raise ValueError(f"split_bf16: K {kp} not a multiple of 32")
    hi = w.to(BF16)
    lo = (w - hi.float()).to(BF16)
    return torch.stack((hi.view(n, kp // 32, 32), lo.view(n, kp // 32, 32)), 2).reshape(n, 2 * kp).contiguous()


def split3_bf16(w: torch.Tensor) -> torch.Tensor:
    """f32 [N, Kp] (Kp % 32 == 0) → bf16 [N, 4·Kp]: per 32-deep K-tile, bf16 hi, mid, lo parts then 32
    zeros (each remainder exact in f32, each part round-to-nearest-even; the RDMI_F32_X6 weight layout
    of rdmi.h, 256 B per row and K-tile).  The result carries `_rdmi_parts = 3`."""
    n, kp = w.shape
    if kp % 32:
        raise ValueError(f"split3_bf16: K {kp} not a multiple of 32")
    hi = w.to(BF16)
    r = w - hi.float()
    mid = r.to(BF16)
    lo = (r - mid.float()).to(BF16)
    z = torch.zeros_like(hi)
    out = torch.stack([t.view(n, kp // 32, 32) for t in (hi, mid, lo, z)], 2).reshape(n, 4 * kp).contiguous()
    out._rdmi_parts = 3
    return out


def _split_f32_weights(out: torch.Tensor, parts: int) -> torch.Tensor:
    if parts == 2:
        return split_bf16(out)
    if parts == 3:
        return split3_bf16(out)
    return out


def pack_linear(w: torch.Tensor, device, dtype=F16) -> torch.Tensor:
    """[N, K] → [N, Kp] in the storage dtype (K zero-padded to a multiple of 32); f32 with bf16-split
    products for Linear layers (_f32_parts("linear")): split_bf16 ([N, 2·Kp] bf16) or split3_bf16
    ([N, 4·Kp] bf16) of that."""
    n, k = w.shape
    kp = (k + 31) // 32 * 32
    out = torch.zeros((n, kp), dtype=dtype, device=device)
    out[:, :k] = w.to(device=device, dtype=dtype)
    return _split_f32_weights(out, _f32_parts("linear")) if dtype == F32 else out


def split_parts(w: torch.Tensor, kt: int, name: str = "weight") -> int:
    """Part count of a bf16-split weight for reduction length kt: 2 (split_bf16, row 2·Kp) or 3
    (split3_bf16, row 4·Kp), Kp = kt rounded up to 32; ValueError for any other row length or a
    `_rdmi_parts` tag that contradicts it."""
    kp = (kt + 31) // 32 * 32
    row = w.shape[-1]
    parts = {2 * kp: 2, 4 * kp: 3}.get(row)
    tag = getattr(w, "_rdmi_parts", None)
    if parts is None or (tag is not None and tag != parts):
        raise ValueError(f"{name}: bf16-split weight row of {row} elements matches neither the x3 ({2 * kp}) "
                         f"nor the x6 ({4 * kp}) layout of K = {kt}" +
                         (f" (tagged _rdmi_parts={tag})" if tag is not None else ""))
    return parts


def _w_code(a: torch.Tensor, w: torch.Tensor, name: str, kt: int) -> int:
    """dtype code of a GEMM/conv: the activations' dtype, or RDMI_F32_X3 / RDMI_F32_X6 for f32
    activations against split_bf16 / split3_bf16 weights.  kt = the reduction length (K of a GEMM,
    kh·kw·Cin of a conv).  The split layout is read from the weight's row length — 2·Kp (x3) or 4·Kp
    (x6), Kp = kt rounded up to 32 — so a copy that dropped the `_rdmi_parts` tag still runs the right
    engine, and a tag that disagrees with the row length fails loudly instead of running the other
    engine on the wrong layout."""
    if a.dtype == F32 and w.dtype == BF16:
        _need(w, BF16, name)
        return _N.RDMI_F32_X6 if split_parts(w, kt, name) == 3 else _N.RDMI_F32_X3
    _need(w, a.dtype, name)
    return _N.RDMI_F32 if a.dtype == F32 else _N.RDMI_F16


def geglu_permute(w: torch.Tensor, b: torch.Tensor):
    """Row permutation that puts value/gate rows of GEGLU's proj (out 2·I) side by side in
    64-row slabs: slab s = [h rows 32s..32s+31, g rows 32s..32s+31] (gemm.hip GEGLU epilogue)."""
    two_i = w.shape[0]
    i = two_i // 2
    assert i % 32 == 0
    idx = []
    for s in range(i // 32):
        idx.extend(range(32 * s, 32 * s + 32))
        idx.extend(range(i + 32 * s, i + 32 * s + 32))
    idx = torch.tensor(idx, dtype=torch.long)
    return w[idx], b[idx]


def pad_channels(c: int) -> int:
    return (c + 7) // 8 * 8


def pack_conv(w: torch.Tensor, device, cin_pad: Optional[int] = None, dtype=F16) -> torch.Tensor:
    """[Cout, Cin, kh, kw] → [Cout, Kp] in the implicit-GEMM K order of gemm.hip (rdmi.h): f16:
    [Cout][Cin_pad/64][kh][kw][64] when kh·kw > 1 and Cin_pad % 64 == 0, else [Cout][kh][kw][Cin_pad];
    f32 (gemm_f32.hip): always [Cout][kh][kw][Cin_pad]; zero padded to Kp % 32 == 0 (with f32_x3():
    split_bf16 of that)."""
    co, ci, kh, kw = w.shape
    cp = cin_pad or pad_channels(ci)
    t = torch.zeros((co, kh, kw, cp), dtype=F32)
    t[..., :ci] = w.permute(0, 2, 3, 1).float()
    if dtype == F16 and kh * kw > 1 and cp % 64 == 0:
        t = t.reshape(co, kh, kw, cp // 64, 64).permute(0, 3, 1, 2, 4).contiguous()
    k = kh * kw * cp
    kp = (k + 31) // 32 * 32
    out = torch.zeros((co, kp), dtype=dtype)
    out[:, :k] = t.reshape(co, k).to(dtype)
    if dtype == F32:
        parts = _f32_parts("conv")
        out = _split_f32_weights(out, parts).to(device)
        if parts == 3:
            out._rdmi_parts = 3
        return out
    return out.to(device)


def pack_conv_up2(w: torch.Tensor, device, cin_pad: Optional[int] = None) -> Optional[torch.Tensor]:
    """3×3 weights [Cout, Cin, 3, 3] of a conv behind a nearest ×2 upsample → the four output
    phases' merged 2×2 weights as f16 hi / lo pairs (rdmi.h rdmi_conv_args.w_up2): [4 (2a + c), Cout,
    7·Cin_pad] f16 in the order [Cin_pad/64][7][64] — the hi parts of taps (dy, dx) = (0,0), (0,1),
    (1,0), (1,1), then the lo parts of the three taps other than (a, c).  Phase a reads source rows
    (i − 1 + a, i + a): 3×3 rows {0}, {1, 2} for a = 0 and {0, 1}, {2} for a = 1 land on them
    (columns likewise), so their weights are summed — in f32 from the f16-rounded weights the 9-tap
    conv multiplies by (exact: ≤ 4 f16 values) — and split hi = f16(Σ), lo = f16(Σ − hi).  Tap (a, c)
    is a single 3×3 weight (lo = 0, not stored).  None when Cin_pad % 64."""
    co, ci, kh, kw = w.shape
    cp = cin_pad or pad_channels(ci)
    if (kh, kw) != (3, 3) or cp % 64:
        return None
    sets = (((0,), (1, 2)), ((0, 1), (2,)))
    wf = w.to(F16).float()  # the values pack_conv stores
    out = torch.zeros((4, co, cp // 64, 7, 64), dtype=F16)
    for a in range(2):
        for c in range(2):
            ph = 2 * a + c
            lo_slot = 4
            for t in range(4):
                dy, dx = t >> 1, t & 1
                sm = sum(wf[:, :, ky, kx] for ky in sets[a][dy] for kx in sets[c][dx])  # [Cout, Cin], exact
                tp = torch.zeros((co, cp), dtype=F32)
                tp[:, :ci] = sm
                hi = tp.to(F16)
                out[ph, :, :, t, :] = hi.reshape(co, cp // 64, 64)
                if t != ph:
                    out[ph, :, :, lo_slot, :] = (tp - hi.float()).to(F16).reshape(co, cp // 64, 64)
                    lo_slot += 1
    return out.reshape(4, co, 7 * cp).to(device)


# ----------------------------------------------------------------------------- GEMM / conv
def gemm(a: torch.Tensor, w: torch.Tensor, k: int, out: Optional[torch.Tensor] = None,
         bias: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None,
         rowbias: Optional[torch.Tensor] = None, rows_per_group: int = 0, alpha: float = 1.0,
         geglu: bool = False, out_f32: bool = False, n: Optional[int] = None, silu: bool = False,
         gn: bool = False) -> torch.Tensor:
    """out[m, :] = alpha·a[m, :k] @ w[:, :k]ᵀ + bias (+ rowbias[m // rows_per_group]) (+ residual).
    a: f16 [..., M, lda]; w: f16 [N, Kp]; batched over a leading dim when a is 3-D.
    gn=True: the epilogue also emits the GroupNorm moments of the output (see _gn_part), which a
    following `groupnorm(out, ...)` consumes instead of re-reading the tensor."""
    _need_act(a, "gemm.a")
    code = _w_code(a, w, "gemm.w", k)
    f32 = a.dtype == F32
    out_f32 = out_f32 or f32
    batch = a.shape[0] if a.dim() == 3 else 1
    M = a.shape[-2]
    N = w.shape[-2] if n is None else n
    NO = N // 2 if geglu else N
    if out is None:
        shape = (batch, M, NO) if a.dim() == 3 else (M, NO)
        out = torch.empty(shape, dtype=F32 if out_f32 else F16, device=a.device)
    if residual is not None and residual.dtype != a.dtype:
        raise TypeError("gemm: residual dtype must match the activations")
    g = _gemm_args(a, w, out, bias, residual, rowbias, rows_per_group, alpha, M, N, k, batch, geglu, out_f32)
    g.dtype = code
    if silu:
        g.epilogue = 2
    part = _gn_part(out, M, N) if (gn and batch == 1 and not geglu and not out_f32) else None
    if part is not None:
        g.gn_part, g.gn_ld = part.data_ptr(), part.stride(0)
    es = a.element_size()
    nb = es * (batch * M * k + (batch if w.dim() == 3 else 1) * N * k) + out.element_size() * batch * M * NO
    if residual is not None:
        nb += es * batch * M * NO
    with _Timed(_engine_name(code), 2.0 * M * N * k * batch,
                f"gemm M={M} N={N} K={k} b={batch}", nb):
        check(lib.rdmi_gemm(C.byref(g), _stream()), "rdmi_gemm")
    _gn_attach(out, part)
    return out


# GroupNorm moments emitted by a producing GEMM/conv: f32 [N/4, M/32, 2] = (Σ, Σ²) over 32 rows × 4
# channels of the f16 output (rdmi.h gn_part), attached to the output tensor object; groupnorm()
# of that same tensor object uses them (rdmi_groupnorm_stats_partials) instead of a stats pass.
_GN_ATTR = "_rdmi_gn_part"


def _gn_part(out: torch.Tensor, M: int, N: int) -> Optional[torch.Tensor]:
    if M % 32 or N % 4 or out.stride(-1) != 1 or out.stride(-2) != N or not out.is_contiguous():
        return None
    return torch.empty((N // 4, M // 32, 2), dtype=F32, device=out.device)


def _gn_attach(out: torch.Tensor, part: Optional[torch.Tensor]):
    setattr(out, _GN_ATTR, part)


def gn_view(t: torch.Tensor, shape) -> torch.Tensor:
    """t.view(shape) keeping t's GroupNorm moments (same memory, same row order)."""
    v = t.view(shape)
    _gn_attach(v, getattr(t, _GN_ATTR, None))
    return v


def _engine_name(code: int) -> str:
    return {_N.RDMI_F16: "implicit_gemm", _N.RDMI_F32: "implicit_gemm_f32", _N.RDMI_F32_X3: "implicit_gemm_f32x3",
            _N.RDMI_F32_X6: "implicit_gemm_f32x6"}[code]


def _gemm_args(a, w, out, bias, residual, rowbias, rpg, alpha, M, Nn, K, batch, geglu, out_f32):
    g = _N.GemmArgs()
    g.A = a.data_ptr(); g.lda = a.stride(-2); g.strideA = a.stride(0) if a.dim() == 3 else 0
    g.W = w.data_ptr(); g.ldw = w.stride(0); g.strideW = w.stride(0) * w.shape[0] if w.dim() == 3 else 0
    if w.dim() == 3:
        g.strideW = w.stride(0)
        g.ldw = w.stride(1)
    g.C = out.data_ptr(); g.ldc = out.stride(-2); g.strideC = out.stride(0) if out.dim() == 3 else 0
    g.c_f32 = 1 if out_f32 else 0
    g.bias = _p(bias)
    g.residual = _p(residual)
    if residual is not None:
        g.ldr = residual.stride(-2)
        g.strideR = residual.stride(0) if residual.dim() == 3 else 0
    g.rowbias = _p(rowbias)
    g.rows_per_group = rpg
    g.rowbias_ld = rowbias.stride(0) if rowbias is not None else 0
    g.alpha = alpha
    g.M, g.N, g.K, g.batch = M, Nn, K, batch
    g.epilogue = 1 if geglu else 0
    return g


def _conv_args(x, w, cout, k, stride, pad, pad_tl, upsample, bias, residual, rowbias, out, alpha, Ho, Wo, in_gn,
               w_up2=None):
    B, H, W, Cin = x.shape
    pt = pad if pad_tl is None else pad_tl
    a = _N.ConvArgs()
    a.x, a.w = x.data_ptr(), w.data_ptr()
    a.y = out.data_ptr() if out is not None else None
    a.bias, a.residual, a.rowbias = _p(bias), _p(residual), _p(rowbias)
    a.B, a.H, a.W, a.Cin, a.Cout, a.kh, a.kw = B, H, W, Cin, cout, k, k
    a.stride, a.pad_top, a.pad_left, a.upsample, a.Ho, a.Wo = stride, pt, pt, int(upsample), Ho, Wo
    a.Kp = w.shape[1]
    a.w_up2 = _p(w_up2) if upsample else None
    a.y_ld = out.stride(-2) if out is not None else 0
    a.res_ld = residual.stride(-2) if residual is not None else 0
    a.alpha = alpha
    a.rowbias_ld = 0 if (rowbias is None or rowbias.dim() == 1) else rowbias.stride(0)
    if in_gn is not None:
        mr, gamma, beta, groups, silu = in_gn
        a.in_mean_rstd, a.in_gamma, a.in_beta = _p(mr), _p(gamma), _p(beta)
        a.in_groups, a.in_silu = groups, int(silu)
    return a


def _out_hw(H, W, k, stride, pad, upsample, out_hw):
    Hi, Wi = (2 * H, 2 * W) if upsample else (H, W)
    if out_hw is None:
        out_hw = ((Hi + 2 * pad - k) // stride + 1, (Wi + 2 * pad - k) // stride + 1)
    return out_hw


def conv2d(x: torch.Tensor, w: torch.Tensor, cout: int, k: int, stride: int = 1, pad: int = 1,
           pad_tl: Optional[int] = None, upsample: bool = False, bias: Optional[torch.Tensor] = None,
           residual: Optional[torch.Tensor] = None, rowbias: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None, alpha: float = 1.0, out_hw=None, gn: bool = False,
           in_gn=None, _gn_slot=None, w_up2: Optional[torch.Tensor] = None) -> torch.Tensor:
    """NHWC f16 conv.  x [B, H, W, Cin_pad]; w packed by pack_conv.  `pad` is symmetric; pad_tl
    overrides the top/left padding with bottom/right implied by out_hw (VAE Downsample2D).
    w_up2 (upsample only): pack_conv_up2's phase weights, which the library runs where its
    phase-decomposed form applies — with RDMI_UP2=1 (opt-in; ignored otherwise).
    gn=True: also emit the output's GroupNorm moments (as gemm).
    in_gn=(mean_rstd, gamma, beta, groups, silu): GroupNorm(+SiLU) of x applied as it is read
    (rdmi.h rdmi_conv_args.in_*; only where conv2d_in_gn_supported)."""
    _need_act(x, "conv2d.x")
    code = _w_code(x, w, "conv2d.w", k * k * x.shape[-1])
    f32 = x.dtype == F32
    B, H, W, Cin = x.shape
    Ho, Wo = _out_hw(H, W, k, stride, pad, upsample, out_hw)
    if out is None:
        out = torch.empty((B, Ho, Wo, cout), dtype=x.dtype, device=x.device)
    if f32:
        gn, in_gn = False, None  # the f32 engine fuses neither (the groupnorm pass computes the moments)
    part = _gn_part(out, B * Ho * Wo, cout) if gn and _gn_slot is None else None
    if part is not None and not _split_slots_aligned(B, H * W * Cin, Ho * Wo):
        part = None  # some split level misaligns the moment slots: the next groupnorm computes them
    if B > 1 and B * H * W * Cin >= _SPLIT_ELEMS[x.dtype]:  # 32-bit byte offsets: split the batch
        h = B // 2
        rb = rowbias if (rowbias is None or rowbias.dim() == 1) else None
        # GroupNorm-moment slots of the halves: carved from this call's buffer, or — when this call
        # is itself one half of a split (_gn_slot) — from the caller's slot range, so that a batch
        # split twice (≥ 2^31 elements) still writes every image's moments
        base = (part.data_ptr(), part.stride(0)) if part is not None else _gn_slot
        for s0, s1 in ((0, h), (h, B)):
            slot = None
            if base is not None:  # alignment of every level was checked at the top (_split_slots_aligned)
                slot = (base[0] + (s0 * Ho * Wo // 32) * 2 * 4, base[1])
            ig = None
            if in_gn is not None:
                mr, gamma, beta, groups, silu = in_gn
                ig = (mr[s0 * groups * 2:s1 * groups * 2], gamma, beta, groups, silu)
            conv2d(x[s0:s1], w, cout, k, stride, pad, pad_tl, upsample, bias,
                   None if residual is None else residual[s0:s1],
                   rb if rb is not None or rowbias is None else rowbias[s0:s1],
                   out[s0:s1], alpha, out_hw, in_gn=ig, _gn_slot=slot, w_up2=w_up2)
        _gn_attach(out, part)
        return out
    kp = w.shape[1] // {_N.RDMI_F32_X3: 2, _N.RDMI_F32_X6: 4}.get(code, 1)
    if kp < k * k * Cin:
        raise ValueError(f"conv2d: packed weight K {kp} < {k * k * Cin}")
    if w_up2 is not None and (f32 or os.environ.get("RDMI_UP2", "0") != "1"):
        w_up2 = None  # opt-in (RDMI_UP2=1): DESIGN.md §4 — the phase form moves 0.2 % of the outputs
        # by 1 ulp, and any such change re-draws the depth error's extreme-pixel offset
    if w_up2 is not None and (w_up2.dtype != F16 or tuple(w_up2.shape) != (4, cout, 7 * Cin) or
                              not w_up2.is_contiguous()):
        raise ValueError(f"conv2d: w_up2 must be pack_conv_up2's [4, {cout}, {7 * Cin}] f16")
    a = _conv_args(x, w, cout, k, stride, pad, pad_tl, upsample, bias, residual, rowbias, out, alpha, Ho, Wo, in_gn,
                   w_up2)
    a.dtype = code
    a.Kp = kp
    aff = None
    if in_gn is not None and not f32 and Cin % 64 == 0 and _gn_aff():
        # the norm's scale / shift table (rdmi.h in_affine): any Cin on the two-workgroups-per-CU halo
        # engine, each wave's 8 + 8 values loaded with the halo refill (for Cin <= 256 too: −2…4 %
        # against the LDS table built in the prologue, profiles/r05j_gn8_ab.log RDMI_CONV_GN8=0 columns
        # against r05b_h32_ab.log RDMI_CONV_H32=0)
        mr, gamma, beta, groups, _ = in_gn
        aff = torch.empty((B, Cin // 64, 2, 64), dtype=F32, device=x.device)
        check(lib.rdmi_groupnorm_affine(mr.data_ptr(), gamma.data_ptr(), beta.data_ptr(), B, Cin, groups,
                                        aff.data_ptr(), _stream()), "rdmi_groupnorm_affine")
        a.in_affine = aff.data_ptr()
    if part is not None:
        a.gn_part, a.gn_ld = part.data_ptr(), part.stride(0)
    elif _gn_slot is not None:
        a.gn_part, a.gn_ld = _gn_slot
    es = x.element_size()
    # executed MFMA work: 7 taps per output pixel where the phase-decomposed upsample runs (whose
    # weights are the 4 phases × 7 taps)
    up2 = w_up2 is not None and _up2_runs(a)
    taps = 7 if up2 else k * k
    nb = es * (x.numel() + cout * (28 if up2 else k * k) * Cin +
               (2 if residual is not None else 1) * B * Ho * Wo * cout)
    with _Timed(_engine_name(code), 2.0 * B * Ho * Wo * cout * taps * Cin,
                f"conv{k} B={B} {Ho}x{Wo} {Cin}->{cout} s{stride}{' up' if upsample else ''}{' gn' if in_gn else ''}",
                nb):
        check(lib.rdmi_conv2d(C.byref(a), _stream()), "rdmi_conv2d")
    if _gn_slot is None:
        _gn_attach(out, part)
    return out


def _up2_runs(a) -> bool:
    """Mirror of rdmi_conv2d's choice of the phase-decomposed upsample form (gemm.hip)."""
    hm = int(os.environ.get("RDMI_CONV_HALO", "3"))
    return (a.upsample == 1 and bool(a.w_up2) and not a.in_mean_rstd and a.Ho % 32 == 0 and
            a.Wo % 32 == 0 and hm != 0 and a.kh == 3 and a.kw == 3 and a.Cin % 64 == 0 and a.stride == 1 and
            a.pad_top == 1 and a.pad_left == 1 and a.Ho == 2 * a.H and a.Wo == 2 * a.W)


# conv2d splits its batch when the input reaches 2 GiB (the kernels' 32-bit buffer byte offsets)
_SPLIT_ELEMS = {F16: 1 << 30, F32: 1 << 29}


def _split_slots_aligned(B: int, elems_per_image: int, howo: int) -> bool:
    """Whether every level of conv2d's recursive batch split (B > 1 and ≥ 2^30 f16 input elements)
    starts its second half on a 32-row GroupNorm-moment slot boundary."""
    if B <= 1 or B * elems_per_image < (1 << 30):
        return True
    h = B // 2
    return (h * howo) % 32 == 0 and _split_slots_aligned(h, elems_per_image, howo) and \
        _split_slots_aligned(B - h, elems_per_image, howo)


def _gn_aff() -> bool:
    """RDMI_GN_AFF=0 (A/B): fused input GroupNorm without the scale / shift table (rdmi.h in_affine) —
    the LDS table of the halo engines, so Cin ≤ 256 on the two-workgroups-per-CU engine and ≤ 1024 on
    the 256-wide one (Cout % 256 == 0)."""
    return os.environ.get("RDMI_GN_AFF", "1") != "0"


def conv2d_in_gn_supported(x: torch.Tensor, w: torch.Tensor, cout: int, k: int, groups: int, stride: int = 1,
                           pad: int = 1, upsample: bool = False, rowbias=None, out_hw=None) -> bool:
    """Whether rdmi_conv2d fuses an input GroupNorm for this conv (rdmi_conv2d_in_gn_supported)."""
    B, H, W, Cin = x.shape
    Ho, Wo = _out_hw(H, W, k, stride, pad, upsample, out_hw)
    a = _conv_args(x, w, cout, k, stride, pad, None, upsample, None, None, rowbias, None, 1.0, Ho, Wo,
                   (None, None, None, groups, 0))
    a.dtype = _N.RDMI_F32 if x.dtype == F32 else _N.RDMI_F16
    if x.dtype != F32 and Cin > 256 and Cin % 64 == 0 and _gn_aff():
        a.in_affine = 16  # conv2d passes the scale / shift table here (the query reads no pointer)
    return bool(lib.rdmi_conv2d_in_gn_supported(C.byref(a)))


def gn_conv2d(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, groups: int, eps: float, silu: bool,
              w: torch.Tensor, cout: int, k: int, **conv_kw) -> torch.Tensor:
    """conv2d(silu?(GroupNorm(x))): the norm fused into the conv's input path where the halo
    engine runs it and it pays, else groupnorm then conv2d (identical values either way).
    Policy (RDMI_GN_FUSE): 1 (default) fuses where the conv has Cin ≤ 256 — the 768²/384² VAE convs,
    −4…16 % against apply + conv (tools/kbench.py gnconv) — or Cout ≤ 384, i.e. at most three
    128-channel output tiles normalise the same input halo: at the fast preset's own batch sizes, in
    one process interleaved (tools/gn_fuse_probe.py, profiles/r06n_gn_fuse_probe.log) the UNet's 96²
    320-output convs (Cin 320 / 640 / 960) −4…−6 % and the decoder's 384² 512 → 256 conv −8 %; with four
    or more output tiles the repeated transform eats the saved pass (512 → 512 at 96² / 192²: ±0…+1 %,
    1920 → 640 at 48²: +2…+5 %), so those stay unfused.  The isolated per-launch gains (≈20 ms a step
    summed) do not carry over in full: the pipeline A/B gives −0.1 % of the step, 3 of 4 interleaved
    rounds (tools/pipe_env_ab.py, profiles/r06o_gn_fuse_pipe_ab.log) — inside the pipeline the apply pass
    and the conv after it run back to back on a tensor the previous kernel has just written, which the
    probe does not reproduce.  RDMI_GN_FUSE=3: round 5's Cin ≤ 256-only rule (A/B); 2 fuses wherever
    supported; 0 never."""
    mode = os.environ.get("RDMI_GN_FUSE", "1")
    cin = x.shape[-1]
    want = {"0": False, "2": True, "3": cin <= 256}.get(mode, cin <= 256 or cout <= 384)
    if want and conv2d_in_gn_supported(
            x, w, cout, k, groups, conv_kw.get("stride", 1), conv_kw.get("pad", 1), conv_kw.get("upsample", False),
            conv_kw.get("rowbias"), conv_kw.get("out_hw")):
        mr = groupnorm_stats(x, groups, eps)
        return conv2d(x, w, cout, k, in_gn=(mr, gamma, beta, groups, silu), **conv_kw)
    h = groupnorm(x, gamma, beta, groups, eps, silu)
    return conv2d(h, w, cout, k, **conv_kw)


# ----------------------------------------------------------------------------- norms
_ws_cache = {}


def _workspace(n_floats: int, device) -> torch.Tensor:
    # one scratch buffer per (device, stream): kernels queued on different streams (the pipeline's
    # decode stream, RDMI_DECODE_STREAM) may run concurrently
    key = (device, "ws", torch.cuda.current_stream().cuda_stream)
    t = _ws_cache.get(key)
    if t is None or t.numel() < n_floats:
        t = torch.empty(max(n_floats, 1 << 16), dtype=F32, device=device)
        _ws_cache[key] = t
    return t


def groupnorm_stats(x: torch.Tensor, groups: int, eps: float) -> torch.Tensor:
    _need_act(x, "groupnorm.x")
    B, C = x.shape[0], x.shape[-1]
    HW = x.numel() // (B * C)
    mr = torch.empty((B * groups * 2,), dtype=F32, device=x.device)
    part = getattr(x, _GN_ATTR, None)
    if part is not None and HW % 32 == 0 and (C // groups) % 4 == 0 and part.shape == (C // 4, B * HW // 32, 2):
        check(lib.rdmi_groupnorm_stats_partials(part.data_ptr(), part.stride(0), B, HW, C, groups, eps, mr.data_ptr(),
                                                _stream()), "rdmi_groupnorm_stats_partials")
        return mr
    ws = _workspace(lib.rdmi_groupnorm_workspace(B, groups), x.device)
    check(lib.rdmi_groupnorm_stats(x.data_ptr(), _dtype_code(x), B, HW, C, groups, eps, mr.data_ptr(), ws.data_ptr(),
                                   _stream()), "rdmi_groupnorm_stats")
    return mr


def groupnorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, groups: int, eps: float,
              silu: bool, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    mr = groupnorm_stats(x, groups, eps)
    B, C = x.shape[0], x.shape[-1]
    HW = x.numel() // (B * C)
    out = torch.empty_like(x) if out is None else out
    _gn_attach(out, None)
    if out.dtype != x.dtype:
        raise TypeError("groupnorm: out dtype must match x")
    check(lib.rdmi_groupnorm_apply(x.data_ptr(), out.data_ptr(), _dtype_code(x), B, HW, C, groups, mr.data_ptr(),
                                   gamma.data_ptr(), beta.data_ptr(), int(silu), _stream()), "rdmi_groupnorm_apply")
    return out


def conv3x3_to1_gn(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, groups: int, eps: float, silu: bool,
                   w9: torch.Tensor, bias: float, out: Optional[torch.Tensor] = None,
                   out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """GroupNorm(+SiLU) → 3×3 conv (pad 1) to one channel, fused (rdmi.h rdmi_conv3x3_to1_gn).
    x NHWC f16/f32 [B, H, W, C]; w9 f32 [9, C] (tap = 3·dy + dx); returns [B, H, W, 1] in out_dtype
    (default: out's dtype, else x's; f16 or f32)."""
    _need_act(x, "conv3x3_to1_gn.x")
    _need(w9, F32, "conv3x3_to1_gn.w9")
    B, H, W, C_ = x.shape
    if w9.shape != (9, C_):
        raise ValueError(f"conv3x3_to1_gn: w9 {tuple(w9.shape)} != (9, {C_})")
    mr = groupnorm_stats(x, groups, eps)
    od = out_dtype if out_dtype is not None else (out.dtype if out is not None else x.dtype)
    if od not in (F16, F32):
        raise ValueError(f"conv3x3_to1_gn: output dtype {od} (f16 or f32)")
    out = torch.empty((B, H, W, 1), dtype=od, device=x.device) if out is None else out
    if out.numel() != B * H * W or not out.is_contiguous() or out.dtype != od:
        raise ValueError("conv3x3_to1_gn: out must be a contiguous [B, H, W, 1] tensor of the output dtype")
    ws = _workspace(lib.rdmi_conv3x3_to1_gn_workspace(B, H, W), x.device)
    with _Timed("conv_head", 2.0 * 9 * C_ * B * H * W, f"head B={B} {H}x{W} {C_}->1",
                x.element_size() * B * H * W * C_ + out.element_size() * B * H * W):
        check(lib.rdmi_conv3x3_to1_gn(x.data_ptr(), _dtype_code(x), B, H, W, C_, groups, mr.data_ptr(), gamma.data_ptr(),
                                      beta.data_ptr(), int(silu), w9.data_ptr(), float(bias), out.data_ptr(),
                                      _dtype_code(out), ws.data_ptr(), _stream()), "rdmi_conv3x3_to1_gn")
    return out


def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-5,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _need_act(x, "layernorm.x")
    C_ = x.shape[-1]
    M = x.numel() // C_
    out = torch.empty_like(x) if out is None else out
    check(lib.rdmi_layernorm(x.data_ptr(), out.data_ptr(), _dtype_code(x), M, C_, gamma.data_ptr(), beta.data_ptr(), eps,
                             _stream()), "rdmi_layernorm")
    return out


# ----------------------------------------------------------------------------- attention
def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int, out: Optional[torch.Tensor] = None,
              scale: Optional[float] = None) -> torch.Tensor:
    """q/k/v: f16 [B, S, H*64] views (any row stride, unit column stride) → out [B, Sq, H*64]."""
    _need_act(q, "attention.q")
    for t, nm in ((q, "q"), (k, "k"), (v, "v")):
        _need(t, q.dtype, f"attention.{nm}")
        if t.stride(-1) != 1:
            raise ValueError("attention: inner dim must be contiguous")
    B, Sq, HD = q.shape
    D = HD // heads
    Sk = k.shape[1]
    if out is None:
        out = torch.empty((B, Sq, HD), dtype=q.dtype, device=q.device)
    sc = 1.0 / math.sqrt(D) if scale is None else scale
    code = _dtype_code(q)
    if code == _N.RDMI_F32 and f32_x3("linear"):
        code = _N.RDMI_F32_X3  # bf16-split products (attention_f32.hip attn_fwd_f32s<2>)
    elif code == _N.RDMI_F32 and f32_x6():
        code = _N.RDMI_F32_X6  # three-way split, f32-equivalent products (attn_fwd_f32s<3>)
    name = {_N.RDMI_F16: "attention_fwd", _N.RDMI_F32: "attention_fwd_f32", _N.RDMI_F32_X3: "attention_fwd_f32x3",
            _N.RDMI_F32_X6: "attention_fwd_f32x6"}[code]
    es = q.element_size()
    with _Timed(name, 4.0 * B * heads * Sq * Sk * D, f"attn B={B} H={heads} S={Sq}",
                es * B * heads * D * (2 * Sq + 2 * Sk)):
        check(lib.rdmi_attention_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), B, heads, Sq, Sk, D,
                                     q.stride(1), k.stride(1), v.stride(1), out.stride(1), q.stride(0), k.stride(0),
                                     v.stride(0), out.stride(0), sc, code, _stream()), "rdmi_attention_fwd")
    return out


def fold_attn2_pair(wq: torch.Tensor, wo: torch.Tensor, bo: torch.Tensor, k2: torch.Tensor, v2: torch.Tensor,
                    heads: int):
    """Once-per-context fold for rdmi_cross_attn_pair (weight folding, like packing): wq/wo [C, C]
    f32 (f16-rounded to_q / to_out weights), bo [C], k2/v2 [2, C] the projected context keys /
    values → (w [H, C], u [H, C], c [C]) f32 with w_h = Wq_hᵀ(k1−k0)_h/√d, u_h = Wo_h(v1−v0)_h,
    c = Wo·v0 + bo."""
    C_ = wq.shape[1]
    d = C_ // heads
    k, v = k2.float(), v2.float()
    dk, dv = (k[1] - k[0]).view(heads, d, 1), (v[1] - v[0]).view(1, heads, d)
    w = (dk * wq.view(heads, d, C_)).sum(1) / math.sqrt(d)
    u = (dv * wo.view(-1, heads, d)).sum(2).t()
    c = wo @ v[0] + bo
    return w.contiguous(), u.contiguous(), c.contiguous()


def cross_attn_pair(x: torch.Tensor, ln_g: torch.Tensor, ln_b: torch.Tensor, eps: float, w: torch.Tensor,
                    u: torch.Tensor, c: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x [M, C] f16 → x + c + Σ_h σ(LN(x)·w_h) u_h (attn2 against a two-token context, rdmi.h)."""
    _need(x, F16, "cross_attn_pair.x")
    M, C_ = x.shape
    H = w.shape[0]
    if out is None:
        out = torch.empty_like(x)
    check(lib.rdmi_cross_attn_pair(x.data_ptr(), out.data_ptr(), M, C_, H, ln_g.data_ptr(), ln_b.data_ptr(), eps,
                                   w.data_ptr(), u.data_ptr(), c.data_ptr(), _stream()), "rdmi_cross_attn_pair")
    return out


def attention_smallkv(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """q [B, Sq, H*64] (row stride any), k/v [Bkv, L, H*64] contiguous with Bkv ∈ {1, B}."""
    _need_act(q, "attention_smallkv.q")
    _need(k, q.dtype, "attention_smallkv.k")
    _need(v, q.dtype, "attention_smallkv.v")
    B, Sq, HD = q.shape
    D = HD // heads
    L = k.shape[1]
    k = k.contiguous()
    v = v.contiguous()
    if out is None:
        out = torch.empty((B, Sq, HD), dtype=q.dtype, device=q.device)
    kv_bs = 0 if k.shape[0] == 1 else k.stride(0)
    check(lib.rdmi_attention_smallkv(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), B, heads, Sq, L, D,
                                     q.stride(1), out.stride(1), q.stride(0), out.stride(0), kv_bs,
                                     1.0 / math.sqrt(D), _dtype_code(q), _stream()), "rdmi_attention_smallkv")
    return out


def softmax_rows(s: torch.Tensor, scale: float, out: Optional[torch.Tensor] = None, dtype=F16) -> torch.Tensor:
    """f32 scores [..., cols] → probabilities in `dtype` (or out's dtype); `out` may be wider (row
    stride p_ld ≥ cols: the extra columns are written as zeros)."""
    _need(s, F32, "softmax_rows.s")
    cols = s.shape[-1]
    rows = s.numel() // cols
    out = torch.empty(s.shape, dtype=dtype, device=s.device) if out is None else out
    p_ld = out.shape[-1]
    if out.numel() != rows * p_ld or not out.is_contiguous() or p_ld < cols:
        raise ValueError("softmax_rows: out must be a contiguous [..., >= cols] tensor")
    check(lib.rdmi_softmax_rows(s.data_ptr(), out.data_ptr(), rows, cols, p_ld, scale, _dtype_code(out), _stream()),
          "rdmi_softmax_rows")
    return out


def attention_1head(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float) -> torch.Tensor:
    """Single-head attention for any head dim (the VAE mid-block, d = C): f32 scores GEMM → row
    softmax → PV GEMM.  q [B, Sq, D], k/v [B, Sk, D] (row strides any, 16-B aligned) → [B, Sq, D],
    in q's dtype.  A key count that is not a multiple of 8 runs the PV GEMM on K padded with zero
    probabilities."""
    B, Sq, D = q.shape
    Sk = k.shape[1]
    if D == 512 and q.dtype == F16 and os.environ.get("RDMI_VAE_FLASH", "1") != "0":
        return attention_d512(q, k, v, scale)
    s = gemm(q, k, D, out_f32=True)
    Sp = (Sk + 7) // 8 * 8
    p = softmax_rows(s, scale, out=torch.empty((B, Sq, Sp), dtype=q.dtype, device=q.device))
    del s
    vt = torch.zeros((B, D, Sp), dtype=q.dtype, device=q.device) if Sp != Sk else None
    vt = transpose(v, out=vt)
    return gemm(p, vt, Sp)


def attention_d512(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float) -> torch.Tensor:
    """rdmi_attention_d512: single-head flash attention at head dim 512 (the VAE mid-block).
    q [B, Sq, 512], k / v [B, Sk, 512] (row strides any, 16-B aligned) → [B, Sq, 512] f16.  V is
    transposed once into a zero-padded [B, 512, ceil32(Sk)] buffer (the kernel's PV operand)."""
    B, Sq, D = q.shape
    Sk = k.shape[1]
    if D != 512 or q.dtype != F16 or k.dtype != F16 or v.dtype != F16:
        raise ValueError("attention_d512: f16 q / k / v with head dim 512")
    Skp = (Sk + 31) // 32 * 32
    vt = torch.zeros((B, D, Skp), dtype=F16, device=q.device) if Skp != Sk else None
    vt = transpose(v, out=vt)
    o = torch.empty((B, Sq, D), dtype=F16, device=q.device)
    flags = None
    if os.environ.get("RDMI_D512_W4", "0") == "1":  # opt-in: measured slower (693 vs 816 TF/s)
        flags = torch.empty((B * ((Sq + 127) // 128),), dtype=torch.int32, device=q.device)
    with _Timed("attention_d512", 4.0 * B * Sq * Sk * D, f"attn512 B={B} S={Sq}", 2 * B * D * (2 * Sq + 2 * Sk)):
        check(lib.rdmi_attention_d512(q.data_ptr(), k.data_ptr(), vt.data_ptr(), o.data_ptr(), B, Sq, Sk, Skp,
                                      q.stride(1), k.stride(1), vt.stride(1), o.stride(1), q.stride(0), k.stride(0),
                                      vt.stride(0), o.stride(0), float(scale),
                                      flags.data_ptr() if flags is not None else None, _stream()),
              "rdmi_attention_d512")
    return o


def transpose(src: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[B, R, Cc] (row stride any) → [B, Cc, R] contiguous."""
    _need_act(src, "transpose.src")
    B, R, Cc = src.shape
    out = torch.empty((B, Cc, R), dtype=src.dtype, device=src.device) if out is None else out
    check(lib.rdmi_transpose(src.data_ptr(), out.data_ptr(), B, R, Cc, src.stride(1), out.stride(1), _dtype_code(src),
                             _stream()), "rdmi_transpose")
    return out


# ----------------------------------------------------------------------------- layout / misc
def nchw_to_nhwc(x: torch.Tensor, cpad: int, scale: float = 1.0, dtype=F16) -> torch.Tensor:
    """[B, C, H, W] (any batch/channel strides, e.g. a stride-0 channel repeat) → NHWC in `dtype`."""
    if not x.is_cuda or x.dtype not in (F16, F32):
        raise TypeError("nchw_to_nhwc: device f16/f32 tensor expected")
    B, Cc, H, W = x.shape
    if x.stride(3) != 1 or x.stride(2) != W:
        x = x.contiguous()
    out = torch.empty((B, H, W, cpad), dtype=dtype, device=x.device)
    check(lib.rdmi_nchw_to_nhwc(x.data_ptr(), int(x.dtype == F32), out.data_ptr(), _dtype_code(out), B, Cc, H, W, cpad,
                                scale, x.stride(0), x.stride(1), _stream()), "rdmi_nchw_to_nhwc")
    return out


def nhwc_to_nchw_f32(x: torch.Tensor, c: int, scale: float = 1.0, shift: float = 0.0) -> torch.Tensor:
    _need_act(x, "nhwc_to_nchw.x")
    B, H, W, Cl = x.shape
    out = torch.empty((B, c, H, W), dtype=F32, device=x.device)
    check(lib.rdmi_nhwc_to_nchw_f32(x.data_ptr(), _dtype_code(x), x.stride(2), out.data_ptr(), B, c, H, W, scale, shift,
                                    _stream()), "rdmi_nhwc_to_nchw_f32")
    return out


def concat_channels(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _need_act(a, "concat.a")
    _need(b, a.dtype, "concat.b")
    Ca, Cb = a.shape[-1], b.shape[-1]
    P = a.numel() // Ca
    out = torch.empty((*a.shape[:-1], Ca + Cb), dtype=a.dtype, device=a.device) if out is None else out
    check(lib.rdmi_concat_channels(a.data_ptr(), Ca, b.data_ptr(), Cb, out.data_ptr(), P, _dtype_code(a), _stream()),
          "rdmi_concat")
    return out


def resize_nearest(x: torch.Tensor, size, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """NHWC [B, H, W, C] → [B, Ho, Wo, C], F.interpolate(size=(Ho, Wo), mode="nearest")."""
    _need_act(x, "resize_nearest.x")
    B, H, W, C_ = x.shape
    Ho, Wo = size
    out = torch.empty((B, Ho, Wo, C_), dtype=x.dtype, device=x.device) if out is None else out
    check(lib.rdmi_resize_nearest(x.data_ptr(), B, H, W, C_, out.data_ptr(), Ho, Wo, _dtype_code(x), _stream()),
          "rdmi_resize_nearest")
    return out


def gather_unet_input(rgb: torch.Tensor, depth: torch.Tensor, frame_idx: torch.Tensor, depth_bcast: bool,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """rgb [N, h, w, 8] (channels 0..3 used), depth [N or 1, h, w, 8]; frame_idx int32 device."""
    _need_act(rgb, "gather.rgb")
    _need(depth, rgb.dtype, "gather.depth")
    cnt = frame_idx.numel()
    _, h, w, _c = rgb.shape
    out = torch.empty((cnt, h, w, 8), dtype=rgb.dtype, device=rgb.device) if out is None else out
    check(lib.rdmi_gather_unet_input(rgb.data_ptr(), rgb.stride(0), depth.data_ptr(), depth.stride(0),
                                     int(depth_bcast), frame_idx.data_ptr(), cnt, h * w, out.data_ptr(),
                                     _dtype_code(rgb), _stream()), "rdmi_gather_unet_input")
    return out


def ddim_combine(x: torch.Tensor, e: torch.Tensor, ca: float, cb: float, out_scale: float, c: int, cpad: int,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y[..., :c] = (ca·x + cb·e)·out_scale, y[..., c:cpad] = 0; x/e channel-last views [.., P, ld].
    If e has fewer pixel rows than x (e.g. one noise frame), it is broadcast periodically."""
    _need_act(x, "ddim_combine.x")
    _need(e, x.dtype, "ddim_combine.e")
    P = x.numel() // x.shape[-1]
    Pe = e.numel() // e.shape[-1]
    period = 0 if Pe == P else Pe
    if period and P % Pe:
        raise ValueError("ddim_combine: broadcast operand must tile the sample")
    out = torch.empty((*x.shape[:-1], cpad), dtype=x.dtype, device=x.device) if out is None else out
    check(lib.rdmi_ddim_combine(x.data_ptr(), x.stride(-2) if x.dim() >= 2 else x.shape[-1], e.data_ptr(),
                                e.stride(-2) if e.dim() >= 2 else e.shape[-1], out.data_ptr(), out.stride(-2), P, c, cpad,
                                ca, cb, out_scale, period, _dtype_code(x), _stream()), "rdmi_ddim_combine")
    return out


def snippet_average(src: torch.Tensor, stride: int, N: int, c: int = 4) -> torch.Tensor:
    """src [n, w, h, wd, ld] → [N, h, wd, ld] mean over covering snippets (refine)."""
    _need_act(src, "snippet_average.src")
    n, w, h, wd, ld = src.shape
    src = src.contiguous()
    out = torch.empty((N, h, wd, ld), dtype=src.dtype, device=src.device)
    check(lib.rdmi_snippet_average(src.data_ptr(), n, w, stride, N, h * wd, c, ld, out.data_ptr(), _dtype_code(src),
                                   _stream()), "rdmi_snippet_average")
    return out


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == F16:
        return _N.RDMI_F16
    if t.dtype == F32:
        return _N.RDMI_F32
    raise TypeError(f"expected f16 or f32, got {t.dtype}")


def snippet_accumulate(src: torch.Tensor, k0: int, stride: int, N: int, c: int = 4,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sharded refine, rank-local half: src [nloc, w, h, wd, ld] (global snippets k0 .. k0+nloc-1) →
    f64 [N, h·wd, c] per-frame sums over the local snippets (zeros elsewhere; exact sums, so the
    all-reduce order does not change the averages)."""
    nloc, w, h, wd, ld = src.shape
    src = src.contiguous()
    out = torch.empty((N, h * wd, c), dtype=torch.float64, device=src.device) if out is None else out
    check(lib.rdmi_snippet_accumulate(src.data_ptr() if nloc else None, _dtype_code(src), k0, nloc, w, stride, N,
                                      h * wd, c, ld, out.data_ptr(), _stream()), "rdmi_snippet_accumulate")
    return out


def snippet_finish(sums: torch.Tensor, n: int, w: int, stride: int, hw, ld: int, dtype=F16) -> torch.Tensor:
    """Sharded refine, after the all-reduce: f64 [N, P, c] sums → [N, h, wd, ld] means (÷ the frame's
    cover count over all n snippets)."""
    if sums.dtype != torch.float64:
        raise TypeError("snippet_finish: f64 sums expected (snippet_accumulate)")
    N, P, c = sums.shape
    h, wd = hw
    out = torch.empty((N, h, wd, ld), dtype=dtype, device=sums.device)
    check(lib.rdmi_snippet_finish(sums.data_ptr(), n, w, stride, N, P, c, ld, out.data_ptr(), _dtype_code(out),
                                  _stream()), "rdmi_snippet_finish")
    return out


def minmax(x: torch.Tensor) -> torch.Tensor:
    if x.dtype not in (F16, F32):
        raise TypeError("minmax: f16/f32 expected")
    out = torch.empty(2, dtype=F32, device=x.device)
    ws = _workspace(2048, x.device)
    check(lib.rdmi_minmax(x.data_ptr(), int(x.dtype == F32), x.numel(), out.data_ptr(), ws.data_ptr(), _stream()),
          "rdmi_minmax")
    return out


def renormalize_(x: torch.Tensor, mm: torch.Tensor) -> torch.Tensor:
    _need(x, F32, "renormalize.x")
    check(lib.rdmi_renormalize_f32(x.data_ptr(), x.numel(), mm.data_ptr(), _stream()), "rdmi_renormalize")
    return x


# ----------------------------------------------------------------------------- aligner
def aligner_prepare(x: torch.Tensor, shift: torch.Tensor, border: int, factor: int) -> torch.Tensor:
    """x [n, w, H, W] f16/f32 → f32 [n, w, P]."""
    n, w, H, W = x.shape
    hs = (H - 2 * border + factor - 1) // factor
    ws_ = (W - 2 * border + factor - 1) // factor
    out = torch.empty((n, w, hs * ws_), dtype=F32, device=x.device)
    check(lib.rdmi_aligner_prepare(x.data_ptr(), int(x.dtype == F32), n, w, H, W, border, factor, shift.data_ptr(),
                                   out.data_ptr(), _stream()), "rdmi_aligner_prepare")
    return out


def aligner_optimize(xs: Sequence[torch.Tensor], scales: Sequence[torch.Tensor], trans: Sequence[torch.Tensor],
                     strides: Sequence[int], seq_len: int, lr: float, betas, eps: float, lmda2: float, lmda3: float,
                     depth_w: float, loss_scale: float, iters: int, history: Optional[torch.Tensor]):
    a = _N.AlignerArgs()
    a.n_dil = len(xs)
    for d, (x, s, t, st) in enumerate(zip(xs, scales, trans, strides)):
        _need(x, F32, "aligner.x")
        a.x[d] = x.data_ptr()
        a.s[d] = s.data_ptr()
        a.t[d] = t.data_ptr()
        a.n[d] = x.shape[0]
        a.stride[d] = st
        a.w[d] = x.shape[1]
    a.seq_len = seq_len
    a.P = xs[0].shape[2]
    a.lr, a.beta1, a.beta2, a.eps = lr, betas[0], betas[1], eps
    a.lmda2, a.lmda3, a.depth_w, a.loss_scale = lmda2, lmda3, depth_w, loss_scale
    a.iters = iters
    a.history = _p(history)
    nws = lib.rdmi_aligner_workspace(C.byref(a))
    ws = torch.empty(nws + 16, dtype=F32, device=xs[0].device)
    a.workspace = ws.data_ptr()
    check(lib.rdmi_aligner_optimize(C.byref(a), _stream()), "rdmi_aligner_optimize")
    return ws  # keep alive until the stream has consumed it


def aligner_merge(xf: Sequence[torch.Tensor], scales, trans, strides, seq_len: int, shift: torch.Tensor,
                  f32_arith: bool = False) -> torch.Tensor:
    """xf[d] [n_d, w_d, H, W] (f16/f32) → [seq_len, H, W] f32.  f16 snippets are merged in the
    reference's f16 arithmetic unless f32_arith (rdmi.h rdmi_aligner_merge x_f32 = 2)."""
    nd = len(xf)
    H, W = xf[0].shape[-2:]
    wv = (C.c_int * nd)(*[x.shape[1] for x in xf])
    out = torch.empty((seq_len, H, W), dtype=F32, device=xf[0].device)
    xp = (C.c_void_p * nd)(*[x.data_ptr() for x in xf])
    sp = (C.c_void_p * nd)(*[s.data_ptr() for s in scales])
    tp = (C.c_void_p * nd)(*[t.data_ptr() for t in trans])
    nn = (C.c_int * nd)(*[x.shape[0] for x in xf])
    stv = (C.c_int * nd)(*list(strides))
    mode = 1 if xf[0].dtype == F32 else (2 if f32_arith else 0)
    check(lib.rdmi_aligner_merge(nd, xp, mode, sp, tp, nn, stv, wv, seq_len, H * W,
                                 shift.data_ptr(), out.data_ptr(), _stream()), "rdmi_aligner_merge")
    return out


def aligner_merge_partial_window(xf: Sequence[Optional[torch.Tensor]], k0: Sequence[int], n: Sequence[int], scales,
                                 trans, strides, w: Sequence[int], f0: int, nf: int, HW: int, shift: torch.Tensor,
                                 x_f32, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sharded merge, rank-local half (rdmi_aligner_merge_partial_window): xf[d] [nloc_d, w_d, H, W] =
    global snippets k0[d] .. of dilation d (None / 0 rows when the rank owns none) → f64 [nf, HW] sums of
    s·x+t over frames f0 .. f0+nf-1 (a range the rank's snippets cover; `out`: a contiguous f64 [nf, HW]
    view to write into)."""
    nd = len(xf)
    if out is None:
        out = torch.empty((nf, HW), dtype=torch.float64, device=shift.device)
    elif out.dtype != torch.float64 or tuple(out.shape) != (nf, HW) or not out.is_contiguous():
        raise ValueError("aligner_merge_partial_window: out must be contiguous f64 [nf, HW]")
    xp = (C.c_void_p * nd)(*[(x.data_ptr() if x is not None and x.shape[0] else None) for x in xf])
    sp = (C.c_void_p * nd)(*[s.data_ptr() for s in scales])
    tp = (C.c_void_p * nd)(*[t.data_ptr() for t in trans])
    nn = (C.c_int * nd)(*list(n))
    kk = (C.c_int * nd)(*list(k0))
    nl = (C.c_int * nd)(*[(x.shape[0] if x is not None else 0) for x in xf])
    stv = (C.c_int * nd)(*list(strides))
    wv = (C.c_int * nd)(*list(w))
    check(lib.rdmi_aligner_merge_partial_window(nd, xp, int(x_f32), sp, tp, nn, stv, kk, nl, wv, f0, nf, HW,
                                                shift.data_ptr(), out.data_ptr(), _stream()),
          "rdmi_aligner_merge_partial_window")
    return out


def aligner_merge_finish_pieces(recv: torch.Tensor, pieces: Sequence[Tuple[int, int]], n: Sequence[int],
                                strides: Sequence[int], w: Sequence[int], f0: int, nf: int, HW: int) -> torch.Tensor:
    """Sharded merge over frame windows, after the all-to-all: recv f64 [Σ nf_q, HW] = the pieces
    (first frame, frame count) back to back in source-rank order → f32 [nf, HW] means of frames f0 .."""
    if recv.dtype != torch.float64:
        raise TypeError("aligner_merge_finish_pieces: f64 sums expected")
    nd, npc = len(n), len(pieces)
    out = torch.empty((nf, HW), dtype=F32, device=recv.device)
    nn = (C.c_int * nd)(*list(n))
    stv = (C.c_int * nd)(*list(strides))
    wv = (C.c_int * nd)(*list(w))
    pf = (C.c_int * max(npc, 1))(*[p[0] for p in pieces])
    pn = (C.c_int * max(npc, 1))(*[p[1] for p in pieces])
    check(lib.rdmi_aligner_merge_finish_pieces(nd, nn, stv, wv, f0, nf, HW, npc, pf, pn,
                                               recv.data_ptr() if recv.numel() else None, out.data_ptr(),
                                               _stream()), "rdmi_aligner_merge_finish_pieces")
    return out


# ----------------------------------------------------------------------------- frame ingest / resize
_RESIZE_MODES = {"NEAREST": _N.RDMI_RESIZE_NEAREST, "BILINEAR": _N.RDMI_RESIZE_BILINEAR,
                 "BICUBIC": _N.RDMI_RESIZE_BICUBIC}


def resize(x: torch.Tensor, size, mode: str = "BILINEAR", normalize: bool = False, channels_last: bool = False,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """rdmi_resize: torchvision resize(antialias=True) of a float / uint8 image batch → f32 [N, C, Ho, Wo].
    x: [N, C, H, W] (any strides), or [N, H, W, C] with channels_last=True (decoded rgb24 frames).
    normalize: (v / 255)·2 − 1 after the resize (video_io.py:123)."""
    if not x.is_cuda:
        raise ValueError(f"resize: expected a device tensor, got {x.device}")
    if x.dtype == torch.uint8:
        code = _N.RDMI_U8
    elif x.dtype == F32:
        code = _N.RDMI_F32
    else:
        raise TypeError(f"resize: uint8 or float32 input, got {x.dtype}")
    if mode not in _RESIZE_MODES:
        raise NotImplementedError(f"resize: interpolation {mode} (NEAREST, BILINEAR, BICUBIC)")
    if x.dim() != 4:
        raise ValueError(f"resize: 4-D input expected, got {tuple(x.shape)}")
    if channels_last:
        N, H, W, Cc = x.shape
        sn, sy, sx, sc = x.stride()
    else:
        N, Cc, H, W = x.shape
        sn, sc, sy, sx = x.stride()
    Ho, Wo = int(size[0]), int(size[1])
    if out is None:
        out = torch.empty((N, Cc, Ho, Wo), dtype=F32, device=x.device)
    if out.shape != (N, Cc, Ho, Wo) or out.dtype != F32 or not out.is_contiguous():
        raise ValueError("resize: out must be a contiguous f32 [N, C, Ho, Wo] tensor")
    ws = None
    nb = lib.rdmi_resize_workspace(N, Cc, H, W, Ho, Wo)
    if nb:
        ws = torch.empty(nb, dtype=torch.uint8, device=x.device)
    check(lib.rdmi_resize(x.data_ptr(), code, sn, sc, sy, sx, N, Cc, H, W, Ho, Wo, _RESIZE_MODES[mode],
                          int(normalize), out.data_ptr(), _p(ws), _stream()), "rdmi_resize")
    return out
