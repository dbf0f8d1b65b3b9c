"""f32 cross-frame attention engines at the paper preset's L0 / L1 shapes (768², 15-snippet UNet
batch): exact f32-input MFMA, bf16x3 split, bf16x6 split — time (HIP events) and max |Δ| against an
f64 softmax on 256 sampled rows.

    python tools/f32_attn_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402


def sdpa64(q, k, v, H):
    B, Sq, HD = q.shape
    D = HD // H
    qh = q.double().view(B, Sq, H, D).transpose(1, 2)
    kh = k.double().view(B, -1, H, D).transpose(1, 2)
    vh = v.double().view(B, -1, H, D).transpose(1, 2)
    return F.scaled_dot_product_attention(qh, kh, vh).transpose(1, 2).reshape(B, Sq, HD)


g = torch.Generator(device="cuda").manual_seed(0)
for lab, B, S, H in (("L0 768^2 x15", 15, 27648, 5), ("L1 768^2 x15", 15, 6912, 10)):
    C = H * 64
    qkv = torch.randn(B, S, 3 * C, device="cuda", generator=g) * 0.7
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    rows = torch.randint(0, S, (256,), device="cuda", generator=g)
    ref = sdpa64(q[:1, rows].contiguous(), k[:1], v[:1], H)
    for name, env in (("exact", {"RDMI_F32_X3": "0"}), ("x3", {"RDMI_F32_X3": "1"}),
                      ("x6", {"RDMI_F32_X3": "conv", "RDMI_F32_X6": "1"})):
        os.environ.update(env)
        o = K.attention(q, k, v, H)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            K.attention(q, k, v, H, out=o)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 3
        err = (o[:1, rows].double() - ref).abs().max().item()
        fl = 4.0 * B * H * S * S * 64
        print(f"{lab:14s} {name:6s} {ms:9.2f} ms {fl / ms / 1e9:7.1f} f32-TF/s  max |d| {err:.2e}", flush=True)
