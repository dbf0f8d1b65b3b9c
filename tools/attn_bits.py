"""Bit fingerprints of the f16 cross-frame attention (K.attention) at the UNet's shapes and ragged key
counts, for A/B builds that must be bitwise equal (schedule-only changes to attention.hip):

    python tools/attn_bits.py > a.txt; RDMI_LIB=tools/librdmi_ab_old.so python tools/attn_bits.py > b.txt"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
for B, S, H in ((4, 27648, 5), (4, 6912, 10), (8, 1728, 20), (8, 432, 20), (2, 1000, 5), (3, 77, 2)):
    C = 64 * H
    qkv = (torch.randn(B, S, 3 * C, device="cuda", generator=g) * 1.5).half()
    o = K.attention(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], H)
    torch.cuda.synchronize()
    v = o.contiguous().view(torch.int16).flatten().to(torch.int64)
    w = torch.arange(v.numel(), device="cuda", dtype=torch.int64) % 65521 + 1
    print(f"B={B} S={S} H={H}: {int(v.sum())} {int((v * w).sum() % (1 << 61))}", flush=True)
