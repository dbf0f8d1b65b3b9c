"""Attention output error on sampled query rows vs an f64 softmax (A/B numerics of kernel variants
selected by environment switches, e.g. RDMI_ATTN_EXP16=1).

    python tools/attn_err.py [--S 27648] [--H 5] [--B 2] [--temp 1.0]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--S", type=int, default=27648)
ap.add_argument("--H", type=int, default=5)
ap.add_argument("--B", type=int, default=2)
ap.add_argument("--rows", type=int, default=256)
a = ap.parse_args()
for temp in (1.0, 2.0, 4.0):
    torch.manual_seed(0)
    C = a.H * 64
    q = (torch.randn(a.B, a.S, C, device="cuda") * temp).half()
    k = torch.randn(a.B, a.S, C, device="cuda").half()
    v = torch.randn(a.B, a.S, C, device="cuda").half()
    out = K.attention(q, k, v, a.H)
    torch.cuda.synchronize()
    rows = torch.randperm(a.S, device="cuda")[: a.rows]
    errs, rel = [], []
    for b in range(a.B):
        for h in range(a.H):
            qs = q[b, rows, h * 64:(h + 1) * 64].double()
            kk = k[b, :, h * 64:(h + 1) * 64].double()
            vv = v[b, :, h * 64:(h + 1) * 64].double()
            p = torch.softmax(qs @ kk.T / 8.0, dim=-1)
            ref = p @ vv
            got = out[b, rows, h * 64:(h + 1) * 64].double()
            errs.append((got - ref).abs().mean().item())
            rel.append(((got - ref).abs().max() / ref.abs().max()).item())
    tag = os.environ.get("RDMI_ATTN_EXP16", "0")
    print(f"exp16={tag} temp={temp}: mean|err| {sum(errs) / len(errs):.3e}  max rel {max(rel):.3e}")
