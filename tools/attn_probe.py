"""Run one attention (or conv) shape a few times — a target for rocprofv3 PMC passes.

    python tools/attn_probe.py [--what attn|conv] [--iters 5] [--shape B,H,W,Cin,Cout]"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--what", default="attn")
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--shape", default="8,192,192,512,512", help="conv: B,H,W,Cin,Cout")
a = ap.parse_args()
torch.manual_seed(0)
if a.what == "attn":
    B, S, H = 8, 27648, 5
    C = H * 64
    qkv = torch.randn(B, S, 3 * C, device="cuda").half()
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    out = torch.empty(B, S, C, device="cuda", dtype=torch.float16)
    fn = lambda: K.attention(q, k, v, H, out=out)  # noqa: E731
else:
    B, H, W, ci, co = (int(v) for v in a.shape.split(","))
    x = torch.randn(B, H, W, ci, device="cuda").half()
    w = K.pack_conv(torch.randn(co, ci, 3, 3) / math.sqrt(ci * 9), "cuda", ci)
    out = torch.empty(B, H, W, co, device="cuda", dtype=torch.float16)
    fn = lambda: K.conv2d(x, w, co, 3, out=out)  # noqa: E731
for _ in range(a.iters):
    fn()
torch.cuda.synchronize()
print("done")
