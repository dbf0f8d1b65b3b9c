"""A/B of an attention switch read per launch (e.g. RDMI_ATTN_SPRIO): the f16 cross-frame attention at the
pipeline's shapes, values alternated over rounds, outputs compared bitwise.

    python tools/attn_env_ab.py --env RDMI_ATTN_SPRIO [--values 0,1] [--rounds 4]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--env", required=True)
ap.add_argument("--values", default="0,1")
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
vals = a.values.split(",")
torch.manual_seed(0)
for lab, B, S, H in [("L0 S=27648 H=5 b=25", 25, 27648, 5), ("L1 S=6912 H=10 b=25", 25, 6912, 10),
                     ("L2 S=1728 H=20 b=25", 25, 1728, 20)]:
    C = H * 64
    qkv = torch.randn(B, S, 3 * C, device="cuda").half()
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    outs = {x: torch.empty(B, S, C, device="cuda", dtype=torch.float16) for x in vals}
    best = {x: 1e9 for x in vals}
    for _ in range(a.rounds):
        for x in vals:
            os.environ[a.env] = x
            K.attention(q, k, v, H, out=outs[x])
            torch.cuda.synchronize()
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(a.iters):
                K.attention(q, k, v, H, out=outs[x])
            s1.record()
            torch.cuda.synchronize()
            best[x] = min(best[x], s0.elapsed_time(s1) / a.iters)
    fl = 4.0 * B * H * S * S * 64
    same = all(torch.equal(outs[vals[0]], outs[x]) for x in vals[1:])
    print(f"attn {lab:22s} " + "  ".join(f"{a.env}={x}: {best[x] * 1e3:9.1f} us {fl / best[x] / 1e9:7.1f} TF/s"
                                          for x in vals) + f"  bitwise-equal={same}", flush=True)
