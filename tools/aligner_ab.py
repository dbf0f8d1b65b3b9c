"""Aligner loop A/B at the fast preset's shape (N = 100, dilations [1, 25], 768², 2 000 iterations):
RDMI_ALIGNER_FUSED = 2 (persistent single launch, opt-in, where it fits), 1 (two launches per iteration,
the default), 0 (three launches) — outputs compared bitwise against the first value, then timed in
alternating rounds.

    python tools/aligner_ab.py [--rounds 3] [--values 1,2]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import DepthAligner  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--values", default="1,2")
ap.add_argument("--iters", type=int, default=2000)
a = ap.parse_args()
vals = a.values.split(",")
g = torch.Generator(device="cuda").manual_seed(0)
sn = [(torch.rand(n, 3, 1, 768, 768, device="cuda", generator=g) * 0.8 + 0.1).half() for n in (98, 50)]
al = DepthAligner("cuda", num_iterations=a.iters)
outs = {}
for v in vals:
    os.environ["RDMI_ALIGNER_FUSED"] = v
    m, s, t, h = al.run(sn, [1, 25])
    torch.cuda.synchronize()
    outs[v] = (m.cpu(), [x.cpu() for x in s], [x.cpu() for x in t], h)
ref = outs[vals[0]]
for v in vals[1:]:
    o = outs[v]
    same_m = torch.equal(o[0], ref[0])
    same_st = all(torch.equal(x, y) for x, y in zip(o[1] + o[2], ref[1] + ref[2]))
    same_h = o[3] == ref[3]
    nd = sum(int((x != y).sum()) for x, y in zip(o[1] + o[2], ref[1] + ref[2]))
    print(f"RDMI_ALIGNER_FUSED={v} vs {vals[0]}: merged bitwise {same_m}, s/t bitwise {same_st} ({nd} differ), "
          f"history equal {same_h}, finite {bool(torch.isfinite(o[0]).all())}", flush=True)
best = {v: 1e9 for v in vals}
for r in range(a.rounds):
    for v in vals:
        os.environ["RDMI_ALIGNER_FUSED"] = v
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        al.run(sn, [1, 25])
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        best[v] = min(best[v], ms)
        print(f"round {r} RDMI_ALIGNER_FUSED={v}: {ms:8.2f} ms (DepthAligner.run incl. prepare + merge)", flush=True)
print("best: " + "  ".join(f"{v}: {best[v]:.2f} ms" for v in vals))
