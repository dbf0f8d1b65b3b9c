"""Bit fingerprints of DepthAligner.run (scales, translations, loss history, merged depth) for A/B builds
that must be bitwise equal (schedule-only changes to aligner.hip): run once per library and diff.

    python tools/aligner_bits.py > a.txt; RDMI_LIB=tools/librdmi_ab_old.so python tools/aligner_bits.py > b.txt
    diff a.txt b.txt
With --time: also the per-call time of each case (2000 iterations)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rollingdepth_amd import DepthAligner  # noqa: E402


def fp(t: torch.Tensor) -> str:
    t = t.contiguous()
    v = (t.view(torch.int16) if t.element_size() == 2 else t.view(torch.int32)).flatten().to(torch.int64)
    w = torch.arange(v.numel(), device=v.device, dtype=torch.int64) % 65521 + 1
    return f"{int(v.sum())} {int((v * w).sum() % (1 << 61))}"


def snippets(g, n, w, res, dtype):
    # smooth per-frame depth (a ramp + a blob) under per-snippet scale / shift and noise: the optimiser
    # has something to align
    yy, xx = torch.meshgrid(torch.linspace(0, 1, res, device="cuda"), torch.linspace(0, 1, res, device="cuda"),
                            indexing="ij")
    base = 0.3 + 0.4 * yy + 0.2 * torch.exp(-((xx - 0.5) ** 2 + (yy - 0.4) ** 2) * 8)
    s = 0.7 + 0.6 * torch.rand(n, 1, 1, 1, 1, device="cuda", generator=g)
    t = 0.1 * torch.randn(n, 1, 1, 1, 1, device="cuda", generator=g)
    noise = 0.02 * torch.randn(n, w, 1, res, res, device="cuda", generator=g)
    return (base * s + t + noise).clamp(0.0, 1.0).to(dtype)


def main():
    timing = "--time" in sys.argv
    cases = [("fast N=100 [1,25] 768^2 f16", [(98, 3), (50, 3)], [1, 25], 768, torch.float16),
             ("paper-like N=60 [1,10,25] 256^2 f32", [(58, 3), (40, 3), (10, 3)], [1, 10, 25], 256, torch.float32),
             ("mixed lengths [3,2] 256^2 f16", [(28, 3), (27, 2)], [1, 3], 256, torch.float16)]
    for lab, shapes, dil, res, dt in cases:
        g = torch.Generator(device="cuda").manual_seed(0)
        sn = [snippets(g, n, w, res, dt) for n, w in shapes]
        al = DepthAligner("cuda")
        merged, sc, tr, hist = al.run(sn, dil)
        torch.cuda.synchronize()
        line = (f"{lab:40s} s {fp(torch.cat([x.flatten() for x in sc]))} | t {fp(torch.cat([x.flatten() for x in tr]))}"
                f" | merged {fp(merged)} | hist {fp(torch.as_tensor(hist, dtype=torch.float32))}")
        if timing:
            al.run(sn, dil)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                al.run(sn, dil)
            torch.cuda.synchronize()
            line += f" | {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms"
        print(line, flush=True)


if __name__ == "__main__":
    main()
