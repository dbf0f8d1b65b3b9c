"""GEMM engine policy A/B at the pipeline's Linear shapes (snippet batch 25 → 75 frames per UNet
call): every engine setting timed alternately in one process (the switches are read per launch).

    python tools/gemm_policy_ab.py [--rounds 3] [--iters 10]"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()

F0 = 75 * 9216  # L0 rows per UNet call (25 snippets × 3 frames × 96²)
SHAPES = [("L0 qkv", F0, 960, 320, False, False), ("L0 ff1 geglu", F0, 2560, 320, True, False),
          ("L0 proj_out +res", F0, 320, 320, False, True), ("L0 to_out +res", F0, 320, 320, False, True),
          ("L0 ff2 +res", F0, 320, 1280, False, True), ("L1 qkv", F0 // 4, 1920, 640, False, False),
          ("L1 ff1 geglu", F0 // 4, 5120, 640, True, False), ("L1 proj +res", F0 // 4, 640, 640, False, True),
          ("L1 ff2 +res", F0 // 4, 640, 2560, False, True), ("L2 qkv", F0 // 16, 3840, 1280, False, False),
          ("L2 ff1 geglu", F0 // 16, 10240, 1280, True, False), ("L2 proj +res", F0 // 16, 1280, 1280, False, True),
          ("L2 ff2 +res", F0 // 16, 1280, 5120, False, True), ("vae qkv 75fr", 75 * 9216, 1536, 512, False, False),
          ("vae 1x1 256->128 768^2 x4", 4 * 589824, 128, 256, False, False)]
SETTINGS = {"default": {}, "occ2-all": {"RDMI_GEMM_OCC2": "2"}, "occ2-off": {"RDMI_GEMM_OCC2": "0"},
            "pp-forced": {"RDMI_GEMM_OCC2": "0", "RDMI_GEMM_PP": "2"}, "classic": {"RDMI_GEMM_OCC2": "0", "RDMI_GEMM_PP": "0"}}


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


torch.manual_seed(0)
for lab, M, N, Kd, geglu, res in SHAPES:
    x = torch.randn(M, Kd, device="cuda").half()
    w = K.pack_linear(torch.randn(N, Kd) / math.sqrt(Kd), "cuda")
    b = 0.02 * torch.randn(N, device="cuda")
    r = torch.randn(M, N, device="cuda").half() if res else None
    best = {}
    for _ in range(a.rounds):
        for name, env in SETTINGS.items():
            for k in ("RDMI_GEMM_OCC2", "RDMI_GEMM_PP"):
                os.environ.pop(k, None)
            os.environ.update(env)
            try:
                ms = timeit(lambda: K.gemm(x, w, Kd, bias=b, residual=r, geglu=geglu), a.iters)
            except Exception as ex:  # noqa: BLE001 — an engine that refuses the shape
                ms = float("inf")
            best[name] = min(best.get(name, float("inf")), ms)
    for k in ("RDMI_GEMM_OCC2", "RDMI_GEMM_PP"):
        os.environ.pop(k, None)
    fl = 2.0 * M * N * Kd
    win = min(best, key=best.get)
    print(f"{lab:26s} " + " ".join(f"{n}={fl / t / 1e9:6.0f}" for n, t in best.items()) +
          f"  TF/s  best={win} ({best['default'] / best[win]:.3f}x default)", flush=True)
