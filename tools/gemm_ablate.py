"""Ablation probe of the ping-pong GEMM engine on dense square GEMMs (RDMI_GEMM_DBG bits:
1 no main-loop DMA, 2 no barriers, 4 no ds_reads; results garbage, timings isolate costs).

    RDMI_GEMM_DBG=<bits> python tools/gemm_ablate.py [--n 4096,8192]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402
from tools.kbench import timeit  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", default="4096,8192")
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
for n in [int(x) for x in a.n.split(",")]:
    A = (torch.rand(n, n, device="cuda") * 2 - 1).half()
    W = (torch.rand(n, n, device="cuda") * 2 - 1).half()
    out = torch.empty(n, n, device="cuda", dtype=torch.float16)
    ms = timeit(lambda: K.gemm(A, W, n, out=out), a.iters)
    print(f"DBG={os.environ.get('RDMI_GEMM_DBG', '0')} n={n} {ms * 1e3:9.1f} us {2.0 * n ** 3 / ms / 1e9:8.1f} TFLOP/s",
          flush=True)
