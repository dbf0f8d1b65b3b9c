"""The UNet's GEGLU projections (attention.py:421-548 FeedForward, proj = Linear(C, 8C) → h·gelu(g)) at
the bench's launch shapes on each GEMM engine: HIP-event time per launch and bitwise equality against
the default policy.

    python tools/geglu_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

ENGINES = (("default", {}), ("occ2", {"RDMI_GEMM_OCC2": "2"}), ("classic", {"RDMI_GEMM_PP": "0", "RDMI_GEMM_OCC2": "0"}),
           ("default", {}), ("occ2", {"RDMI_GEMM_OCC2": "2"}))
g = torch.Generator(device="cuda").manual_seed(0)
for lab, M, C in (("L0 M=691200 K=320 N=2560", 691200, 320), ("L1 M=172800 K=640 N=5120", 172800, 640),
                  ("L2 M=43200 K=1280 N=10240", 43200, 1280)):
    a = torch.randn(M, C, device="cuda", generator=g).half()
    w = torch.randn(8 * C, C, generator=torch.Generator().manual_seed(1)) / C ** 0.5
    b = torch.randn(8 * C) * 0.1
    wp, bp = K.geglu_permute(w, b)
    W = K.pack_linear(wp, "cuda")
    bias = bp.to("cuda")
    y = torch.empty(M, 4 * C, device="cuda", dtype=torch.float16)
    ref = None
    for name, env in ENGINES:
        for k in ("RDMI_GEMM_OCC2", "RDMI_GEMM_PP"):
            os.environ.pop(k, None)
        os.environ.update(env)
        K.gemm(a, W, C, out=y, bias=bias, geglu=True)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            K.gemm(a, W, C, out=y, bias=bias, geglu=True)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        if ref is None:
            ref = y.clone()
        same = torch.equal(y.view(torch.int16), ref.view(torch.int16))
        print(f"{lab:28s} {name:8s} {ms * 1e3:8.1f} us {2 * M * 8 * C * C / ms / 1e9:7.1f} TF/s  bitwise {same}", flush=True)
