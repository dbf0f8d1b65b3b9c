"""Probe: L0 attention speed before/after large allocations (placement / translation effects)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402


def timeit(fn, n=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def attn_run(tag):
    B, S, H = 25, 27648, 5
    C = H * 64
    qkv = torch.randn(B, S, 3 * C, device="cuda").half()
    out = torch.empty(B, S, C, device="cuda", dtype=torch.float16)
    ms = timeit(lambda: K.attention(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], H, out=out))
    print(f"{tag:40s} {ms:8.2f} ms  {4.0 * B * H * S * S * 64 / ms / 1e9:7.1f} TF/s  ptr {qkv.data_ptr():#x}", flush=True)
    del qkv, out


import math  # noqa: E402
import time  # noqa: E402

attn_run("fresh")
B = 8
x = torch.randn(B, 768, 768, 128, device="cuda").half()
w = K.pack_conv(torch.randn(128, 128, 3, 3) / math.sqrt(128 * 9), "cuda", 128)
o = torch.empty_like(x)
for secs in (0.5, 2.0, 5.0):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs:
        for _ in range(20):
            K.conv2d(x, w, 128, 3, out=o)
        torch.cuda.synchronize()
    attn_run(f"right after {secs:.1f} s of 768^2 convs")
time.sleep(5)
attn_run("after 5 s idle")
