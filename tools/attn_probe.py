"""Run the L0 cross-frame attention shape a few times (for rocprofv3 --pmc passes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402

B, S, H = 2, 27648, 5
C = H * 64
qkv = torch.randn(B, S, 3 * C, device="cuda").half()
out = torch.empty(B, S, C, device="cuda", dtype=torch.float16)
for _ in range(3):
    K.attention(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], H, out=out)
torch.cuda.synchronize()
x = torch.randn(8, 192, 192, 512, device="cuda").half()
w = K.pack_conv(torch.randn(512, 512, 3, 3) / 48, "cuda", 512)
for _ in range(3):
    K.conv2d(x, w, 512, 3)
torch.cuda.synchronize()
print("ok")
