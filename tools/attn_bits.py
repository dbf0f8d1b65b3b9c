"""Bit fingerprints of the attention kernels at the UNet's / VAE's shapes and ragged key counts, for A/B
builds that must be bitwise equal (schedule-only changes to attention.hip / attention_d512.hip /
attention_f32.hip):

    python tools/attn_bits.py > a.txt; RDMI_LIB=tools/librdmi_ab_old.so python tools/attn_bits.py > b.txt

Covers attn_fwd_d64 (default and RDMI_ATTN_PIPE=1), attn_fwd_d512 (and its RDMI_D512_W4 pass), and the
f32 engines attn_fwd_f32 / attn_fwd_f32s<2|3> (RDMI_F32_X3 / RDMI_F32_X6 modes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import kernels as K  # noqa: E402


def fp(o):
    torch.cuda.synchronize()
    v = o.contiguous().view(torch.int16 if o.dtype == torch.float16 else torch.int32).flatten().to(torch.int64)
    w = torch.arange(v.numel(), device="cuda", dtype=torch.int64) % 65521 + 1
    return f"{int(v.sum())} {int((v * w).sum() % (1 << 61))}"


g = torch.Generator(device="cuda").manual_seed(0)
for B, S, H in ((4, 27648, 5), (4, 6912, 10), (8, 1728, 20), (8, 432, 20), (2, 1000, 5), (3, 77, 2)):
    C = 64 * H
    qkv = (torch.randn(B, S, 3 * C, device="cuda", generator=g) * 1.5).half()
    o = K.attention(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], H)
    print(f"d64 B={B} S={S} H={H}: {fp(o)}", flush=True)
    if "--pipe" in sys.argv:
        os.environ["RDMI_ATTN_PIPE"] = "1"
        o = K.attention(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], H)
        os.environ.pop("RDMI_ATTN_PIPE")
        print(f"pipe B={B} S={S} H={H}: {fp(o)}", flush=True)
for B, S in ((3, 9216), (2, 2304), (2, 1000)):
    qkv = (torch.randn(B, S, 1536, device="cuda", generator=g) * 0.6).half()
    o = K.attention_d512(qkv[..., :512], qkv[..., 512:1024], qkv[..., 1024:], 512 ** -0.5)
    print(f"d512 B={B} S={S}: {fp(o)}", flush=True)
    os.environ["RDMI_D512_W4"] = "1"
    o = K.attention_d512(qkv[..., :512], qkv[..., 512:1024], qkv[..., 1024:], 512 ** -0.5)
    os.environ.pop("RDMI_D512_W4")
    print(f"d512w4 B={B} S={S}: {fp(o)}", flush=True)
for mode, env in (("f32", {"RDMI_F32_X3": "0"}), ("x3", {"RDMI_F32_X3": "1"}), ("x6", {"RDMI_F32_X3": "conv"})):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    for B, S, H in ((2, 6912, 5), (3, 1000, 10), (2, 77, 2)):
        C = 64 * H
        qkv = torch.randn(B, S, 3 * C, device="cuda", generator=g) * 1.5
        o = K.attention(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], H)
        print(f"{mode} B={B} S={S} H={H}: {fp(o)}", flush=True)
    for k_, v_ in old.items():
        if v_ is None:
            os.environ.pop(k_)
        else:
            os.environ[k_] = v_
