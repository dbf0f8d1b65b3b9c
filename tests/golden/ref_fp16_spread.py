"""How far the REFERENCE's own fp16 pipeline lands from its fp32 pipeline on the golden inputs.

Context for the depth-parity bar: the fast preset runs the reference in fp16
(run_video.py's dtype), while the goldens of this repository are fp32 runs of the reference.  This
script re-runs the reference pipeline (imported from /root/reference by _refload, build container
only — like make_golden.py it never travels to the GPU box) with the UNet and VAE cast to fp16, on
exactly the golden's inputs (same synthetic weights, frames and init noise — the fp32 noise of the
golden rounded to fp16, as the reference's own fp16 `torch.randn` would differ), and reports the
depth L1 and latent errors against the committed fp32 golden with the metrics the GPU parity tests
use.  CPU fp16 arithmetic (PyTorch's CPU half kernels) is not the reference's GPU fp16 arithmetic,
so this is one sample of "the reference in fp16", not the distribution.

  GOLDEN_THREADS=4 python tests/golden/ref_fp16_spread.py --case sd2_256
  GOLDEN_THREADS=4 python tests/golden/ref_fp16_spread.py --case sd2_768
"""
import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from safetensors.torch import load_file  # noqa: E402

import _refload  # noqa: E402
import make_golden as MG  # noqa: E402
from rollingdepth_amd import config as C  # noqa: E402
from rollingdepth_amd import weights as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="sd2_256", choices=["sd2_256", "sd2_768"])
    a = ap.parse_args()
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", "4")))
    P, _ = _refload.load_reference()
    g = load_file(os.path.join(HERE, a.case + ".safetensors"))
    meta = json.load(open(os.path.join(HERE, a.case + ".json")))
    pipe = MG.build_pipe(P, C.SD2_UNET, C.SD2_VAE, C.RD_SCHEDULER)
    pipe.to(torch.float16)
    pipe.empty_text_embed = pipe.empty_text_embed.to(torch.float16)
    if "frames" in g:
        frames = g["frames"]
    else:
        n, res = meta["n_frames"], meta["res"]
        frames = W.synth_frames(n, res, res, seed=0)
    noise32 = g["init_noise"]
    real_randn = torch.randn

    def randn(*shape, **kw):  # the forward's init noise: the golden's fp32 noise in the run's dtype
        shp = tuple(shape[0]) if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)) else shape
        if shp == tuple(noise32.shape):
            return noise32.to(kw.get("dtype") or torch.float32)
        return real_randn(*shape, **kw)

    torch.randn = randn
    t0 = time.time()
    try:
        out, rec = MG.run_pipe(pipe, frames, meta["dilations_in"], meta["cap_dilation"], 1)
    finally:
        torch.randn = real_randn
    dt = time.time() - t0
    res = {"case": a.case, "threads": torch.get_num_threads(), "seconds": round(dt, 1)}
    dp = out.depth_pred.float()
    dc = out.depth_coaligned.float()
    if "depth_pred" in g:
        res["depth_pred_l1"] = (dp - g["depth_pred"]).abs().mean().item()
        res["depth_coaligned_l1"] = (dc - g["depth_coaligned"]).abs().mean().item()
    else:
        s = meta["depth_stride"]
        res["depth_pred_l1_sub"] = (dp[..., ::s, ::s] - g["depth_pred_sub"].float()).abs().mean().item()
        res["depth_coaligned_l1_sub"] = (dc[..., ::s, ::s] - g["depth_coaligned_sub"].float()).abs().mean().item()
        st = torch.tensor([dp.double().mean().item(), dp.double().abs().mean().item()])
        res["depth_pred_stats_diff"] = (st - g["depth_pred_stats"].double()).abs().tolist()
    u = rec["unet_out"][0]
    gu = g["unet_out_first"].float()
    res["unet_out_rel"] = ((u - gu).norm() / gu.norm()).item()
    lat = rec["snip_lat"][0][0] if "snippet_latent_0_first" in g else rec["snip_lat"][0]
    gl = (g["snippet_latent_0_first"] if "snippet_latent_0_first" in g else g["snippet_latent_0"]).float()
    res["snippet_latent_rel"] = ((lat - gl).norm() / gl.norm()).item()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
