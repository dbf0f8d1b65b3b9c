"""The reference's own CPU path against the oracle port, same threads, this container (build host only:
the reference never travels to the GPU box).  configs[0]: one 3-frame 256x256 snippet, SD2-shaped random
weights, dilation [1], 1 DDIM step, 2000-iteration aligner, fp32 — `RollingDepthPipeline.forward` of
/root/reference (diffusers 0.30 vendored, loaded by tests/golden/_refload.py) and `oracle.rd_oracle.
pipeline_forward` (what bench.py's cpu_baseline times), each median of 3 after a warm-up.

    python tools/ref_cpu_baseline.py [--threads 8]"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--threads", type=int, default=len(os.sched_getaffinity(0)))
ap.add_argument("--runs", type=int, default=3)
a = ap.parse_args()
torch.set_num_threads(a.threads)

import make_golden as G  # noqa: E402  (imports _refload: the reference's modules, read-only)
from oracle import rd_oracle as O  # noqa: E402
from rollingdepth_amd import config as C  # noqa: E402
from rollingdepth_amd import weights as W  # noqa: E402

P, _ = G._refload.load_reference()
frames = W.synth_frames(3, 256, 256, seed=0)
pipe = G.build_pipe(P, C.SD2_UNET, C.SD2_VAE, C.RD_SCHEDULER)
usd = W.synth_state_dict(W.unet_param_shapes(C.SD2_UNET))
vsd = W.synth_state_dict(W.vae_param_shapes(C.SD2_VAE))
ctx = W.synth_context(1024)
noise = W.synth_noise(32, 32)


def ref():
    g = torch.Generator().manual_seed(0)
    with torch.no_grad():
        t0 = time.perf_counter()
        pipe.forward(input_frames=frames[None], dilations=[1], cap_dilation=False, snippet_lengths=[3],
                     init_infer_steps=[1], strides=[1], coalign_kwargs=None, refine_step=0, refine_snippet_len=3,
                     refine_start_dilation=6, generator=g, verbose=False, max_vae_bs=4, unload_snippet=False)
        return time.perf_counter() - t0


def port():
    with torch.no_grad():
        t0 = time.perf_counter()
        O.pipeline_forward(usd, C.SD2_UNET, vsd, C.SD2_VAE, C.RD_SCHEDULER, frames, noise, ctx, [1], False)
        return time.perf_counter() - t0


for name, fn in (("reference RollingDepthPipeline.forward (CPU, fp32)", ref), ("oracle port (bench.py cpu_baseline)", port)):
    fn()
    ts = [fn() for _ in range(a.runs)]
    m = statistics.median(ts)
    print(f"{name}: median {m:.2f} s = {3.0 / m:.3f} depth frames/s on {a.threads} threads "
          f"(runs {', '.join(f'{t:.2f}' for t in ts)})", flush=True)
