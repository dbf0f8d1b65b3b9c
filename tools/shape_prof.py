"""Per-launch-shape time table of one fast-preset forward (implicit GEMM / conv / attention),
timed with HIP events on the launch stream: where the step's time goes, by shape.

    RDMI_PROF_SHAPES=1 python tools/shape_prof.py [--frames 100] [--res 768] [--top 40]"""
import argparse
import os
import sys

os.environ.setdefault("RDMI_PROF_SHAPES", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import config as C  # noqa: E402
from rollingdepth_amd import kernels as K  # noqa: E402
from rollingdepth_amd import weights as W  # noqa: E402
from rollingdepth_amd.pipeline import RollingDepthPipeline  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=100)
ap.add_argument("--res", type=int, default=768)
ap.add_argument("--top", type=int, default=45)
ap.add_argument("--snippet-batch", type=int, default=8)
a = ap.parse_args()
pipe = RollingDepthPipeline.from_synthetic(C.SD2_UNET, C.SD2_VAE, C.RD_SCHEDULER, device="cuda")
pipe.snippet_batch = a.snippet_batch
frames = W.synth_frames(a.frames, a.res, a.res, seed=0)[None].to("cuda", torch.float16)
noise = W.synth_noise(a.res // 8, a.res // 8).to("cuda")
run = lambda: pipe.forward(frames, [1, 25], True, [3], [1], [1], {"num_iterations": 10}, 0, 3, 6, None,  # noqa: E731
                           False, 4, False, init_noise=noise)
run()
torch.cuda.synchronize()
K.profile_start()
run()
prof = K.profile_stop()
tot = sum(v["ms"] for v in prof.values())
print(f"timed kernels: {tot:.1f} ms")
for name, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"])[: a.top]:
    print(f"{v['ms']:9.1f} ms {100 * v['ms'] / tot:5.1f}% {v['n']:5d} x {v['flop'] / (v['ms'] * 1e-3) / 1e12:7.1f} TF/s  {name}")
