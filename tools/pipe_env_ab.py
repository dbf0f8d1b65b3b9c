"""Interleaved pipeline A/B of a switch the host code reads per call (an RDMI_* variable such as
RDMI_GN_FUSE): the fast preset's forward (frames resident in HBM, as bench.py) under each value in one
process, outputs compared bitwise first, then timed in alternating rounds.

    python tools/pipe_env_ab.py --var RDMI_GN_FUSE --values 3,1 [--frames 100] [--rounds 3] [--steps 2]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rollingdepth_amd import config as C  # noqa: E402
from rollingdepth_amd import weights as W  # noqa: E402
from rollingdepth_amd.pipeline import RollingDepthPipeline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--var", required=True)
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--res", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    vals = a.values.split(",")
    dev = torch.device("cuda", 0)
    pipe = RollingDepthPipeline.from_synthetic(C.SD2_UNET, C.SD2_VAE, C.RD_SCHEDULER, device=dev)
    frames = W.synth_frames(a.frames, a.res, a.res, seed=0)[None].to(dev, torch.float16)
    noise = W.synth_noise(a.res // 8, a.res // 8).to(dev)

    def fwd():
        return pipe.forward(frames, [1, 25], True, [3], [1], [1], None, 0, 3, 6, None, False, 4, False,
                            init_noise=noise)

    outs = {}
    for v in vals:
        os.environ[a.var] = v
        o = fwd()
        torch.cuda.synchronize()
        outs[v] = (o.depth_pred.clone(), torch.cat([s.reshape(-1) for s in o.snippet_ls]).clone())
    same = all(torch.equal(x, y) for x, y in zip(outs[vals[0]], outs[vals[-1]]))
    print(f"{a.var} {vals}: outputs bitwise equal: {same}", flush=True)
    for r in range(a.rounds):
        for v in vals:
            os.environ[a.var] = v
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                fwd()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps
            print(f"round {r} {a.var}={v}: {dt * 1e3:8.1f} ms  {a.frames / dt:6.2f} depth frames/s", flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
