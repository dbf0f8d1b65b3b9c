"""A/B of the snippet decode on a second stream (RollingDepthPipeline.decode_stream, RDMI_DECODE_STREAM):
bitwise comparison of the forward's outputs, then interleaved wall-clock timing of the fast preset's
forward (frames resident in HBM, as bench.py), both modes in one process.

    python tools/decode_stream_ab.py [--frames 100] [--rounds 3] [--steps 2]"""
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
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--res", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    pipe = RollingDepthPipeline.from_synthetic(C.SD2_UNET, C.SD2_VAE, C.RD_SCHEDULER, device=dev)
    frames = W.synth_frames(a.frames, a.res, a.res, seed=0)[None].to(dev, torch.float16)
    noise = W.synth_noise(a.res // 8, a.res // 8).to(dev)

    def fwd():
        return pipe.forward(frames, [1, 25], True, [3], [1], [1], None, 0, 3, 6, None, False, 4, False,
                            init_noise=noise)

    outs = {}
    for mode in (False, True):
        pipe.decode_stream = mode
        o = fwd()
        torch.cuda.synchronize()
        outs[mode] = (o.depth_pred.clone(), torch.cat([s.reshape(-1) for s in o.snippet_ls]).clone())
    same = all(torch.equal(x, y) for x, y in zip(outs[False], outs[True]))
    print(f"decode stream outputs bitwise equal to the serial forward: {same}", flush=True)
    for r in range(a.rounds):
        for mode in (False, True):
            pipe.decode_stream = mode
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                fwd()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps
            print(f"round {r} decode_stream={int(mode)}: {dt * 1e3:8.1f} ms  {a.frames / dt:6.2f} depth frames/s",
                  flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
