"""Benchmark: RollingDepth snippet-denoise hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames F] [--res R] [--dilations 1,25]
    torchrun --nproc-per-node N bench.py --gpus N ...      (driver form, one rank per GPU)

Workload (BASELINE.json configs[1], "fast" preset): synthetic 768×768 RGB video of F=100 frames
per GPU (weak scaling: F·N frames at N GPUs), dilations [1,25] (cap_dilation=True), snippet
length 3, 1-step DDIM, fp16, no refine; SD2-shaped UNet (866 M) + KL-f8 VAE with random-init
weights (no checkpoint offline).  One step = RollingDepthPipeline.forward over the whole video
(encode, every snippet's UNet step + 3 VAE decodes, 2000-iteration DepthAligner, merge,
renormalise) with frames already resident in HBM.  value = frames processed by all ranks / max
over ranks of the timed wall time.

Extra JSON fields: `roofline` for the dominant kernel (the implicit-GEMM conv/linear kernel or the
fused attention, whichever has more total time) — achieved = algorithmic FLOPs of every launch of
that kernel in the timed steps ÷ their summed HIP-event durations (events recorded on the launch
stream) — and `cpu_baseline`: the CPU oracle (oracle/rd_oracle.py, fp32 PyTorch restatement of
the reference pipeline, pinned to reference golden vectors) timed on this host on a bounded
sample: one 3-frame 256² snippet (BASELINE configs[0]).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_F16_TFLOPS = 2500.0  # MI355X dense f16/bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def _cpu_baseline():
    """Oracle forward on a 3-frame 256² snippet (configs[0]), fp32, all host threads."""
    from oracle import rd_oracle as O
    from rollingdepth_amd import config as C
    from rollingdepth_amd import weights as W

    nthreads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    nthreads = min(nthreads, 16)
    torch.set_num_threads(nthreads)
    usd = W.synth_state_dict(W.unet_param_shapes(C.SD2_UNET))
    vsd = W.synth_state_dict(W.vae_param_shapes(C.SD2_VAE))
    frames = W.synth_frames(3, 256, 256, seed=0)
    noise = W.synth_noise(32, 32)
    ctx = W.synth_context(1024)
    with torch.no_grad():
        t0 = time.perf_counter()
        O.pipeline_forward(usd, C.SD2_UNET, vsd, C.SD2_VAE, C.RD_SCHEDULER, frames, noise, ctx, [1], False)
        dt = time.perf_counter() - t0
    cpu = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": 3.0 / dt, "unit": "depth frames/s", "cores": nthreads, "kind": "port",
            "sample": f"oracle fp32 RollingDepth forward, 3 frames 256x256, dilation [1], 1 step, "
                      f"2000-it aligner; {dt:.1f} s on {nthreads} threads ({cpu})"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--frames", type=int, default=100, help="frames per GPU (weak scaling)")
    ap.add_argument("--res", type=int, default=768)
    ap.add_argument("--dilations", default="1,25")
    # snippets per UNet call, a cap (balanced batches, pipeline._snippet_batches): 25 measured
    # 20.9 depth frames/s vs 20.6 at 16 (16/16 had measured +4.5 % over 8/8)
    ap.add_argument("--snippet-batch", type=int, default=25)
    ap.add_argument("--vae-batch", type=int, default=75)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--aligner-iters", type=int, default=2000)
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from rollingdepth_amd import config as C
    from rollingdepth_amd import kernels as K
    from rollingdepth_amd import weights as W
    from rollingdepth_amd.pipeline import RollingDepthPipeline
    from rollingdepth_amd.shard import sharded_forward

    pipe = RollingDepthPipeline.from_synthetic(C.SD2_UNET, C.SD2_VAE, C.RD_SCHEDULER, device=dev)
    pipe.snippet_batch = a.snippet_batch
    pipe.vae_batch = a.vae_batch
    N = a.frames * world
    from rollingdepth_amd.shard import chunk_bounds
    if world > 1:  # each rank materialises only its own chunk of the synthetic video
        lo, hi = chunk_bounds(N, world)[rank]
        frames = W.synth_frames(N, a.res, a.res, seed=0, first=lo, count=hi - lo).to(dev, torch.float16)
    else:
        frames = W.synth_frames(N, a.res, a.res, seed=0)[None].to(dev, torch.float16)
    noise = W.synth_noise(a.res // 8, a.res // 8).to(dev)
    dil0 = [int(x) for x in a.dilations.split(",")]
    coalign = {"num_iterations": a.aligner_iters}

    def step():
        if world > 1:
            return sharded_forward(pipe, frames, list(dil0), True, 3, coalign, init_noise=noise, num_frames=N,
                                   to_host=True)
        return pipe.forward(frames, list(dil0), True, [3], [1], [1], coalign, 0, 3, 6, None, False, 4, False,
                            init_noise=noise)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    K.profile_start()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = K.profile_stop()
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
    total_frames = N * a.steps
    # roofline of the dominant kernel (by summed event time)
    dom = max(prof, key=lambda k: prof[k]["ms"]) if prof else None
    roof = None
    if dom:
        p = prof[dom]
        ach = p["flop"] / (p["ms"] * 1e-3) / 1e12
        roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 1), "peak": PEAK_F16_TFLOPS,
                "unit": "TFLOP/s", "frac": round(ach / PEAK_F16_TFLOPS, 4), "traffic": None,
                "launches": p["n"], "avg_launch_us": round(p["ms"] * 1e3 / max(p["n"], 1), 2),
                "per_kernel": {k: {"tflops": round(v["flop"] / (v["ms"] * 1e-3) / 1e12, 1),
                                   "ms": round(v["ms"], 1), "launches": v["n"]} for k, v in prof.items()}}
    cpu = None
    if rank == 0 and not a.no_cpu_baseline:
        cpu = _cpu_baseline()
    if rank == 0:
        line = {
            "metric": "depth frames/sec at 768px snip_len=3, 1-step denoise; 1/2/4/8 MI355X",
            "value": round(total_frames / dt, 4), "unit": "depth frames/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 1), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f16", "data": "synthetic",
            "config": {"workload": f"fast preset: {N}-frame {a.res}x{a.res} video, dilations {dil0} "
                                   f"(cap_dilation), snippet_len 3, 1-step DDIM, aligner {a.aligner_iters} it, "
                                   f"no refine; SD2-shaped UNet+VAE random-init",
                       "frames": N, "res": a.res, "dilations": dil0, "parallelism": f"snippet-dp{world}"},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
