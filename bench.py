"""Benchmark: RollingDepth snippet-denoise hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--preset fast|fast1024|full|paper]
                    [--frames F | --frames-total T] [--res R] [--dilations 1,25]
    torchrun --nproc-per-node N bench.py --gpus N ...      (driver form, one rank per GPU)

`--gpus N` without a torchrun environment re-launches this script under torch.distributed.run with
N ranks (before anything touches the GPU) and exits with its status; under torchrun, WORLD_SIZE must
equal --gpus or the bench exits non-zero.

Workload (default = BASELINE.json configs[1], the "fast" preset): synthetic 768×768 RGB video,
dilations [1,25] (cap_dilation=True), snippet length 3, 1-step DDIM, fp16, no refine; SD2-shaped UNet
(866 M) + KL-f8 VAE with random-init weights (no checkpoint offline).  Strong scaling by default: one
100-frame video (the paper preset: 500 frames) split over the N GPUs — the multi-GPU question of
BASELINE.json configs[4] is how fast one video gets done; `--frames F` runs F frames per GPU instead
(weak scaling).  (With dilations [1, 25] the work per frame grows with the video length — the d = 25
snippet count is N − 52 — so a weak-scaling curve mixes that growth with the communication cost:
the algorithm alone caps 8-GPU weak-scaling efficiency near 0.77)  One step = the whole forward over the video (encode,
every snippet's UNet step + 3 VAE decodes, 2000-iteration DepthAligner, merge, renormalise, refine
when the preset has it) with the frames already resident in HBM, outputs copied to pinned host
memory; at N > 1 shard.sharded_forward (snippet data parallel over RCCL).  value = frames processed
by all ranks / max over ranks of the timed wall time.

After the timed steps the output is validated (non-zero exit otherwise): depth finite and
renormalised to [-1, 1], and the first snippet re-run alone (batch 1, its own 3-frame encode) must
match the batched result within the north_star depth bound (mean |Δ| ≤ 1e-3).

Extra JSON fields: `roofline` for the dominant kernel family by summed time (achieved = algorithmic
FLOPs of every launch of that family in the timed steps ÷ their summed HIP-event durations, events
recorded on the launch stream), with the fused attention reported beside it (`roofline.attention`);
`roofline.traffic` = HBM bytes per launch of that family from the committed rocprofv3 PMC passes over
one step of the same preset (bench_traffic.json, tools/pmc_bench.sh), beside the algorithmic
bytes per launch (every operand read once, output written once) measured here;
`cpu_baseline`: the CPU oracle (oracle/rd_oracle.py, fp32 PyTorch restatement of the reference
pipeline, pinned to reference golden vectors) on this host — BASELINE configs[0] (3 frames 256²),
median of 3 after a warm-up, plus one 3-frame 768² snippet.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_F16_TFLOPS = 2500.0  # MI355X dense f16/bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3   # MI355X f32-input MFMA (= f32 vector peak)
# the bf16-split f32 engine (RDMI_F32_X3) spends three bf16 MFMA products per f32 multiply-add: its
# ceiling in f32 flops is the bf16 peak / 3
PEAK_F32X3_TFLOPS = PEAK_F16_TFLOPS / 3
PEAK_F32X6_TFLOPS = PEAK_F16_TFLOPS / 6  # the three-way split (RDMI_F32_X6): six bf16 products per f32 MAC
PEAK_HBM_GBS = 8000.0

# run_video.py:413-452 presets (BASELINE.json configs[1..4])
PRESETS = {
    "fast": dict(res=768, dilations=[1, 25], refine=0, cap=True, dtype="f16", frames=None, frames_total=100),
    "fast1024": dict(res=1024, dilations=[1, 25], refine=0, cap=True, dtype="f16", frames=None, frames_total=100),
    "full": dict(res=1024, dilations=[1, 10, 25], refine=10, cap=True, dtype="f16", frames=None, frames_total=100),
    "paper": dict(res=768, dilations=[1, 10, 25], refine=10, cap=False, dtype="f32", frames=None,
                  frames_total=500),
}


def _cpu_threads() -> int:
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    # the pool gives a GPU box a share of its host cores and says so in OMP_NUM_THREADS
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def _cpu_baseline(runs_768: int):
    """Oracle forward (fp32, all granted host threads): configs[0] = one 3-frame 256² snippet,
    dilation [1], 1 step, 2000-iteration aligner — median of 3 after one warm-up — and one 3-frame
    768² snippet (`runs_768` runs, median)."""
    import torch

    from oracle import rd_oracle as O
    from rollingdepth_amd import config as C
    from rollingdepth_amd import weights as W

    nthreads = _cpu_threads()
    torch.set_num_threads(nthreads)
    usd = W.synth_state_dict(W.unet_param_shapes(C.SD2_UNET))
    vsd = W.synth_state_dict(W.vae_param_shapes(C.SD2_VAE))
    ctx = W.synth_context(1024)

    def run(res):
        frames = W.synth_frames(3, res, res, seed=0)
        noise = W.synth_noise(res // 8, res // 8)
        with torch.no_grad():
            t0 = time.perf_counter()
            O.pipeline_forward(usd, C.SD2_UNET, vsd, C.SD2_VAE, C.RD_SCHEDULER, frames, noise, ctx, [1], False)
            return time.perf_counter() - t0

    run(256)  # warm-up
    t256 = [run(256) for _ in range(3)]
    t768 = [run(768) for _ in range(runs_768)]
    cpu = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    m256 = statistics.median(t256)
    out = {"value": round(3.0 / m256, 4), "unit": "depth frames/s", "cores": nthreads, "kind": "port",
           "sample": f"oracle fp32 RollingDepth forward (CPU restatement pinned to reference goldens), 3 frames "
                     f"256x256, dilation [1], 1 step, 2000-it aligner: median of 3 after a warm-up "
                     f"{m256:.2f} s (runs {', '.join(f'{t:.2f}' for t in t256)}) on {nthreads} threads ({cpu})"}
    if t768:
        m768 = statistics.median(t768)
        out["value_768"] = round(3.0 / m768, 5)
        out["sample_768"] = f"one 3-frame 768x768 snippet, same path: {m768:.1f} s ({len(t768)} run(s))"
    return out


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _relaunch(n: int) -> int:
    """Start N ranks under torch.distributed.run as a child (never exec from this process)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def _pmc_traffic(preset: str, family: str):
    """HBM bytes per launch of `family` from the committed PMC passes over this preset's bench step
    (tools/pmc_bench.sh → tools/bench_traffic.py → bench_traffic.json; the per-kernel table is
    profiles/r02_pmc_bench_fast.txt), or None."""
    f = os.path.join(ROOT, "bench_traffic.json")
    try:
        ent = json.load(open(f))[preset]
        fam = ent["families"][family]
    except (OSError, KeyError, ValueError):
        return None
    return {"bytes_per_launch": fam["bytes_per_launch"], "source": ent["source"]}


def _validate(pipe, frames_dev, noise, dil0, snippet0, depth_host, coaligned_host, whole=True) -> dict:
    """Output checks after the timed steps; raises on failure.  The co-aligned depth is renormalised
    to [-1, 1] (rollingdepth_pipeline.py:315-317); the refined depth_pred is a decoder output and is
    not (:336-342), so only its finiteness is checked.  whole=False: a rank's frame range, which
    need not reach both ends of the range."""
    import torch

    d = depth_host.float()
    if not torch.isfinite(d).all():
        raise RuntimeError("bench validation: depth_pred has non-finite values")
    c = coaligned_host.float()
    if not torch.isfinite(c).all():
        raise RuntimeError("bench validation: depth_coaligned has non-finite values")
    lo, hi = c.min().item(), c.max().item()
    if lo < -1.0 - 1e-3 or hi > 1.0 + 1e-3 or (whole and min(-lo, hi) < 1.0 - 1e-3):
        raise RuntimeError(f"bench validation: depth_coaligned range [{lo}, {hi}] is not [-1, 1]")
    info = {"depth_finite": True, "coaligned_range": [round(lo, 4), round(hi, 4)],
            "depth_range": [round(d.min().item(), 4), round(d.max().item(), 4)]}
    if snippet0 is None:
        return info
    # re-run the first snippet of dilation 1 alone: frames 0..2, 1 snippet per UNet call, 3-frame encode
    lat = pipe.encode_rgb(frames_dev[:3])
    nz = pipe._noise_nhwc(noise, lat.shape[1], lat.shape[2])
    sb = pipe.snippet_batch
    pipe.snippet_batch = 1
    try:
        again = pipe.init_snippet_infer(lat, nz, [1], [3], [1], [1])[0][0]
    finally:
        pipe.snippet_batch = sb
    a, b = again.float().cpu(), snippet0.float().cpu().reshape(again.shape)
    if not torch.isfinite(b).all():
        raise RuntimeError("bench validation: decoded snippets have non-finite values")
    diff = (a - b).abs()
    mean, mx, ref = diff.mean().item(), diff.max().item(), b.abs().max().item()
    info.update(snippet0_rerun_mean_abs=float(f"{mean:.3e}"), snippet0_rerun_max_abs=float(f"{mx:.3e}"))
    if not (mean <= 1e-3 and mx <= 5e-2 * max(ref, 1e-6)):
        raise RuntimeError(f"bench validation: batch-1 re-run of snippet 0 differs (mean {mean:.2e}, max {mx:.2e})")
    return info


# Collective cost model for the rank-slice prediction (an assumption, stated with the numbers): RCCL over
# xGMI, 7 links per MI355X; all-gathers and the merge all-to-all move each rank's share over several links
# at once.  A deliberately conservative aggregate per GPU and a fixed cost per collective.
SLICE_XGMI_GBS = 100.0
SLICE_COLL_US = 50.0


def _slice_main(a) -> int:
    """bench.py --slice-world W[,W..]: for each W and each rank r < W, run exactly rank r's work of the
    W-rank strong-scaling forward (shard.sharded_forward with shard.SliceGroup: its encode chunk, its
    snippets' UNet steps and decodes, the replicated aligner, its windowed partial merge, its egress;
    collectives replaced by local no-ops) on this one GPU, timed per phase with HIP events; beside it the
    single-GPU step of the same preset.  Prints one JSON line per W: per-rank step times, phases, the
    predicted W-GPU step = max over ranks + a collective model (SLICE_XGMI_GBS, SLICE_COLL_US), and the
    predicted efficiency T1 / (W · T_W).  Not a scaling number: nothing here ran on W GPUs."""
    import torch

    from rollingdepth_amd import config as C
    from rollingdepth_amd import weights as W
    from rollingdepth_amd.pipeline import RollingDepthPipeline
    from rollingdepth_amd.shard import SliceGroup, chunk_bounds, merge_exchange_plan, rank_subsets, sharded_forward

    pr = dict(PRESETS[a.preset])
    res = a.res or pr["res"]
    dil0 = [int(x) for x in a.dilations.split(",")] if a.dilations else list(pr["dilations"])
    N = a.frames_total or pr["frames_total"]
    dev = torch.device("cuda", 0)
    tdt = torch.float32 if pr["dtype"] == "f32" else torch.float16
    pipe = RollingDepthPipeline.from_synthetic(C.SD2_UNET, C.SD2_VAE, C.RD_SCHEDULER, device=dev, torch_dtype=tdt)
    pipe.snippet_batch = a.snippet_batch
    pipe.vae_batch = a.vae_batch
    frames_all = W.synth_frames(N, res, res, seed=0)
    noise = W.synth_noise(res // 8, res // 8).to(dev)
    coalign = {"num_iterations": a.aligner_iters}
    refine = pr["refine"]

    # single-GPU reference step (the same forward bench.py times at N = 1)
    f1dev = frames_all[None].to(dev, tdt)

    def one():
        pipe.forward(f1dev, list(dil0), pr["cap"], [3], [1], [1], coalign, refine, 3, 6, None, False, 4, False,
                     init_noise=noise)

    for _ in range(a.warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one()
    torch.cuda.synchronize()
    t1 = (time.perf_counter() - t0) / a.steps
    del f1dev
    print(f"single-GPU step {t1 * 1e3:.1f} ms ({N / t1:.2f} depth frames/s)", flush=True)

    dil = [pipe.cap_max_dilation(N, 3, d) for d in dil0] if pr["cap"] else list(dil0)
    counts = [len(pipe.get_snippet_indice(0, [0], N, 3, d, d, 1)) for d in dil]
    h = res // 8
    P = ((res - 4 + 9) // 10) ** 2  # aligner inputs: border 2, every 10th pixel (depth_aligner.py:82-92)
    for Wd in [int(x) for x in a.slice_world.split(",")]:
        ranks = []
        for r in range(Wd):
            lo, hi = chunk_bounds(N, Wd)[r]
            fr = frames_all[lo:hi].to(dev, tdt)
            g = SliceGroup(r, Wd)

            def step(timing=None):
                sharded_forward(pipe, fr, list(dil0), pr["cap"], 3, coalign, init_noise=noise, num_frames=N,
                                to_host=True, refine_step=refine, group=g, timing=timing)

            for _ in range(a.warmup):
                step()
            torch.cuda.synchronize()
            phases, walls = {}, []
            for _ in range(a.steps):
                tm = []
                ts = time.perf_counter()
                step(tm)
                torch.cuda.synchronize()
                walls.append(time.perf_counter() - ts)
                for (n0, e0), (n1, e1) in zip(tm, tm[1:]):
                    phases[n1] = phases.get(n1, 0.0) + e0.elapsed_time(e1) / a.steps
            sub = rank_subsets(counts, Wd, r)
            rng_, send, recv = merge_exchange_plan(counts, dil, [3] * len(dil), N, Wd, r)
            nrecv = [sum(m for _, m in pc) for pc in recv]
            ranks.append({"rank": r, "ms": round(statistics.median(walls) * 1e3, 1),
                          "phases_ms": {k: round(v, 1) for k, v in phases.items()},
                          "frames": hi - lo, "snippets": [len(x) for x in sub], "merge_frames": rng_,
                          "merge_rows_sent": sum(send) - send[r], "merge_rows_recv": sum(nrecv) - nrecv[r]})
            del fr
            print(f"W={Wd} rank {r}: {ranks[-1]['ms']} ms {ranks[-1]['phases_ms']}", flush=True)
        # collective model: latents + aligner-input all-gathers, the merge all-to-all, two min/max all-reduces
        esz = 2 if tdt == torch.float16 else 4
        lat_b = (Wd - 1) / Wd * N * h * h * 8 * esz
        ali_b = (Wd - 1) / Wd * sum(counts) * 3 * P * 4
        m_rows = max(max(x["merge_rows_sent"], x["merge_rows_recv"]) for x in ranks)
        merge_b = m_rows * res * res * 8
        n_coll = 5 + (2 * refine if refine else 0)
        ref_b = (2 * (Wd - 1) / Wd * N * h * h * 4 * 8 * refine + (Wd - 1) / Wd * N * h * h * 8 * esz) if refine else 0
        comm_s = (lat_b + ali_b + merge_b + ref_b) / (SLICE_XGMI_GBS * 1e9) + n_coll * SLICE_COLL_US * 1e-6
        tmax = max(x["ms"] for x in ranks) * 1e-3
        tw = tmax + comm_s
        line = {"mode": "rank-slice", "note": "not a scaling number: each rank's share of a W-rank run timed "
                                              "alone on one GPU, collectives modelled",
                "preset": a.preset, "frames": N, "res": res, "dilations": dil, "world": Wd,
                "single_gpu_ms": round(t1 * 1e3, 1), "ideal_ms": round(t1 / Wd * 1e3, 1),
                "max_rank_ms": round(tmax * 1e3, 1), "comm_model_ms": round(comm_s * 1e3, 2),
                "comm_model": f"{SLICE_XGMI_GBS:.0f} GB/s per GPU + {SLICE_COLL_US:.0f} us per collective: "
                              f"latents {lat_b / 1e6:.1f} MB, aligner inputs {ali_b / 1e6:.1f} MB, merge "
                              f"{merge_b / 1e6:.1f} MB, refine {ref_b / 1e6:.1f} MB",
                "predicted_ms": round(tw * 1e3, 1), "predicted_efficiency": round(t1 / (Wd * tw), 4),
                "predicted_depth_frames_per_s": round(N / tw, 2), "ranks": ranks}
        print(json.dumps(line), flush=True)
    return 0


def _rank_times(marks, colls, steps: int, rank: int, wall_s: float) -> dict:
    """This rank's per-phase and per-collective times over the timed steps (ms per step, HIP events on
    the launch stream): phases between shard.sharded_forward's marks (encode, snippets, prepare,
    aligner, merge, refine, egress); collectives summed by kind (all_gather / all_reduce / broadcast /
    all_to_all) with their count and bytes per step, each span including any wait for the slowest rank."""
    phases = {}
    for tm in marks:
        for (_, e0), (n1, e1) in zip(tm, tm[1:]):
            phases[n1] = phases.get(n1, 0.0) + e0.elapsed_time(e1) / steps
    coll = {}
    for kind, e0, e1, nb in colls:
        c = coll.setdefault(kind, {"ms": 0.0, "count": 0, "mbytes": 0.0})
        c["ms"] += e0.elapsed_time(e1) / steps
        c["count"] += 1
        c["mbytes"] += nb / 1e6
    for c in coll.values():
        c["ms"] = round(c["ms"], 2)
        c["count"] = c["count"] // steps
        c["mbytes"] = round(c["mbytes"] / steps, 2)
    return {"rank": rank, "wall_ms_per_step": round(wall_s / steps * 1e3, 1),
            "phases_ms": {k: round(v, 1) for k, v in phases.items()}, "collectives": coll}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--preset", default="fast", choices=sorted(PRESETS))
    ap.add_argument("--frames", type=int, default=None, help="frames per GPU (weak scaling)")
    ap.add_argument("--frames-total", type=int, default=None, help="total frames (strong scaling)")
    ap.add_argument("--res", type=int, default=None)
    ap.add_argument("--dilations", default=None)
    # snippets per UNet call, a cap (balanced batches, pipeline._snippet_batches): 25 measured
    # 20.9 depth frames/s vs 20.6 at 16 (16/16 had measured +4.5 % over 8/8)
    ap.add_argument("--snippet-batch", type=int, default=25)
    ap.add_argument("--vae-batch", type=int, default=75)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-768-runs", type=int, default=1)
    ap.add_argument("--no-validate", action="store_true")
    ap.add_argument("--aligner-iters", type=int, default=2000)
    ap.add_argument("--slice-world", default=None,
                    help="e.g. 2,4,8: on ONE GPU, time each rank's share of a W-rank run (collectives as local "
                         "no-ops, shard.SliceGroup) beside the single-GPU step — not a scaling number")
    a = ap.parse_args()
    if a.slice_world:
        sys.exit(_slice_main(a))

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and a.gpus > 1:
        sys.exit(_relaunch(a.gpus))
    world = int(world_env or "1")
    if world != a.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank path on a one-GPU box: every rank on cuda:0, gloo collectives
    # (the scaling runs themselves use one GPU per rank and RCCL)
    shared = os.environ.get("RDMI_BENCH_SHARED_GPU") == "1"
    if shared:
        local = 0

    import torch
    import torch.distributed as dist

    pr = dict(PRESETS[a.preset])
    res = a.res or pr["res"]
    dil0 = [int(x) for x in a.dilations.split(",")] if a.dilations else list(pr["dilations"])
    if a.frames is not None:
        N = a.frames * world
        scaling = "weak"
    else:
        N = a.frames_total or pr["frames_total"]
        scaling = "strong"

    if world > 1:
        torch.cuda.set_device(local)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from rollingdepth_amd import config as C
    from rollingdepth_amd import kernels as K
    from rollingdepth_amd import weights as W
    from rollingdepth_amd.pipeline import RollingDepthPipeline
    from rollingdepth_amd.shard import chunk_bounds, sharded_forward

    tdt = torch.float32 if pr["dtype"] == "f32" else torch.float16
    pipe = RollingDepthPipeline.from_synthetic(C.SD2_UNET, C.SD2_VAE, C.RD_SCHEDULER, device=dev, torch_dtype=tdt)
    pipe.snippet_batch = a.snippet_batch
    pipe.vae_batch = a.vae_batch
    if world > 1:  # each rank materialises only its own chunk of the synthetic video
        lo, hi = chunk_bounds(N, world)[rank]
        frames = W.synth_frames(N, res, res, seed=0, first=lo, count=hi - lo).to(dev, tdt)
    else:
        frames = W.synth_frames(N, res, res, seed=0)[None].to(dev, tdt)
    noise = W.synth_noise(res // 8, res // 8).to(dev)
    coalign = {"num_iterations": a.aligner_iters}
    refine = pr["refine"]
    last = {}

    def step(timing=None):
        if world > 1:
            so = sharded_forward(pipe, frames, list(dil0), pr["cap"], 3, coalign, init_noise=noise, num_frames=N,
                                 to_host=True, refine_step=refine, timing=timing)
            last["depth"] = so.depth_pred
            last["coaligned"] = so.depth_coaligned
            last["snip0"] = so.snippet_rows[0][0] if rank == 0 and so.snippet_rows[0].shape[0] else None
            return
        out = pipe.forward(frames, list(dil0), pr["cap"], [3], [1], [1], coalign, refine, 3, 6, None, False, 4,
                           False, init_noise=noise)
        last["depth"] = out.depth_pred
        last["coaligned"] = out.depth_coaligned
        last["snip0"] = out.snippet_ls[0][0]

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    K.profile_start()
    marks = [[] for _ in range(a.steps)] if world > 1 else None
    if world > 1:
        import rollingdepth_amd.shard as S
        S.collective_timing = []
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(marks[i] if marks else None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = K.profile_stop()
    per_rank = None
    if world > 1:
        per_rank = _rank_times(marks, S.collective_timing, a.steps, rank, dt)
        S.collective_timing = None
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
        gathered = [None] * world
        dist.all_gather_object(gathered, per_rank)
        per_rank = gathered
    validation = None
    if not a.no_validate:
        try:
            vframes = frames if world > 1 else frames[0]
            validation = _validate(pipe, vframes, noise, dil0, last["snip0"] if rank == 0 else None, last["depth"],
                                   last["coaligned"], whole=world == 1)
            ok = 1
        except Exception as e:  # noqa: BLE001 — reported, then non-zero exit
            print(f"rank {rank}: {e}", file=sys.stderr, flush=True)
            ok = 0
        if world > 1:
            t = torch.tensor([ok], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ok = int(t.item())
        if not ok:
            sys.exit(3)
    total_frames = N * a.steps
    roof = None
    if prof:
        def _fam(name):
            p = prof[name]
            return p["flop"] / (p["ms"] * 1e-3) / 1e12

        dom = max(prof, key=lambda k: prof[k]["ms"])
        p = prof[dom]
        ach = _fam(dom)
        peak = (PEAK_F32_TFLOPS if dom.endswith("_f32") else PEAK_F32X3_TFLOPS if dom.endswith("_f32x3")
                else PEAK_F32X6_TFLOPS if dom.endswith("_f32x6") else PEAK_F16_TFLOPS)
        tr = _pmc_traffic(a.preset, dom)
        roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 1), "peak": peak, "unit": "TFLOP/s",
                "frac": round(ach / peak, 4), "traffic": tr and round(tr["bytes_per_launch"]),
                "algorithmic_bytes_per_launch": round(p["bytes"] / max(p["n"], 1)),
                "traffic_source": tr and tr["source"], "launches": p["n"],
                "avg_launch_us": round(p["ms"] * 1e3 / max(p["n"], 1), 2),
                "per_kernel": {k: {"tflops": round(_fam(k), 1), "ms": round(v["ms"], 1), "launches": v["n"]}
                               for k, v in prof.items()}}
        for an, apk in (("attention_fwd", PEAK_F16_TFLOPS), ("attention_fwd_f32", PEAK_F32_TFLOPS),
                        ("attention_fwd_f32x3", PEAK_F32X3_TFLOPS), ("attention_fwd_f32x6", PEAK_F32X6_TFLOPS)):
            if an in prof:
                att = _fam(an)
                roof["attention"] = {"kernel": an, "achieved": round(att, 1), "peak": apk, "unit": "TFLOP/s",
                                     "frac": round(att / apk, 4)}
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:  # the CPU leg is an N = 1 figure
        cpu = _cpu_baseline(a.cpu_768_runs)
    if rank == 0:
        line = {
            "metric": "depth frames/sec at 768px snip_len=3, 1-step denoise; 1/2/4/8 MI355X",
            "value": round(total_frames / dt, 4), "unit": "depth frames/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 1), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "data": "synthetic",
            "dtype": pr["dtype"] + (f" ({K.f32_precision_label()})" if pr["dtype"] == "f32" else ""),
            "config": {"workload": f"{a.preset} preset: {N}-frame {res}x{res} video, dilations {dil0} "
                                   f"(cap_dilation={pr['cap']}), snippet_len 3, 1-step DDIM, aligner "
                                   f"{a.aligner_iters} it, refine {refine}; SD2-shaped UNet+VAE random-init",
                       "preset": a.preset, "frames": N, "res": res, "dilations": dil0,
                       "parallelism": f"snippet-dp{world}"},
            "roofline": roof, "cpu_baseline": cpu, "validation": validation,
        }
        if per_rank is not None:
            line["per_rank"] = per_rank
        if shared:
            line["rehearsal"] = "RDMI_BENCH_SHARED_GPU=1: all ranks on one GPU over gloo (not a scaling number)"
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
