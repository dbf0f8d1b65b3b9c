"""Where does the sharded f16 refine leave the single-GPU refine?  

    python tools/refine_diverge.py [--world 3] [--dtype float16] [--fixture tiny_refine]

Runs the fixture's forward sharded over W gloo ranks sharing the one GPU and single-GPU, recording
the refine's inputs (rgb latents, encoded co-aligned depth latents, noise) and the averaged latents
after every refine step, and prints the first tensor that differs and by how much."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from safetensors.torch import load_file  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")


def _hook(pipe, rec):
    from rollingdepth_amd import kernels as K
    orig_refine = pipe.refine

    def refine(rgb_latent, depth_latents, init_noise, *a, **k):
        rec["rgb_latent"] = rgb_latent.float().cpu()
        rec["dlat"] = depth_latents.float().cpu()
        rec["noise"] = init_noise.float().cpu()
        return orig_refine(rgb_latent, depth_latents, init_noise, *a, **k)

    pipe.refine = refine
    steps = rec.setdefault("steps", [])
    preds = rec.setdefault("preds", [])
    for name in ("snippet_average", "snippet_finish"):
        f = getattr(K, name)

        def wrap(*a, _f=f, **k):
            o = _f(*a, **k)
            steps.append(o.float().cpu())
            return o

        setattr(K, name, wrap)
    fa = K.snippet_accumulate

    def acc(src, *a, **k):
        preds.append(src.float().cpu())
        return fa(src, *a, **k)

    K.snippet_accumulate = acc
    fs = K.snippet_average

    def avg(src, *a, **k):
        preds.append(src.float().cpu())
        return fs(src, *a, **k)

    K.snippet_average = avg


def _pipe(meta, t, dtype):
    from rollingdepth_amd.pipeline import RollingDepthPipeline
    pipe = RollingDepthPipeline.from_synthetic(meta["unet"], meta["vae"], meta["scheduler"], device="cuda",
                                               torch_dtype=dtype)
    pipe.empty_text_embed = t["context"]
    return pipe


def _worker(rank, world, port, fixture, dtype_name, batch):
    import torch.distributed as dist
    from rollingdepth_amd.shard import sharded_forward
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = load_file(os.path.join(G, fixture + ".safetensors"))
    meta = json.load(open(os.path.join(G, fixture + ".json")))
    pipe = _pipe(meta, t, getattr(torch, dtype_name))
    pipe.snippet_batch = batch
    rec = {}
    _hook(pipe, rec)
    so = sharded_forward(pipe, t["frames"][None].cuda(), list(meta["dilations_in"]), True, 3, None,
                         init_noise=t["init_noise"].cuda(), refine_step=meta.get("refine_step", 0),
                         refine_start_dilation=meta.get("refine_start_dilation", 6), gather=True)
    torch.cuda.synchronize()
    rec["coaligned"] = _full(so.depth_coaligned, so, world)
    rec["depth"] = so.depth_pred_full.float().cpu()
    if rank == 0:
        torch.save(rec, os.path.join(ROOT, "gpurun_out", "refdiv_sharded.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _full(local, so, world):
    from rollingdepth_amd.shard import _all_gather_rows
    return _all_gather_rows(local.contiguous(), so.depth_pred_full.shape[0], world).float().cpu()


def _cmp(name, a, b):
    d = (a - b).abs()
    nz = (d > 0).float().mean().item()
    print(f"  {name:28s} shape {tuple(a.shape)}  mean|d| {d.mean().item():.3e}  max|d| {d.max().item():.3e}  "
          f"frac differing {nz:.4f}  mean|a| {a.abs().mean().item():.3e}")
    return d.max().item() > 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=3)
    ap.add_argument("--dtype", default="float16")
    ap.add_argument("--fixture", default="tiny_refine")
    ap.add_argument("--batch", type=int, default=3, help="snippet batch of both runs (the test: 3 sharded, 8 single)")
    ap.add_argument("--single-batch", type=int, default=None)
    args = ap.parse_args()
    import socket
    import torch.multiprocessing as mp
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, args.world, port, args.fixture, args.dtype, args.batch))
             for r in range(args.world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    sh = torch.load(os.path.join(ROOT, "gpurun_out", "refdiv_sharded.pt"))

    t = load_file(os.path.join(G, args.fixture + ".safetensors"))
    meta = json.load(open(os.path.join(G, args.fixture + ".json")))
    torch.cuda.set_device(0)
    pipe = _pipe(meta, t, getattr(torch, args.dtype))
    pipe.snippet_batch = args.single_batch or args.batch
    rec = {}
    _hook(pipe, rec)
    out = pipe.forward(t["frames"][None], list(meta["dilations_in"]), True, [3], [1], [1], None,
                       meta.get("refine_step", 0), 3, meta.get("refine_start_dilation", 6), None, False, 4, False,
                       init_noise=t["init_noise"])
    rec["coaligned"] = out.depth_coaligned.float()
    rec["depth"] = out.depth_pred.float()
    print(f"{args.fixture} {args.dtype}: sharded world {args.world} vs single GPU (snippet batch "
          f"{args.batch} / {pipe.snippet_batch})")
    _cmp("coaligned depth", sh["coaligned"].view(-1), rec["coaligned"].view(-1))
    for k in ("rgb_latent", "dlat", "noise"):
        _cmp(k, sh[k], rec[k])
    for i, (a, b) in enumerate(zip(sh["preds"], rec["preds"])):
        if a.shape == b.shape:
            _cmp(f"refine step {i} preds", a, b)
        else:
            print(f"  refine step {i} preds: shapes {tuple(a.shape)} vs {tuple(b.shape)} (rank 0's share)")
            n = a.shape[0]
            _cmp(f"refine step {i} preds[:{n}]", a, b[:n])
    for i, (a, b) in enumerate(zip(sh["steps"], rec["steps"])):
        _cmp(f"refine step {i} averaged", a, b)
    _cmp("depth", sh["depth"].view(-1), rec["depth"].view(-1))


if __name__ == "__main__":
    main()
