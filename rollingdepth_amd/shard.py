"""Snippet data-parallel sharding across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI):
  1. frames are split into W equal contiguous chunks; each rank VAE-encodes its chunk and the
     latents are all-gathered (73.7 KB/frame at 768², negligible on xGMI);
  2. the flattened (dilation, snippet) list of rollingdepth_pipeline.py:390-446 is split into W
     equal contiguous ranges; each rank runs the 1-step UNet and the VAE decode of its range
     (≈94 % of the FLOPs);
  3. the decoded snippets are all-gathered (the north_star's all-gather of per-snippet depth
     before co-alignment) and rank 0 runs the DepthAligner, the merge and the renormalisation.
The arithmetic per snippet is identical to the single-GPU path (batching-invariant kernels),
so sharded output == single-GPU output bitwise.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist

F16 = torch.float16


def chunk_bounds(total: int, world: int) -> List[Tuple[int, int]]:
    """Equal contiguous chunks of ceil(total/world) (the last ones may be short or empty)."""
    c = (total + world - 1) // world
    return [(min(r * c, total), min((r + 1) * c, total)) for r in range(world)]


def flat_snippets(counts: Sequence[int]) -> List[Tuple[int, int]]:
    return [(d, k) for d, n in enumerate(counts) for k in range(n)]


def rank_subsets(counts: Sequence[int], world: int, rank: int) -> List[List[int]]:
    """Snippet indices per dilation owned by `rank` under the contiguous flat split."""
    flat = flat_snippets(counts)
    lo, hi = chunk_bounds(len(flat), world)[rank]
    sub = [[] for _ in counts]
    for d, k in flat[lo:hi]:
        sub[d].append(k)
    return sub


def _all_gather_rows(local: torch.Tensor, total: int, world: int, group=None) -> torch.Tensor:
    """All-gather equal-size row chunks (padded) → [total, ...]."""
    c = (total + world - 1) // world
    if local.shape[0] < c:
        pad = torch.zeros((c - local.shape[0], *local.shape[1:]), dtype=local.dtype, device=local.device)
        local = torch.cat([local, pad])
    out = torch.empty((c * world, *local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out[:total]


def local_rows(snippets: Sequence[torch.Tensor], counts: Sequence[int], world: int, rank: int) -> torch.Tensor:
    """This rank's decoded snippets in flat (dilation, snippet) order → [rows, w, H, W]."""
    flat = flat_snippets(counts)
    lo, hi = chunk_bounds(len(flat), world)[rank]
    ref = next(s for s in snippets if s is not None)
    out = torch.empty((max(hi - lo, 0), *ref.shape[1:]), dtype=ref.dtype, device=ref.device)
    for i, (d, k) in enumerate(flat[lo:hi]):
        out[i] = snippets[d][k]
    return out


def gather_snippets(local: torch.Tensor, counts: Sequence[int], world: int, group=None) -> List[torch.Tensor]:
    """All-gather every rank's rows and split them back per dilation."""
    allsn = _all_gather_rows(local, sum(counts), world, group)
    per_d, o = [], 0
    for n in counts:
        per_d.append(allsn[o:o + n])
        o += n
    return per_d


@torch.no_grad()
def sharded_forward(pipe, input_frames: torch.Tensor, dilations: List[int], cap_dilation: bool = True,
                    snippet_len: int = 3, coalign_kwargs=None, init_noise: torch.Tensor = None, group=None,
                    num_frames: int = None, to_host: bool = False):
    """Multi-GPU RollingDepthPipeline.forward (refine_step = 0).  Returns the depth [N,1,H,W] f16
    on rank 0 (None elsewhere) and the per-dilation snippets on rank 0.

    `input_frames` is either the whole video [1,N,3,H,W] / [N,3,H,W], or — with `num_frames=N`
    — only this rank's contiguous chunk chunk_bounds(N, world)[rank] (each rank then holds 1/W of
    the video in host/device memory).

    `to_host=True` mirrors forward()'s D2H boundary, distributed: every rank copies its own chunk
    of input_rgb and its own snippet rows to pinned host memory (overlapping the gathers and the
    aligner), rank 0 the coaligned depth; rank 0 returns (depth_host, per-dilation device
    snippets), other ranks (None, None) — after their copies completed."""
    from . import kernels as K
    from .aligner import DepthAligner

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = pipe.device
    frames = input_frames[0] if input_frames.dim() == 5 else input_frames
    N = frames.shape[0] if num_frames is None else num_frames
    dil = list(dilations)
    if cap_dilation:
        dil = [pipe.cap_max_dilation(N, snippet_len, d) for d in dil]
    # 1. encode my frame chunk, all-gather latents
    lo, hi = chunk_bounds(N, world)[rank]
    f = pipe.vae.factor
    H, W = frames.shape[-2:]
    h, w = H // f, W // f
    mine_frames = frames[lo:hi] if num_frames is None else frames
    if num_frames is not None and mine_frames.shape[0] != hi - lo:
        raise ValueError(f"rank {rank} holds {mine_frames.shape[0]} frames, expected {hi - lo}")
    if hi > lo:
        mine = pipe.encode_rgb(mine_frames.to(dev))
    else:
        mine = torch.zeros((0, h, w, 8), dtype=F16, device=dev)
    rgb_latent = _all_gather_rows(mine, N, world, group)
    if init_noise is None:
        g = torch.Generator(device=dev).manual_seed(0)
        init_noise = torch.randn((1, 4, h, w), device=dev, dtype=F16, generator=g)
    noise = K.nchw_to_nhwc(init_noise.to(dev), 8)
    # 2. my snippets
    counts = [len(pipe.get_snippet_indice(0, [0], N, snippet_len, d, d, 1)) for d in dil]
    subsets = rank_subsets(counts, world, rank)
    snippets = pipe.init_snippet_infer(rgb_latent, noise, dil, [snippet_len] * len(dil), [1] * len(dil),
                                       [1] * len(dil), snippet_subset=subsets)
    local = local_rows(snippets, counts, world, rank)
    d2h = torch.cuda.Stream(dev) if to_host else None
    if to_host:
        for t in local:
            if t.shape[0]:
                pipe._to_host_async(t, d2h)
        if hi > lo:
            pipe._to_host_async(mine_frames.to(dev, F16) / 2.0 + 0.5, d2h)
    # 3. all-gather decoded snippets, co-align on rank 0
    per_d = gather_snippets(local, counts, world, group)
    if rank != 0:
        if d2h is not None:
            d2h.synchronize()
        return None, None
    aligner = DepthAligner(device=dev, **(coalign_kwargs or {}))
    merged, _, _, _ = aligner.run([s.view(s.shape[0], snippet_len, 1, H, W) for s in per_d], dil)
    d = merged.float().contiguous()
    K.renormalize_(d, K.minmax(d))
    depth = d.to(F16)
    if d2h is not None:
        depth = pipe._to_host_async(depth, d2h)
        pipe._to_host_async(d.to(F16), d2h)  # depth_pred (== coaligned without refine)
        d2h.synchronize()
    return depth, per_d
