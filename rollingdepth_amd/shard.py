"""Snippet data-parallel sharding across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Per forward:
  1. frames are split into W contiguous chunks; each rank VAE-encodes its chunk and the latents are
     all-gathered ([N, h, w, 8] f16, 147 KB/frame at 768²);
  2. the flattened (dilation, snippet) list of rollingdepth_pipeline.py:390-446 is split into W
     contiguous ranges of equal size (every snippet costs the same); each rank runs the 1-step UNet
     and the VAE decode of its range (≈94 % of the FLOPs) and keeps the decoded snippets;
  3. co-alignment (depth_aligner.py:68-120) without moving full-resolution depth:
       all-reduce MIN of the local snippet minima (the shift of :78);
       each rank crops / subsamples its own snippets (:82-92) and the [n, w, P] f32 aligner inputs
       are all-gathered (3·P·4 B = 71 KB per snippet at 768², the north_star's all-gather of
       per-snippet depth before co-alignment);
       every rank runs the same deterministic 2000-iteration Adam kernel on the same inputs, so every
       rank holds the same scales / translations with no broadcast;
       merge_scaled_triplets (:231-262) windowed: each rank sums s·x+t (f64) over only the frame
       ranges its own full-resolution snippets cover, one uneven all-to-all sends those rows to the
       owners of the frame chunks, and each owner adds the received pieces per frame in source-rank
       order and divides by the frame's cover count (no world-size limit: the library splits a piece
       table wider than its 64-entry kernel argument by frame range);
       all-reduce MIN / MAX for the renormalisation (rollingdepth_pipeline.py:316-318);
  4. refine (full / paper presets): each rank encodes its chunk of the co-aligned depth, the depth
     latents are all-gathered, and every refine step splits its snippets over the ranks with one
     all-reduce of the [N, h·w, 4] f32 per-frame sums (pipeline.refine(group=...)); each rank decodes
     its own frame chunk of the refined latents.
Outputs stay distributed: rank r holds depth / coaligned depth for frames chunk_bounds(N, W)[r]
(and its own decoded snippets); `gather=True` assembles the full maps on every rank.

Numerics vs the single-GPU forward: identical per-snippet arithmetic.  The cross-rank sums — the
merge of s·x+t per frame and refine's per-frame average of snippet predictions — are f64 sums on
both paths (aligner.hip merge_k, elementwise.hip snippet_*): exact for f16 terms, and for f32 terms
exact unless a frame's terms span more than ≈29 exponent bits (rare), so the order RCCL reduces them
in does not change a bit in practice; the aligner runs the same kernel on the same (all-gathered)
inputs.  What can still differ is the kernel engine chosen per launch shape (the f32 accumulation
order inside a conv / GEMM depends on the batch a rank runs), which at SD2 shapes is not bitwise.
Stated tolerance: depth mean |Δ| ≤ 1e-3 (the north_star bound) against the single-GPU result
(tests/test_pipeline_gpu.py); at the test sizes the sharded forward, refine included, reproduces the
single-GPU forward bitwise.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist

F16, F32 = torch.float16, torch.float32


def chunk_bounds(total: int, world: int) -> List[Tuple[int, int]]:
    """Equal contiguous chunks of ceil(total/world) (the last ones may be short or empty)."""
    c = (total + world - 1) // world
    return [(min(r * c, total), min((r + 1) * c, total)) for r in range(world)]


def flat_snippets(counts: Sequence[int]) -> List[Tuple[int, int]]:
    return [(d, k) for d, n in enumerate(counts) for k in range(n)]


def rank_subsets(counts: Sequence[int], world: int, rank: int) -> List[List[int]]:
    """Snippet indices per dilation owned by `rank` under the contiguous flat split (contiguous
    within each dilation)."""
    flat = flat_snippets(counts)
    lo, hi = chunk_bounds(len(flat), world)[rank]
    sub = [[] for _ in counts]
    for d, k in flat[lo:hi]:
        sub[d].append(k)
    return sub


class SliceGroup:
    """Stand-in process group for timing ONE rank's share of a W-rank run on one GPU (bench.py
    --slice-world): the rank runs exactly its own encode chunk, snippets, decode, aligner and partial
    merge, and every collective is a local no-op that fills the received buffers with this rank's own
    data (so the kernels after it see data of the same shape and range).  Not a scaling measurement:
    it leaves out the collectives' time and overlap."""

    def __init__(self, rank: int, world: int):
        if not 0 <= rank < world:
            raise ValueError(f"slice rank {rank} of world {world}")
        self.rank, self.world = rank, world


def _rank(group) -> int:
    return group.rank if isinstance(group, SliceGroup) else dist.get_rank(group)


def _world(group) -> int:
    return group.world if isinstance(group, SliceGroup) else dist.get_world_size(group)


def _via_host(group, t: torch.Tensor) -> bool:
    """gloo has no device transport: device tensors are staged through host memory (tests that run
    several ranks on one GPU, or CPU ranks); RCCL moves device memory directly over xGMI."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


# Per-collective timing (bench.py --gpus N): when a list, every collective below appends (kind, start
# event, end event, bytes) — HIP events recorded on the current stream right before the collective is
# issued and right after the current stream was made to wait for it, so a span covers the transfer plus
# any wait for the slowest rank to arrive.
collective_timing: Optional[list] = None


class _Coll:
    """Brackets one collective with timing events when `collective_timing` is a list."""

    def __init__(self, kind: str, nbytes: int):
        self.kind, self.nbytes = kind, nbytes

    def __enter__(self):
        if collective_timing is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        if collective_timing is not None and exc[0] is None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            collective_timing.append((self.kind, self.e0, e1, self.nbytes))
        return False


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def _gather_into(out: torch.Tensor, inp: torch.Tensor, group=None):
    if isinstance(group, SliceGroup):  # every rank's slot gets this rank's rows
        out.view(-1, inp.numel()).copy_(inp.reshape(1, -1).expand(out.numel() // max(inp.numel(), 1), -1))
        return
    with _Coll("all_gather", _nbytes(out)):
        if _via_host(group, inp):
            o = out.cpu()
            dist.all_gather_into_tensor(o, inp.cpu(), group=group)
            out.copy_(o)
        else:
            dist.all_gather_into_tensor(out, inp, group=group)


def _all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None):
    if isinstance(group, SliceGroup):
        return
    with _Coll("all_reduce", _nbytes(t)):
        if _via_host(group, t):
            h = t.cpu()
            dist.all_reduce(h, op=op, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op, group=group)


def _all_gather_rows(local: torch.Tensor, total: int, world: int, group=None) -> torch.Tensor:
    """All-gather the rows of chunk_bounds(total, world)[rank] from every rank → [total, ...]."""
    c = (total + world - 1) // world
    if local.shape[0] < c:
        pad = torch.zeros((c - local.shape[0], *local.shape[1:]), dtype=local.dtype, device=local.device)
        local = torch.cat([local, pad])
    out = torch.empty((c * world, *local.shape[1:]), dtype=local.dtype, device=local.device)
    _gather_into(out, local.contiguous(), group)
    return out[:total]


def _broadcast(t: torch.Tensor, src: int = 0, group=None):
    """Broadcast from the group's rank `src` (device tensors staged through the host under gloo)."""
    if isinstance(group, SliceGroup):
        return
    root = dist.get_global_rank(group, src) if group is not None and group != dist.group.WORLD else src
    with _Coll("broadcast", _nbytes(t)):
        if _via_host(group, t):
            h = t.cpu()
            dist.broadcast(h, root, group=group)
            t.copy_(h)
        else:
            dist.broadcast(t, root, group=group)


def gather_rows_by_dilation(local: Sequence[torch.Tensor], counts: Sequence[int], world: int,
                            group=None) -> List[torch.Tensor]:
    """Every rank's rows (its part of the flat split rank_subsets(counts, world, rank), per dilation
    in `local`: [m_d, *row_shape_d], row shapes may differ per dilation — snippet lengths per
    dilation) all-gathered and split back per dilation: → [n_d, *row_shape_d] for every d.
    One all-gather of each rank's rows flattened into one buffer (padded to the largest rank's)."""
    shapes = [tuple(t.shape[1:]) for t in local]
    sizes = [math.prod(sh) for sh in shapes]
    ref = local[0]
    plan = [rank_subsets(counts, world, r) for r in range(world)]
    per_rank = [sum(len(sub[d]) * sizes[d] for d in range(len(counts))) for sub in plan]
    cap = max(max(per_rank), 1)
    rank = _rank(group)
    for d, t in enumerate(local):
        if t.shape[0] != len(plan[rank][d]):
            raise ValueError(f"rank {rank} holds {t.shape[0]} rows of dilation {d}, its plan {len(plan[rank][d])}")
    flat = torch.zeros(cap, dtype=ref.dtype, device=ref.device)
    if per_rank[rank]:
        torch.cat([t.reshape(-1) for t in local if t.numel()], out=flat[:per_rank[rank]])
    allv = torch.empty(cap * world, dtype=ref.dtype, device=ref.device)
    _gather_into(allv, flat, group)
    per_d = [torch.empty((n, *shapes[d]), dtype=ref.dtype, device=ref.device) for d, n in enumerate(counts)]
    for r in range(world):
        o = r * cap
        for d in range(len(counts)):
            m = len(plan[r][d])
            if m:
                k0 = plan[r][d][0]
                per_d[d][k0:k0 + m] = allv[o:o + m * sizes[d]].view(m, *shapes[d])
                o += m * sizes[d]
    return per_d


def _all_reduce_minmax(mm: torch.Tensor, group=None) -> torch.Tensor:
    """[min, max] f32 → the global [min, max] (one MIN all-reduce of [min, −max])."""
    t = torch.stack([mm[0], -mm[1]])
    _all_reduce(t, dist.ReduceOp.MIN, group)
    return torch.stack([t[0], -t[1]])


def frame_ranges(subsets: Sequence[Sequence[int]], strides: Sequence[int], w: Sequence[int]) -> List[Tuple[int, int]]:
    """Frames a rank's snippets cover, as sorted disjoint ranges [lo, hi): slot j of snippet k of
    dilation d is frame k + j·stride_d (depth_aligner.py:179-188); one range per dilation's contiguous
    snippet run (a dilation's frames between its slots included), overlapping ranges joined."""
    rs = sorted((min(sub), max(sub) + (wd - 1) * st + 1) for sub, st, wd in zip(subsets, strides, w) if sub)
    out: List[Tuple[int, int]] = []
    for lo, hi in rs:
        if out and lo <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], hi))
        else:
            out.append((lo, hi))
    return out


def _cut(ranges: Sequence[Tuple[int, int]], lo: int, hi: int) -> List[Tuple[int, int]]:
    """Parts of `ranges` inside [lo, hi) as (first frame, frame count), in order."""
    return [(max(a, lo), min(b, hi) - max(a, lo)) for a, b in ranges if min(b, hi) > max(a, lo)]


def merge_exchange_plan(counts: Sequence[int], strides: Sequence[int], w: Sequence[int], N: int, world: int,
                        rank: int):
    """The all-to-all of the windowed merge, from the plan alone (no communication): this rank's
    frame ranges, the rows it sends to each rank (its rows inside that rank's frame chunk — the
    ranges' rows are stored in frame order, so each destination's rows are contiguous) and the pieces
    (first frame, frame count) it receives from each rank (the sender's ranges cut by this rank's
    chunk, in frame order)."""
    ranges = [frame_ranges(rank_subsets(counts, world, r), strides, w) for r in range(world)]
    chunks = chunk_bounds(N, world)
    send = [sum(m for _, m in _cut(ranges[rank], *chunks[r])) for r in range(world)]
    recv = [_cut(ranges[r], *chunks[rank]) for r in range(world)]
    return ranges[rank], send, recv


def _merge_windowed(rows, k0, counts, scales, trans, strides, slens, N: int, HW: int, shift, x_f32, group):
    """merge_scaled_triplets over W ranks: per-rank f64 sums of only the frames its snippets cover, an
    all-to-all of the rows each rank's frame chunk needs (uneven row counts; RCCL over xGMI), then
    the received pieces added per frame in source-rank order and ÷ the cover count (f64 sums: the
    single-GPU merge bitwise).  Returns this rank's chunk
    [f1 − f0, HW] f32.  Moves each rank's covered frames instead of N·HW·8 B per rank."""
    from . import kernels as K

    world, rank = _world(group), _rank(group)
    ranges, send, recv = merge_exchange_plan(counts, strides, slens, N, world, rank)
    f0, f1 = chunk_bounds(N, world)[rank]
    sums = torch.empty((sum(b - a for a, b in ranges), HW), dtype=torch.float64, device=shift.device)
    o = 0
    for a, b in ranges:
        K.aligner_merge_partial_window([r if r.shape[0] else None for r in rows], k0, counts, scales, trans,
                                       strides, slens, a, b - a, HW, shift, x_f32, out=sums[o:o + b - a])
        o += b - a
    rbuf = exchange_window_rows(sums, send, [sum(m for _, m in pc) for pc in recv], group)
    pieces = [pc for src in recv for pc in src]
    return K.aligner_merge_finish_pieces(rbuf, pieces, counts, strides, slens, f0, f1 - f0, HW)


def exchange_window_rows(sums: torch.Tensor, send: Sequence[int], recv: Sequence[int], group) -> torch.Tensor:
    """The windowed merge's all-to-all: `sums` [rows, ...] (this rank's covered frames in frame order,
    send[r] rows for rank r, back to back) → the received rows [Σ recv, ...], recv[s] rows from rank s,
    in source-rank order."""
    row = math.prod(sums.shape[1:])
    in_split = [n * row for n in send]
    out_split = [n * row for n in recv]
    rbuf = torch.empty((sum(recv), *sums.shape[1:]), dtype=sums.dtype, device=sums.device)
    if isinstance(group, SliceGroup):  # local no-op: this rank's own rows stand in for every source
        if rbuf.numel():
            src = sums.reshape(-1)
            if src.numel():
                reps = (rbuf.numel() + src.numel() - 1) // src.numel()
                rbuf.view(-1).copy_(src.repeat(reps)[:rbuf.numel()])
            else:
                rbuf.zero_()
    else:
        with _Coll("all_to_all", max(_nbytes(sums), _nbytes(rbuf))):
            if _via_host(group, sums):
                h = torch.empty(rbuf.shape, dtype=rbuf.dtype)
                dist.all_to_all_single(h.view(-1), sums.reshape(-1).cpu(), out_split, in_split, group=group)
                rbuf.copy_(h)
            else:
                dist.all_to_all_single(rbuf.view(-1), sums.reshape(-1), out_split, in_split, group=group)
    return rbuf


def _mark(timing: Optional[list], name: str):
    """Phase boundary for bench.py's per-phase times: a timing event on the current stream."""
    if timing is not None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        timing.append((name, ev))


class ShardedOutput:
    """Distributed RollingDepthOutput: this rank's frame chunk [f0, f1) of depth_pred /
    depth_coaligned / input_rgb, its own decoded snippets (snippet_rows[d] are global snippets
    snippet_k0[d] ..), and — when gathered — the full maps."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


@torch.no_grad()
def sharded_forward(pipe, input_frames: torch.Tensor, dilations: List[int], cap_dilation: bool = True,
                    snippet_len: Union[int, Sequence[int]] = 3, coalign_kwargs=None,
                    init_noise: Optional[torch.Tensor] = None, group=None, num_frames: Optional[int] = None,
                    to_host: bool = False, refine_step: int = 0, refine_snippet_len: int = 3,
                    refine_start_dilation: int = 6, gather: bool = False, record: Optional[dict] = None,
                    generator: Optional[torch.Generator] = None,
                    init_infer_steps: Union[int, Sequence[int]] = 1, timing: Optional[list] = None) -> ShardedOutput:
    """Multi-GPU RollingDepthPipeline.forward (every preset: refine_step > 0 included).

    `input_frames` is either the whole video [1,N,3,H,W] / [N,3,H,W], or — with `num_frames=N` —
    only this rank's contiguous chunk chunk_bounds(N, world)[rank] (each rank then holds 1/W of the
    video in host / device memory).  `to_host=True` mirrors forward()'s D2H boundary, distributed:
    every rank copies its own depth / coaligned / input_rgb chunk and its own snippet rows to pinned
    host memory.  `gather=True` also all-gathers the full depth_pred / depth_coaligned on every rank
    (tests, small N).  `dilations` is not mutated (forward() mutates the caller's list; this is the
    build's own entry point).  `snippet_len`: one length, or one per dilation.  `group` defaults to
    the world group (refine's all-reduce included).  `init_infer_steps`: DDIM steps per snippet, one
    count or one per dilation (rollingdepth_pipeline.py:421-445), as forward().  Without `init_noise` the shared noise is drawn
    on rank 0 exactly as forward() draws it (from `generator`) and broadcast.  `timing` (a list):
    phase-boundary events (name, torch.cuda.Event) are appended to it (bench.py --slice-world)."""
    from . import kernels as K
    from .aligner import DepthAligner, check_row_layout

    if group is None:
        group = dist.group.WORLD
    world = _world(group)
    rank = _rank(group)
    dev = pipe.device
    frames = input_frames[0] if input_frames.dim() == 5 else input_frames
    N = frames.shape[0] if num_frames is None else num_frames
    dil = list(dilations)
    slens = [int(x) for x in snippet_len] if isinstance(snippet_len, (list, tuple)) else [int(snippet_len)] * len(dil)
    if len(slens) != len(dil):
        raise ValueError(f"snippet lengths {slens} vs dilations {dil}")
    steps = [int(x) for x in init_infer_steps] if isinstance(init_infer_steps, (list, tuple)) \
        else [int(init_infer_steps)] * len(dil)
    if len(steps) == 1:
        steps = steps * len(dil)
    if len(steps) != len(dil) or min(steps) < 1:
        raise ValueError(f"init_infer_steps {steps} vs dilations {dil} (one count >= 1 per dilation)")
    if cap_dilation:
        dil = [pipe.cap_max_dilation(N, sl, d) for d, sl in zip(dil, slens)]
        refine_start_dilation = pipe.cap_max_dilation(N, refine_snippet_len, refine_start_dilation)
    if 1 not in dil:
        raise AssertionError("dilations should include 1")
    f0, f1 = chunk_bounds(N, world)[rank]
    mine_frames = frames[f0:f1] if num_frames is None else frames
    if num_frames is not None and mine_frames.shape[0] != f1 - f0:
        raise ValueError(f"rank {rank} holds {mine_frames.shape[0]} frames, expected {f1 - f0}")
    H_in, W_in = frames.shape[-2:]
    h, w = pipe.vae.latent_hw(H_in, W_in)
    _mark(timing, "start")
    # 1. encode my frame chunk, all-gather the latents
    if f1 > f0:
        mine = pipe.encode_rgb(mine_frames.to(dev))
    else:
        mine = torch.zeros((0, h, w, pipe.vae.lat_pad), dtype=pipe.dtype, device=dev)
    rgb_latent = _all_gather_rows(mine, N, world, group)
    if init_noise is None:  # rollingdepth_pipeline.py:282-288, drawn once (rank 0) and broadcast
        if rank == 0:
            init_noise = torch.randn((1, 4, h, w), device=dev, dtype=pipe.dtype, generator=generator)
        else:
            init_noise = torch.empty((1, 4, h, w), device=dev, dtype=pipe.dtype)
        _broadcast(init_noise, 0, group)
    noise = pipe._noise_nhwc(init_noise, h, w)
    _mark(timing, "encode")
    # 2. my snippets (compact: row r of dilation d is global snippet subsets[d][r])
    counts = [len(pipe.get_snippet_indice(0, [0], N, sl, d, d, 1)) for d, sl in zip(dil, slens)]
    subsets = rank_subsets(counts, world, rank)
    k0 = [s[0] if s else 0 for s in subsets]
    aligner = DepthAligner(device=dev, **(coalign_kwargs or {}))
    check_row_layout(slens, aligner.num_iterations)
    rows = pipe.init_snippet_infer(rgb_latent, noise, dil, slens, steps, [1] * len(dil),
                                   snippet_subset=subsets)
    H, W = rows[0].shape[-2:]
    d2h = torch.cuda.Stream(dev) if to_host else None
    snip_host = [pipe._to_host_async(r.to(pipe.dtype), d2h) if r.shape[0] else None for r in rows] if to_host else None
    _mark(timing, "snippets")
    # 3. co-alignment
    local_mm = [K.minmax(r) for r in rows if r.shape[0]]
    mm = K.minmax(torch.stack(local_mm).reshape(-1)) if local_mm else \
        torch.tensor([float("inf"), float("-inf")], device=dev)
    shift = _all_reduce_minmax(mm, group)  # shift[0] = global min
    prepared = [aligner.prepare([r], shift)[0] if r.shape[0] else None for r in rows]
    P = ((H - 2 * aligner.border + aligner.factor - 1) // aligner.factor) * \
        ((W - 2 * aligner.border + aligner.factor - 1) // aligner.factor)
    xs = gather_rows_by_dilation([p if p is not None else torch.empty((0, sl, P), dtype=F32, device=dev)
                                  for p, sl in zip(prepared, slens)], counts, world, group)
    strides = list(dil)
    seq_len = aligner.sequence_length(counts, slens[0], dil)
    assert seq_len == N
    _mark(timing, "prepare")
    scales, trans, hist, ws = aligner.optimize_prepared(xs, strides, N)
    rows_f32 = rows[0].dtype == F32
    _mark(timing, "aligner")
    merged = _merge_windowed(rows, k0, counts, scales, trans, strides, slens, N, H * W, shift,
                             1 if rows_f32 else (2 if pipe.merge_f32 else 0), group)
    # merge_scaled_triplets returns the snippets' dtype (unless the pipeline merges in f32)
    d = (merged if (pipe.merge_f32 or rows_f32) else merged.to(pipe.dtype).float()).contiguous()
    mm_d = K.minmax(d) if d.numel() else torch.tensor([float("inf"), float("-inf")], device=dev)
    gmm = _all_reduce_minmax(mm_d, group)
    if d.numel():
        K.renormalize_(d, gmm)
    coaligned = d.to(pipe.dtype).view(f1 - f0, 1, H, W)
    del ws
    _mark(timing, "merge")
    # 4. refine
    if refine_step > 0:
        if f1 > f0:
            dlat_mine = pipe.encode_rgb(coaligned.expand(-1, 3, -1, -1))
        else:
            dlat_mine = torch.zeros((0, h, w, pipe.vae.lat_pad), dtype=pipe.dtype, device=dev)
        dlat = _all_gather_rows(dlat_mine, N, world, group)
        new = pipe.refine(rgb_latent, dlat, noise, refine_step, refine_snippet_len, refine_start_dilation,
                          group=group)
        if record is not None:
            record["refined_latent"] = new
        depth = torch.empty((f1 - f0, H, W, 1), dtype=pipe.depth_dtype, device=dev)
        if f1 > f0:
            z = K.ddim_combine(new[f0:f1, ..., :4], new[f0:f1, ..., :4], 1.0 / pipe.depth_latent_scale_factor, 0.0,
                               1.0, 4, 8)
            pipe.decode_depth(z, depth)
        depth = depth.view(f1 - f0, 1, H, W).to(pipe.dtype)
    else:
        depth = coaligned
    if refine_step > 0:
        _mark(timing, "refine")
    if record is not None:
        record.update(rgb_latent=rgb_latent, scales=scales, translations=trans, dilations=list(dil),
                      loss_history=hist)
    out = ShardedOutput(frame_range=(f0, f1), depth_pred=depth, depth_coaligned=coaligned, snippet_rows=rows,
                        snippet_k0=k0, snippet_counts=counts, dilations=dil, input_rgb=None, snippet_host=snip_host)
    if gather:
        out.depth_pred_full = _all_gather_rows(depth, N, world, group)
        out.depth_coaligned_full = _all_gather_rows(coaligned, N, world, group)
    if to_host:
        out.depth_pred = pipe._to_host_async(depth, d2h)
        out.depth_coaligned = pipe._to_host_async(coaligned, d2h) if refine_step > 0 else out.depth_pred
        if f1 > f0:
            out.input_rgb = pipe._to_host_async(mine_frames.to(dev, pipe.dtype) / 2.0 + 0.5, d2h)
        d2h.synchronize()
    _mark(timing, "egress")
    return out
