"""World-size-2, 3 and 8 gloo tests (CPU) of the multi-GPU plan of rollingdepth_amd/shard.py
(SURVEY.md §8e).  The collectives and the rank/frame/snippet bookkeeping are the product's own
functions; the per-rank device kernels (rdmi_aligner_merge_partial_window / rdmi_snippet_accumulate) are
stood in for by a CPU restatement of their contract (the GPU tests check the kernels against the
single-GPU merge and refine).  Checked against the oracle's single-process merge / refine average:
  * the flat snippet split + all-gather of per-snippet aligner inputs reassembles every dilation;
  * all-reduce MIN of [min, −max] gives the global min / max;
  * windowed merge: per-rank sums over the frames its snippets cover + all-to-all of each frame chunk's
    rows + ÷ cover count == merge_scaled_triplets;
  * per-rank refine sums + all-reduce + ÷ cover count == the single-process snippet average.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _snippet(d, k, shape):
    return torch.full(shape, float(1000 * d + k)) + torch.arange(shape[-1]).float()


def _merge_partial_cpu(rows, k0, n, strides, scales, trans, w, N, HW):
    """CPU restatement of rdmi_aligner_merge_partial_window (f32 snippets) over all N frames: per frame
    the sum over this rank's (dilation, local snippet, slot) of s·x + t, slots in the reference's
    k-ascending order (w: snippet length per dilation); the window's rows are slices of it."""
    out = torch.zeros((N, HW), dtype=torch.float32)
    for f in range(N):
        acc = torch.zeros(HW, dtype=torch.float32)
        for d, r in enumerate(rows):
            for j in range(w[d] - 1, -1, -1):
                k = f - j * strides[d]
                if k < k0[d] or k >= k0[d] + r.shape[0]:
                    continue
                acc = acc + (r[k - k0[d], j].reshape(-1) * scales[d][k] + trans[d][k])
        out[f] = acc
    return out


def _cover(n, strides, w, f):
    return sum(1 for d in range(len(n)) for j in range(w[d]) if 0 <= f - j * strides[d] < n[d])


def _worker(rank, world, port, res):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import rd_oracle as O
    from rollingdepth_amd.shard import (_all_gather_rows, _all_reduce_minmax, _broadcast, chunk_bounds, exchange_window_rows, frame_ranges, gather_rows_by_dilation,
                                        merge_exchange_plan, rank_subsets)

    ok = True
    # --- flat split + all-gather of per-snippet rows (the aligner inputs) -----------------------
    counts = [9, 5]
    shape = (3, 2, 5)
    sub = rank_subsets(counts, world, rank)
    local = [torch.stack([_snippet(d, k, shape) for k in sub[d]]) if sub[d] else torch.zeros((0, *shape))
             for d in range(len(counts))]
    per_d = gather_rows_by_dilation(local, counts, world)
    ok &= all(torch.equal(per_d[d][k], _snippet(d, k, shape)) for d, n in enumerate(counts) for k in range(n))
    # every rank's subset is contiguous within a dilation (compact rows = global k0 ..)
    ok &= all(s == list(range(s[0], s[0] + len(s))) for s in sub if s)
    # rows of different shapes per dilation (snippet lengths [3, 2]) through the same all-gather
    shapes = [(3, 2, 5), (2, 2, 5)]
    local = [torch.stack([_snippet(d, k, shapes[d]) for k in sub[d]]) if sub[d] else torch.zeros((0, *shapes[d]))
             for d in range(len(counts))]
    per_d = gather_rows_by_dilation(local, counts, world)
    ok &= all(torch.equal(per_d[d][k], _snippet(d, k, shapes[d])) for d, n in enumerate(counts) for k in range(n))
    # the shared init noise drawn on rank 0 and broadcast (sharded_forward without init_noise)
    nz = torch.randn(1, 4, 3, 3, generator=torch.Generator().manual_seed(5)) if rank == 0 else torch.zeros(1, 4, 3, 3)
    _broadcast(nz, 0)
    ok &= torch.equal(nz, torch.randn(1, 4, 3, 3, generator=torch.Generator().manual_seed(5)))
    # --- frame-chunk latents all-gather ------------------------------------------------------------
    N = 11
    lo, hi = chunk_bounds(N, world)[rank]
    lat = _all_gather_rows(torch.arange(lo, hi).float().view(-1, 1).expand(-1, 4).contiguous(), N, world)
    ok &= torch.equal(lat[:, 0], torch.arange(N).float())
    # --- global min / max -----------------------------------------------------------------------------
    mm = _all_reduce_minmax(torch.tensor([float(rank) - 5.0, 10.0 * rank]))
    ok &= mm.tolist() == [-5.0, 10.0 * (world - 1)]
    # --- windowed merge: sums over the rank's covered frame ranges only, all-to-all of the rows each
    # chunk needs, pieces added per frame in source-rank order (rdmi_aligner_merge_finish_pieces),
    # ÷ cover count == merge_scaled_triplets ------------------------------------------------------------
    N, H, W = 14, 4, 5
    w = [3, 2]  # snippet lengths per dilation
    dil = [1, 4]
    g = torch.Generator().manual_seed(11)
    full = [torch.rand((N - (wd - 1) * d, wd, H, W), generator=g) for d, wd in zip(dil, w)]
    n = [x.shape[0] for x in full]
    sc = [0.5 + torch.rand(m, generator=g) for m in n]
    tr = [0.1 * torch.randn(m, generator=g) for m in n]
    sub = rank_subsets(n, world, rank)
    k0 = [s[0] if s else 0 for s in sub]
    rows = [full[d][k0[d]:k0[d] + len(sub[d])] for d in range(len(dil))]
    sums = _merge_partial_cpu(rows, k0, n, dil, sc, tr, w, N, H * W)
    f0, f1 = chunk_bounds(N, world)[rank]
    idx = [O.aligner_indices(N, d - 1, wd) for d, wd in zip(dil, w)]
    ref = O.aligner_merge([x.numpy()[:, :, None] for x in full], idx, [s.numpy() for s in sc],
                          [t.numpy() for t in tr], N)
    ranges, send, recv = merge_exchange_plan(n, dil, w, N, world, rank)
    ok &= ranges == frame_ranges(sub, dil, w)
    covered = {f for d in range(len(dil)) for k in sub[d] for j in range(w[d]) for f in [k + j * dil[d]]}
    inr = {f for a, b in ranges for f in range(a, b)}
    ok &= covered <= inr and all(b1 < a2 for (_, b1), (a2, _) in zip(ranges, ranges[1:]))
    wsum = torch.cat([sums[a:b] for a, b in ranges]).double() if ranges else torch.zeros((0, H * W),
                                                                                          dtype=torch.float64)
    ok &= sum(send) == wsum.shape[0]
    rbuf = exchange_window_rows(wsum, send, [sum(m for _, m in pc) for pc in recv], None)
    acc = torch.zeros((f1 - f0, H * W), dtype=torch.float64)
    o = 0
    for src in recv:
        for a, m in src:
            acc[a - f0:a - f0 + m] += rbuf[o:o + m]
            o += m
    ok &= o == rbuf.shape[0]
    mine_w = torch.stack([acc[i] / _cover(n, dil, w, f0 + i) for i in range(f1 - f0)]).float() if f1 > f0 \
        else torch.zeros((0, H * W))
    merged_w = _all_gather_rows(mine_w, N, world)
    ok &= bool(np.abs(merged_w.numpy() - ref.reshape(N, H * W)).max() < 1e-5)
    # --- refine step: rank-local sums of its snippets' predictions, all-reduce, ÷ cover count ---------
    Nf, L, P, C = 13, 3, 6, 4
    stride = 2
    nsn = Nf - (L - 1) * stride
    preds = torch.randn((nsn, L, P, C), generator=g)
    a, b = chunk_bounds(nsn, world)[rank]
    acc = torch.zeros((Nf, P, C))
    for s in range(a, b):
        for j in range(L):
            acc[s + j * stride] += preds[s, j]
    dist.all_reduce(acc)
    cnt = torch.tensor([sum(1 for j in range(L) if 0 <= f - j * stride < nsn) for f in range(Nf)]).float()
    got = acc / cnt[:, None, None]
    want = torch.zeros((Nf, P, C))
    for s in range(nsn):
        for j in range(L):
            want[s + j * stride] += preds[s, j]
    want /= cnt[:, None, None]
    ok &= torch.allclose(got, want, atol=1e-6)
    res[rank] = int(ok)
    dist.destroy_process_group()


def _run(world):
    ctx = mp.get_context("spawn")
    res = ctx.Array("i", [0] * world)
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, res)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    assert list(res) == [1] * world


def test_shard_plan_world2():
    _run(2)


def test_shard_plan_world3():
    """An uneven split (ragged last chunks) — the same plan at W = 3."""
    _run(3)


class _StopAtSnippets(Exception):
    pass


class _PlanPipe:
    """Host-only stand-in for RollingDepthPipeline up to the snippet stage of sharded_forward: records
    the arguments init_snippet_infer receives on each rank, then stops the forward (the device stages
    after it are covered by the GPU tests)."""

    def __init__(self):
        from rollingdepth_amd.pipeline import RollingDepthPipeline
        from types import SimpleNamespace
        self.device = torch.device("cpu")
        self.dtype = torch.float32
        self.vae = SimpleNamespace(latent_hw=lambda H, W: (H // 8, W // 8), lat_pad=8)
        self.get_snippet_indice = RollingDepthPipeline.get_snippet_indice
        self.cap_max_dilation = RollingDepthPipeline.cap_max_dilation
        self.calls = []

    def encode_rgb(self, frames):
        return torch.zeros((frames.shape[0], frames.shape[-2] // 8, frames.shape[-1] // 8, 8))

    def _noise_nhwc(self, noise, h, w):
        return torch.zeros((1, h, w, 8))

    def init_snippet_infer(self, rgb_latent, noise, dilations, snippet_lengths, init_infer_steps, strides,
                           snippet_subset=None, record=None):
        self.calls.append(dict(dilations=list(dilations), steps=list(init_infer_steps), subset=snippet_subset))
        raise _StopAtSnippets


def _steps_worker(rank, world, port, res):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rollingdepth_amd.shard import rank_subsets, sharded_forward

    ok = True
    for steps, want in (([2], [2, 2]), ([1, 3], [1, 3]), (4, [4, 4])):
        pipe = _PlanPipe()
        try:
            sharded_forward(pipe, torch.zeros((1, 30, 3, 16, 16)), [1, 10], True, 3, None,
                            init_noise=torch.zeros(1, 4, 2, 2), init_infer_steps=steps)
        except _StopAtSnippets:
            pass
        c = pipe.calls[0]
        counts = [30 - 2 * d for d in c["dilations"]]
        ok &= c["steps"] == want and c["subset"] == rank_subsets(counts, world, rank)
    try:  # a count per dilation that does not match the dilations
        sharded_forward(_PlanPipe(), torch.zeros((1, 30, 3, 16, 16)), [1, 10], True, 3, None,
                        init_noise=torch.zeros(1, 4, 2, 2), init_infer_steps=[1, 2, 3])
        ok = False
    except ValueError:
        pass
    res[rank] = int(ok)
    dist.destroy_process_group()


def test_sharded_forward_honours_init_infer_steps_world2():
    """the sharded forward runs the DDIM step count per dilation that forward() was given
    (rollingdepth_pipeline.py:421-445), on every rank, with the rank's own snippet subset."""
    ctx = mp.get_context("spawn")
    res = ctx.Array("i", [0, 0])
    port = _free_port()
    procs = [ctx.Process(target=_steps_worker, args=(r, 2, port, res)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    assert list(res) == [1, 1]


def test_shard_plan_world8():
    """The plan at the driver's largest scaling point, W = 8: most ranks own 1-2 of the 14 merge frames
    and of the 14 + 10 snippets, some none of a dilation, and chunk_bounds(11, 8) leaves the last
    latent chunk empty."""
    _run(8)


def test_merge_exchange_plan_at_bench_shapes():
    """The windowed merge's all-to-all plan (merge_exchange_plan) at the BASELINE configurations'
    snippet counts for W = 2 … 24, planned independently on every rank: what rank s sends to rank r is
    what r expects from s, every piece lies inside r's frame chunk and inside one of s's frame ranges,
    and every frame a snippet slot of s covers reaches its owner from s."""
    from rollingdepth_amd.shard import chunk_bounds, merge_exchange_plan, rank_subsets

    cases = [(100, [1, 25], [3, 3]),        # configs[1] fast (and fast1024)
             (100, [1, 10, 25], [3, 3, 3]),  # configs[3] full
             (500, [1, 10, 25], [3, 3, 3]),  # configs[4] paper
             (30, [1, 10], [3, 2])]          # mixed snippet lengths
    for N, dil, w in cases:
        counts = [N - (wd - 1) * d for d, wd in zip(dil, w)]
        for W in (2, 4, 8, 24):
            plans = [merge_exchange_plan(counts, dil, w, N, W, r) for r in range(W)]
            chunks = chunk_bounds(N, W)
            for s in range(W):
                ranges, send, _ = plans[s]
                assert sum(send) == sum(b - a for a, b in ranges)
                sub = rank_subsets(counts, W, s)
                slots = {k + j * dil[d] for d in range(len(dil)) for k in sub[d] for j in range(w[d])}
                for r in range(W):
                    pieces = plans[r][2][s]
                    assert send[r] == sum(m for _, m in pieces)
                    f0, f1 = chunks[r]
                    for a, m in pieces:
                        assert f0 <= a and a + m <= f1 and m > 0
                        assert any(lo <= a and a + m <= hi for lo, hi in ranges)
                    got = {f for a, m in pieces for f in range(a, a + m)}
                    assert {f for f in slots if f0 <= f < f1} <= got
