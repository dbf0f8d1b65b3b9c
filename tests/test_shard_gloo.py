"""World-size-2 gloo test (CPU) of the multi-GPU collective plan of rollingdepth_amd/shard.py:
each rank produces only its contiguous flat range of snippets, the all-gather + per-dilation
split must reassemble exactly the single-process snippet lists (and latents for the frame split)."""
import os
import socket

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


def _worker(rank, world, port, counts, res):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rollingdepth_amd.shard import _all_gather_rows, chunk_bounds, gather_snippets, local_rows, rank_subsets

    shape = (3, 2, 5)
    sub = rank_subsets(counts, world, rank)
    snippets = []
    for d, n in enumerate(counts):
        buf = torch.full((n, *shape), -1.0)
        for k in sub[d]:
            buf[k] = _snippet(d, k, shape)
        snippets.append(buf)
    per_d = gather_snippets(local_rows(snippets, counts, world, rank), counts, world)
    ok = all(torch.equal(per_d[d][k], _snippet(d, k, shape)) for d, n in enumerate(counts) for k in range(n))
    N = 11
    lo, hi = chunk_bounds(N, world)[rank]
    lat = _all_gather_rows(torch.arange(lo, hi).float().view(-1, 1).expand(-1, 4).contiguous(), N, world)
    ok = ok and torch.equal(lat[:, 0], torch.arange(N).float())
    res[rank] = int(ok)
    dist.destroy_process_group()


def test_gather_reassembles_single_process_layout():
    world = 2
    ctx = mp.get_context("spawn")
    res = ctx.Array("i", [0] * world)
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, [9, 5], res)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert list(res) == [1] * world
