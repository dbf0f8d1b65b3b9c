"""DepthAligner — drop-in for rollingdepth/depth_aligner.py:29-262 running on librdmi.

Same constructor keywords, same `run(snippet_ls, dilations)` contract and return value
(merged [N,1,H,W] in the snippets' dtype, scales / translations as [n_d,1,1] f32, loss history
as a list of (loss, min(summ), max(summ)) tuples).  The 2000-iteration Adam loop is enqueued
entirely on the device (aligner.hip); the only host sync is reading the loss history at the end.
"""
from __future__ import annotations

from typing import List

import torch

from . import kernels as K


MAX_DILATIONS = 8   # aligner.hip MAXD
MAX_ROWS = 64       # aligner.hip MAXR: Σ snippet lengths (rows of the reference's M / M_depth / B tensors)


def check_row_layout(lengths: List[int], num_iterations: int) -> None:
    """The reference scatters dilation i's slots into rows i·w_i .. i·w_i + w_i − 1 of [Σw, N, P]
    tensors (depth_aligner.py:169-188); rows past Σw raise its IndexError (first closure call).
    Also the limits of the aligner kernels (at most 8 dilations, at most 64 rows), checked here so
    that forward() / sharded_forward() reject such a job before any inference runs rather than at
    the aligner call after it."""
    rows = sum(lengths)
    if len(lengths) > MAX_DILATIONS:
        raise NotImplementedError(f"{len(lengths)} dilations: the aligner kernels take at most {MAX_DILATIONS}")
    if num_iterations > 0:
        for i, w in enumerate(lengths):
            if (i + 1) * w > rows:
                raise IndexError(f"index {(i + 1) * w - 1} is out of bounds for dimension 0 with size {rows}")
        if rows > MAX_ROWS:
            raise NotImplementedError(f"snippet lengths {list(lengths)} sum to {rows} aligner rows: the aligner "
                                      f"kernel takes at most {MAX_ROWS}")


class DepthAligner:
    def __init__(self, device: torch.device, factor: int = 10, lmda: float = 1e-1, lmda2: float = 1e-1,
                 lmda3: float = 1e1, lr: float = 1e-3, num_iterations: int = 2000, border: int = 2,
                 verbose: bool = False, depth_loss_weight: float = 1.0, loss_scale=1.0):
        self.factor = factor
        self.lmda = lmda  # kept for signature parity; unused by the reference loss too
        self.lr = lr
        self.num_iterations = num_iterations
        self.border = border
        self.verbose = verbose
        self.device = device
        self.lmda2 = lmda2
        self.depth_loss_weight = depth_loss_weight
        self.loss_scale = loss_scale
        self.lmda3 = lmda3

    def create_triplet_indices(self, sequence_length: int, gap: int, window_size: int) -> torch.Tensor:
        """depth_aligner.py:57-66."""
        gap += 1
        return torch.tensor([[i + j * gap for j in range(window_size)]
                             for i in range(sequence_length - (window_size - 1) * gap)])

    @staticmethod
    def sequence_length(counts: List[int], w: int, dilations: List[int]) -> int:
        """depth_aligner.py:70-76 (from the first dilation's snippet count)."""
        return counts[0] + (w - 1) * (dilations[0] - 1) + (w - 1)

    def prepare(self, flat: List[torch.Tensor], shift: torch.Tensor) -> List[torch.Tensor]:
        """Min shift, border crop, stride subsample (:78-92): [n_d, w, H, W] → f32 [n_d, w, P]."""
        return [K.aligner_prepare(s, shift, self.border, self.factor) for s in flat]

    def optimize_prepared(self, xs: List[torch.Tensor], strides: List[int], seq_len: int):
        """The 2000-iteration Adam loop (:123-229) on prepared inputs → (scales [n_d], trans [n_d],
        history [iters, 3] device tensor, workspace to keep alive until the stream consumed it)."""
        dev = xs[0].device
        scales = [torch.ones(x.shape[0], dtype=torch.float32, device=dev) for x in xs]
        trans = [torch.zeros(x.shape[0], dtype=torch.float32, device=dev) for x in xs]
        hist = torch.zeros((max(self.num_iterations, 1), 3), dtype=torch.float32, device=dev)
        ws = K.aligner_optimize(xs, scales, trans, strides, seq_len, self.lr, (0.5, 0.9), 1e-8, self.lmda2,
                                self.lmda3, self.depth_loss_weight, self.loss_scale, self.num_iterations, hist)
        return scales, trans, hist, ws

    def run(self, snippet_ls: List[torch.Tensor], dilations: List[int], merged_f32: bool = False):
        """depth_aligner.py:68-120.  merged_f32=True (the pipeline's internal use): the merge of f16
        snippets runs in f32 arithmetic and is returned in f32, without the reference's f16 roundings
        of s·x+t and of the merged map (RollingDepthPipeline.merge_f32).

        Snippet lengths may differ per dilation (snippet_ls[d] is [n_d, w_d, 1, H, W]): the sequence
        length comes from the first dilation (:70-76) and the loss uses the reference's row layout
        (row i·w_i + j for slot j of dilation i, :169-188 — see aligner.hip), including its
        IndexError when those rows run past Σ w_i."""
        dev = torch.device(self.device)
        snippet_ls = [s.to(dev) for s in snippet_ls]
        lengths = [s.shape[1] for s in snippet_ls]
        gaps = [d - 1 for d in dilations]
        seq_len = self.sequence_length([s.shape[0] for s in snippet_ls], lengths[0], dilations)
        for s, g, w in zip(snippet_ls, gaps, lengths):
            expect = seq_len - (w - 1) * (g + 1)
            if s.shape[0] != expect:
                raise ValueError(f"snippet count {s.shape[0]} != {expect} for dilation {g + 1} (length {w})")
        check_row_layout(lengths, self.num_iterations)
        dtype = snippet_ls[0].dtype
        flat = [s.reshape(s.shape[0], s.shape[1], s.shape[-2], s.shape[-1]).contiguous() for s in snippet_ls]
        # global min over every snippet (depth_aligner.py:78)
        mins = torch.stack([K.minmax(s) for s in flat]).reshape(-1)
        shift = K.minmax(mins)
        xs = self.prepare(flat, shift)
        strides = [g + 1 for g in gaps]
        scales, trans, hist, ws = self.optimize_prepared(xs, strides, seq_len)
        merged = K.aligner_merge(flat, scales, trans, strides, seq_len, shift, f32_arith=merged_f32)
        merged = (merged if merged_f32 else merged.to(dtype))[:, None]
        loss_ls = [tuple(r) for r in hist[: self.num_iterations].tolist()]
        del ws
        return (merged, [s.view(-1, 1, 1) for s in scales], [t.view(-1, 1, 1) for t in trans], loss_ls)
