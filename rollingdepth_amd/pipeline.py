"""RollingDepthPipeline — the reference's call surface (rollingdepth/rollingdepth_pipeline.py:52-740)
over the librdmi HIP path.

What stays exactly the reference's: argument names/defaults and checks of `forward` (:193-258),
dilation capping (:504-515, including its gap-vs-dilation comparison), snippet indices (:465-502),
the shared init noise broadcast to every frame (:282-288), rgb-latent-first channel concat
(:646-651), 1-step DDIM, decode + channel mean (:706-740), DepthAligner co-alignment and the
min/max renormalisation (:306-318), output layout (:345-353), and the in-place mutation of the
caller's `dilations` list (:246-252).

What is the build's own: snippets of a dilation are batched `snippet_batch` at a time through
one UNet call (the reference's processor only supports b = 1 per call; batching is
legal because each snippet's attention fold is independent), frames are encoded/decoded
`vae_batch` at a time, activations are NHWC f16 on the device, and nothing syncs with the host
until the outputs are copied back.  `init_noise` may be injected for parity runs (the reference
draws it from the device RNG).
"""
from __future__ import annotations

import json
import logging
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from . import kernels as K
from .aligner import DepthAligner, check_row_layout
from .config import RD_SCHEDULER, SD2_UNET, SD2_VAE
from .scheduler import DDIMScheduler
from .unet import UNet
from .vae import VAE
from . import weights as Wt

F16, F32 = torch.float16, torch.float32


@dataclass
class RollingDepthOutput:
    """rollingdepth_pipeline.py RollingDepthOutput (input_rgb, depth_pred, snippet_ls, depth_coaligned).

    The fork's CLI (run_video.py:587-606) was written against the IC-Light experiment's output
    (rollingimg_pipeline.py:424-433) and reads R_pred / G_pred / B_pred / aligned_snippet_pred_ls;
    for the depth pipeline those are filled (by __call__ only) as a compatibility decision
    (SURVEY.md §8b): R = G = B = depth·0.5 + 0.5 ([N,1,H,W] in [0,1], what run_video multiplies by
    255) and aligned_snippet_pred_ls = [the co-aligned depth repeated to 3 channels]."""
    input_rgb: torch.Tensor
    depth_pred: torch.Tensor
    snippet_ls: Optional[List[torch.Tensor]]
    depth_coaligned: Optional[torch.Tensor]
    R_pred: Optional[torch.Tensor] = None
    G_pred: Optional[torch.Tensor] = None
    B_pred: Optional[torch.Tensor] = None
    aligned_snippet_pred_ls: Optional[List[torch.Tensor]] = None

    def __getitem__(self, k):
        return getattr(self, k)


def _load_state_dict(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file

    for name in ("diffusion_pytorch_model.safetensors", "model.safetensors"):
        p = os.path.join(path, name)
        if os.path.exists(p):
            return {k: v.float() for k, v in load_file(p).items()}
    p = os.path.join(path, "diffusion_pytorch_model.bin")
    if os.path.exists(p):
        return {k: v.float() for k, v in torch.load(p, map_location="cpu", weights_only=True).items()}
    raise FileNotFoundError(f"no weights under {path}")


def _balanced(n: int, cap: int) -> List[Tuple[int, int]]:
    """[0, n) in ceil(n / cap) contiguous ranges of (nearly) equal size."""
    if n <= 0:
        return []
    nb = -(-n // max(1, cap))
    base, extra = divmod(n, nb)
    out, b0 = [], 0
    for i in range(nb):
        b1 = b0 + base + (1 if i < extra else 0)
        out.append((b0, b1))
        b0 = b1
    return out


def _resolve(d: torch.device) -> torch.device:
    """An index-less "cuda" names the current device."""
    if d.type == "cuda" and d.index is None:
        return torch.device("cuda", torch.cuda.current_device())
    return d


_PROGRESS = os.environ.get("RDMI_PROGRESS") == "1"


def _progress(msg: str) -> None:
    """RDMI_PROGRESS=1: wait for the device and print a progress line (long runs — e.g. the paper
    preset's 500 frames — must show life to a supervisor; off by default: it synchronises)."""
    if _PROGRESS:
        import sys
        import time

        torch.cuda.synchronize()
        print(f"[rdmi progress {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _contiguous_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Rank's share of `total` equal-cost units: W contiguous ranges of ceil(total/W)."""
    c = (total + world - 1) // world
    return min(rank * c, total), min((rank + 1) * c, total)


class RollingDepthPipeline:
    rgb_latent_scale_factor = 0.18215
    depth_latent_scale_factor = 0.18215
    N_CHANNEL_PER_LATENT = 4

    def __init__(self, unet: UNet, vae: VAE, scheduler: DDIMScheduler, text_encoder=None, tokenizer=None):
        self.unet, self.vae, self.scheduler = unet, vae, scheduler
        self.text_encoder, self.tokenizer = text_encoder, tokenizer
        self.empty_text_embed: Optional[torch.Tensor] = None
        self.snippet_batch = 25  # max snippets per UNet call (75 frames at snippet length 3)
        self.vae_batch = 75      # max frames per VAE encode / decode call (memory-capped: _vae_chunks)
        self._dev = unet.dev
        self._group = None  # torch.distributed group for snippet-parallel forward (enable_snippet_parallel)
        # merge_scaled_triplets of f16 snippets in f32 arithmetic, the merged map kept f32 through the
        # renormalisation (the reference's fp16 run rounds s·x+t and the merged map to f16 first; those
        # roundings of the extreme pixels rescale the whole renormalised map — tools/precision_probe.py:
        # 768² depth L1 vs the fp32 reference 1.13e-3 → 7.6e-4).  RDMI_MERGE_F32=0: the fp16 roundings.
        self.merge_f32 = os.environ.get("RDMI_MERGE_F32", "1") == "1"
        # The decoded depth (the decoder head's output, snippet_ls, the aligner / merge inputs and the
        # refined depth) is kept in f32 in the f16 pipeline: the f16 rounding of |d| ≈ 1–2 (ulp 1–2e-3)
        # otherwise reaches the global min/max renormalisation (rollingdepth_pipeline.py:316-318)
        # directly, where it moves the whole map.  The returned snippet_ls keeps the
        # reference's dtype (the pipeline's).  RDMI_DEPTH_F32=0: f16 decoded depth.
        self.depth_f32 = os.environ.get("RDMI_DEPTH_F32", "1") == "1"
        # Snippet decode on a second stream (RDMI_DECODE_STREAM=1, A/B): the VAE decode of UNet batch i runs
        # beside the UNet of batch i + 1, so each kernel's last partial round of workgroups and the
        # HBM-bound norm passes can share the chip with the other stream's kernels.  Every kernel computes
        # the same values either way (no cross-stream reductions): bitwise the serial forward.
        self.decode_stream = os.environ.get("RDMI_DECODE_STREAM", "0") == "1"
        self._dstream = None

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_pretrained(cls, path: str, torch_dtype=torch.float16, device="cuda", **kw) -> "RollingDepthPipeline":
        """Diffusers-format checkpoint directory (model_index.json, unet/, vae/, scheduler/;
        pipeline_utils.py:480).  Weights via safetensors (or torch.load(weights_only=True))."""
        dtype = torch.float16 if torch_dtype is None else torch_dtype
        if dtype not in (torch.float16, torch.float32):
            raise NotImplementedError(f"torch_dtype {torch_dtype}: the HIP path runs float16 or float32")
        rd = lambda sub: json.load(open(os.path.join(path, sub, "config.json" if sub != "scheduler" else "scheduler_config.json")))
        ucfg, vcfg, scfg = rd("unet"), rd("vae"), rd("scheduler")
        unet = UNet(ucfg, _load_state_dict(os.path.join(path, "unet")), device, dtype)
        vae = VAE(vcfg, _load_state_dict(os.path.join(path, "vae")), device, dtype)
        pipe = cls(unet, vae, DDIMScheduler.from_config(scfg))
        if os.path.isdir(os.path.join(path, "text_encoder")) and os.path.isdir(os.path.join(path, "tokenizer")):
            # encode_empty_text (rollingdepth_pipeline.py:178-191), once at load: the only use of
            # text_encoder / tokenizer on the depth path (text_encoder.py)
            from .text_encoder import empty_text_embedding
            pipe.empty_text_embed = empty_text_embedding(path, dtype)
        else:
            emb = os.path.join(path, "empty_text_embed.safetensors")
            if os.path.exists(emb):
                from safetensors.torch import load_file
                pipe.empty_text_embed = load_file(emb)["embed"]
        return pipe

    @classmethod
    def from_synthetic(cls, unet_cfg=SD2_UNET, vae_cfg=SD2_VAE, sched_cfg=RD_SCHEDULER, seed: int = 0,
                       device="cuda", torch_dtype=torch.float16) -> "RollingDepthPipeline":
        """Random-init weights of the architecture (no checkpoint in the image), deterministic
        per state-dict key (weights.py) — identical to what the golden fixtures used."""
        unet = UNet(unet_cfg, Wt.synth_state_dict(Wt.unet_param_shapes(unet_cfg), seed), device, torch_dtype)
        vae = VAE(vae_cfg, Wt.synth_state_dict(Wt.vae_param_shapes(vae_cfg), seed), device, torch_dtype)
        pipe = cls(unet, vae, DDIMScheduler.from_config(sched_cfg))
        pipe.empty_text_embed = Wt.synth_context(unet_cfg["cross_attention_dim"], seed)
        return pipe

    @property
    def device(self) -> torch.device:
        return self._dev

    @property
    def dtype(self):
        return self.unet.dtype

    @property
    def depth_dtype(self):
        """Storage dtype of decoded depth on the device (f32 unless RDMI_DEPTH_F32=0)."""
        return F32 if self.depth_f32 else self.dtype

    def to(self, *args, **kwargs):
        """DiffusionPipeline.to (pipeline_utils.py:303): weights already live on the device the
        pipeline was built for.  Accepts that device (an index-less "cuda" names the current device),
        a dtype equal to the pipeline's, or both; anything else raises."""
        for a in list(args) + list(kwargs.values()):
            if a is None:
                continue
            if isinstance(a, torch.dtype):
                if a != self.dtype:
                    raise NotImplementedError(f"pipeline built for {self.dtype}; rebuild it with torch_dtype={a}")
                continue
            d, mine = _resolve(torch.device(a)), _resolve(self._dev)
            if d != mine:
                raise NotImplementedError(f"pipeline lives on {mine}; construct it on {d} instead")
        return self

    def enable_snippet_parallel(self, group=None):
        """Run forward() snippet-parallel over the ranks of `group` (default: the world group; one
        process per GPU, torch.distributed initialised with backend "nccl" = RCCL).  Every rank calls
        forward() with the same arguments and receives the full outputs (shard.py holds the plan)."""
        import torch.distributed as dist
        self._group = group if group is not None else dist.group.WORLD
        return self

    def enable_xformers_memory_efficient_attention(self, attention_op=None):
        """pipeline_utils.py:1630.  The cross-frame attention of every UNet / VAE Attention already runs
        on librdmi's fused flash kernel (memory-efficient by construction), so this only records the
        request; run_video.py:534-538 calls it unconditionally."""
        self._xformers_requested = True

    def disable_xformers_memory_efficient_attention(self):
        self._xformers_requested = False

    def encode_empty_text(self):
        """rollingdepth_pipeline.py:178-191.  from_pretrained computes the constant embedding from the
        checkpoint's text_encoder/ + tokenizer/ (text_encoder.py); with a transformers tokenizer and
        text encoder handed to the constructor, they are run here as the reference runs them."""
        if self.text_encoder is None or self.tokenizer is None:
            raise RuntimeError("empty_text_embed not set and no text encoder available")
        ids = self.tokenizer("", padding="do_not_pad", max_length=self.tokenizer.model_max_length, truncation=True,
                             return_tensors="pt").input_ids
        with torch.no_grad():
            self.empty_text_embed = self.text_encoder(ids)[0].to(self.dtype)

    # ------------------------------------------------------------------ reference helpers
    @staticmethod
    def get_snippet_indice(i_step: int, timesteps, seq_len: int, snippet_len: int, dilation_start: int,
                           dilation_end: int, stride: int) -> List[List[int]]:
        gap_start, gap_end = dilation_start - 1, dilation_end - 1
        assert gap_start >= gap_end, f"expect gap_start > gap_end, but got {gap_start} and {gap_end}"
        assert gap_start >= 0 and gap_end >= 0
        total = len(timesteps)
        gap = int((1 - i_step / total) * (gap_start - gap_end) + gap_end)
        win = (snippet_len - 1) * (gap + 1) + 1
        starts = list(range(0, seq_len - win + 1, stride))
        if starts[-1] < seq_len - win:
            starts.append(seq_len - win)
        idx = [list(range(s, s + win, gap + 1)) for s in starts]
        if set(range(seq_len)) != {x for f in idx for x in f}:
            logging.warning("Not every frame is covered. Consider reducing dilation for short videos")
        return idx

    @staticmethod
    def cap_max_dilation(seq_len: int, snippet_len: int, dilation: int, verbose: bool = False) -> int:
        max_gap = int(seq_len / snippet_len) - 1
        if max_gap < dilation:
            (logging.info if verbose else logging.debug)(
                f"dilation = {dilation} is too big for {seq_len} frames. Reduced to {max_gap}")
            dilation = min(max_gap, dilation)
        return dilation

    # ------------------------------------------------------------------ host <-> device plumbing
    def _device_index(self, values) -> torch.Tensor:
        """int32 index list → device tensor through pinned memory, without a host sync (a plain
        torch.tensor(..., device=) waits for the stream and drains the GPU's queue)."""
        t = torch.tensor(values, dtype=torch.int32).pin_memory()
        return t.to(self.device, non_blocking=True)

    @staticmethod
    def _to_host_async(t: torch.Tensor, stream) -> torch.Tensor:
        """Enqueue a device→host copy into pinned memory on `stream` (after the work queued so far
        on the current stream).  The result is valid once `stream` is synchronised."""
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        stream.wait_stream(torch.cuda.current_stream(t.device))
        with torch.cuda.stream(stream):
            h.copy_(t, non_blocking=True)
        t.record_stream(stream)
        return h

    def _noise_nhwc(self, init_noise: torch.Tensor, h: int, w: int) -> torch.Tensor:
        """[1, 4, h, w] (or [4, h, w]) init noise → NHWC [1, h, w, 8] on the device; the shape is checked
        because the UNet-input gather broadcasts h·w pixels out of it."""
        n = init_noise if init_noise.dim() == 4 else init_noise[None]
        if tuple(n.shape) != (1, self.N_CHANNEL_PER_LATENT, h, w):
            raise ValueError(f"init_noise shape {tuple(init_noise.shape)} != (1, 4, {h}, {w}) (the latent size)")
        return K.nchw_to_nhwc(n.to(self.device), 8, dtype=self.dtype)

    # ------------------------------------------------------------------ stages
    def encode_rgb(self, frames_nchw: torch.Tensor) -> torch.Tensor:
        """[N,3,H,W] in [-1,1] (any float dtype, on device) → NHWC f16 [N, h, w, 8] latents·0.18215."""
        N, _, H, W = frames_nchw.shape
        h, w = self.vae.latent_hw(H, W)
        out = torch.zeros((N, h, w, self.vae.lat_pad), dtype=self.dtype, device=self.device)
        for i0, i1 in self._vae_chunks(N, h, w):
            x = K.nchw_to_nhwc(frames_nchw[i0:i1], self.vae.in_pad, dtype=self.dtype)
            self.vae.encode(x, out=out[i0:i1])
        return out

    def _vae_chunks(self, n: int, h: int, w: int) -> List[Tuple[int, int]]:
        """Balanced VAE chunks of at most vae_batch frames, capped so that one full-resolution
        128-channel activation stays ≤ 24 GB and — where the mid-block attention materialises its f32
        scores ([b, h·w, h·w]: the f32 path, or RDMI_VAE_FLASH=0) — the scores ≤ 32 GB.  The f16 flash
        kernel (attention_d512.hip) holds no scores, so f16 chunks are not capped by them (768²: 75
        frames, 1024²: 75 — the scores cap was 62 / 19).  Measured at 768² (75-frame snippet
        batches, round 1): 16 → 21.0, 38 → 21.1, 75 → 21.2 depth frames/s (profiles/r01_vae_batch_ab.log)."""
        hw = h * w
        esz = self.dtype.itemsize  # (f32 path: the probabilities are f32 too, and every activation doubles)
        cap = min(self.vae_batch, max(1, int(24e9 // (hw * 64 * 128 * esz))))
        if self.dtype == F32 or os.environ.get("RDMI_VAE_FLASH", "1") == "0":
            cap = min(cap, max(1, int(32e9 // (hw * hw * (4 + esz)))))
        return _balanced(n, cap)

    def decode_depth(self, z_scaled: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """z_scaled: NHWC [B, h, w, 8] already divided by 0.18215 → out [B, H, W, 1] depth (f16 / f32)."""
        for i0, i1 in self._vae_chunks(z_scaled.shape[0], z_scaled.shape[1], z_scaled.shape[2]):
            self.vae.decode_depth(z_scaled[i0:i1], out=out[i0:i1])
        return out

    def _context(self) -> torch.Tensor:
        if self.empty_text_embed is None:
            self.encode_empty_text()
        ctx = self.empty_text_embed
        if getattr(self, "_ctx16_src", None) is not ctx:
            self._ctx16 = ctx.to(self.device, self.dtype).contiguous()
            self._ctx16_src = ctx
            self.unet.set_context(self._ctx16)
        return self._ctx16

    def _snippet_batches(self, n: int, slen: int, h: int, w: int) -> List[Tuple[int, int]]:
        """Split n snippets into ceil(n / cap) UNet batches of (nearly) equal size: no small trailing
        batch (98 snippets at cap 25 → 25, 25, 24, 24; measured: 16-snippet batches with 2-snippet
        tails 20.6, 25-snippet balanced batches 20.9 depth frames/s).  The cap also keeps the largest
        UNet activation — the [b·slen·h·w, 4·C0] GEGLU output feeding ff2 — below 2^31 bytes (the
        kernels' 32-bit buffer offsets): 30 snippets at 96², 17 at 128²."""
        c0 = int(self.unet.cfg["block_out_channels"][0])
        esz = self.dtype.itemsize
        return _balanced(n, max(1, min(self.snippet_batch, (2 ** 31 - 1) // (slen * h * w * 4 * c0 * esz))))

    def init_snippet_infer(self, rgb_latent: torch.Tensor, init_noise: torch.Tensor, dilations: List[int],
                           snippet_lengths: List[int], init_infer_steps: List[int], strides: List[int],
                           snippet_subset=None, record: Optional[dict] = None) -> List[torch.Tensor]:
        """rollingdepth_pipeline.py:356-463 with snippets batched per UNet call.
        rgb_latent NHWC [N,h,w,8]; init_noise NHWC [1,h,w,8].  Returns per dilation the decoded
        snippets [n_d, w, H, W] in depth_dtype (device).  `snippet_subset[d]` (optional) restricts the work
        to those snippet indices (multi-GPU sharding); other rows are left uninitialised.  With a
        subset, the snippets of consecutive dilations that share a snippet length and a DDIM step count
        run in the same UNet batches and decode chunks (a rank of an 8-way split holding 3 snippets of
        one dilation and 16 of the next runs one 19-snippet batch, not 3 + 16: bench.py --slice-world,
        DESIGN.md §5); the per-dilation outputs are then consecutive views of one buffer."""
        self._context()
        N, h, w, _ = rgb_latent.shape
        H, W = h * self.vae.factor, w * self.vae.factor
        jobs = []  # (dilation index, snippet list, frame indices per snippet)
        for di, (dil, slen, stride, steps) in enumerate(zip(dilations, snippet_lengths, strides, init_infer_steps)):
            self.scheduler.set_timesteps(steps)
            idx = self.get_snippet_indice(0, self.scheduler.timesteps, N, slen, dil, dil, stride)
            todo = list(range(len(idx))) if snippet_subset is None else list(snippet_subset[di])
            jobs.append((di, todo, [idx[k] for k in todo]))
        groups = []  # runs of dilations batched together
        for di, todo, fr in jobs:
            key = (snippet_lengths[di], init_infer_steps[di])
            if snippet_subset is not None and groups and groups[-1][0] == key:
                groups[-1][1].append((di, todo, fr))
            else:
                groups.append((key, [(di, todo, fr)]))
        outs: List[Optional[torch.Tensor]] = [None] * len(dilations)
        ds = None
        if self.decode_stream and self.device.type == "cuda":
            if self._dstream is None:
                self._dstream = torch.cuda.Stream(self.device)
            ds = self._dstream
        for (slen, steps), members in groups:
            self.scheduler.set_timesteps(steps)
            timesteps = self.scheduler.timesteps
            ntodo = sum(len(t) for _, t, _ in members)
            # row r of the group buffer is the r-th snippet of the members' todo lists, in order
            buf = torch.empty((ntodo, slen, H, W), dtype=self.depth_dtype, device=self.device)
            o = 0
            for di, todo, _ in members:
                outs[di] = buf[o:o + len(todo)]
                o += len(todo)
            fidx_all = self._device_index([f for _, _, fr in members for s in fr for f in s]) if ntodo else None
            for b0, b1 in self._snippet_batches(ntodo, slen, h, w):
                nb = b1 - b0
                fidx = fidx_all[b0 * slen:b1 * slen]
                x = K.gather_unet_input(rgb_latent, init_noise, fidx, depth_bcast=True)
                depth_view = x[..., 4:8]
                for si, t in enumerate(timesteps.tolist()):
                    pred = self.unet.forward(x, int(t), num_view=slen)
                    last = si == len(timesteps) - 1
                    if record is not None:  # every UNet call (the reference's single_step outputs)
                        record.setdefault("unet_out", []).append(pred)
                    if last:
                        zin = self.scheduler.step_(pred, int(t), depth_view, 1.0 / self.depth_latent_scale_factor,
                                                   channels=self.N_CHANNEL_PER_LATENT,
                                                   out=torch.empty((x.shape[0], h, w, 8), dtype=self.dtype,
                                                                   device=self.device))
                        if record is not None:
                            record.setdefault("snippet_latent", []).append(
                                self.scheduler.step_(pred, int(t), depth_view, 1.0, channels=4,
                                                     out=torch.empty((x.shape[0], h, w, 8), dtype=self.dtype,
                                                                     device=self.device)))
                    else:
                        x2 = x.clone()
                        self.scheduler.step_(pred, int(t), depth_view, 1.0, channels=4, out=x2[..., 4:])
                        x = x2
                        depth_view = x[..., 4:8]
                if ds is None:
                    self.decode_depth(zin, buf[b0:b1].view(nb * slen, H, W, 1))
                else:  # the decode waits for this batch's DDIM step; the next UNet batch does not wait for it
                    ev = torch.cuda.Event()
                    ev.record()
                    with torch.cuda.stream(ds):
                        ds.wait_event(ev)
                        self.decode_depth(zin, buf[b0:b1].view(nb * slen, H, W, 1))
                    zin.record_stream(ds)
                _progress(f"dilations {[dilations[m[0]] for m in members]}: snippets {b1}/{ntodo} decoded")
        if ds is not None:  # the decoded snippets are read on the launch stream from here on
            done = torch.cuda.Event()
            done.record(ds)
            torch.cuda.current_stream().wait_event(done)
        return outs

    def refine(self, rgb_latent: torch.Tensor, depth_latents: torch.Tensor, init_noise: torch.Tensor,
               refine_step: int, snippet_len: int, start_dilation: int, skip_t_ratio: float = 0.5,
               group=None) -> torch.Tensor:
        """rollingdepth_pipeline.py:517-633 on device.  rgb_latent / depth_latents NHWC [N,h,w,8]
        (channels 0..3), init_noise NHWC [1,h,w,8].  Returns the refined latents [N,h,w,8].

        `group` (a torch.distributed process group of W > 1 ranks): every rank
        holds all N latents; each step's snippet list is split into W contiguous ranges, each rank runs
        the UNet on its range and sums its predictions per frame, and one all-reduce SUM of the
        [N, h·w, 4] f32 sums (+ the cover count, which is data-independent) gives every rank the
        step's averaged latents."""
        world, rank = 1, 0
        if group is not None:
            from .shard import _rank, _world
            world, rank = _world(group), _rank(group)
        self._context()
        N, h, w, _ = rgb_latent.shape
        T = int(refine_step / skip_t_ratio)
        assert T <= self.scheduler.config["num_train_timesteps"], "Too many refinement steps"
        self.scheduler.set_timesteps(T)
        timesteps = self.scheduler.timesteps
        start = int(len(timesteps) * skip_t_ratio)
        ts = timesteps[start:].tolist()
        assert 0 < len(ts) < T, f"invalid {skip_t_ratio = }"
        sa, sb = self.scheduler.add_noise_coefficients(ts[0])
        new = K.ddim_combine(depth_latents[..., :4], init_noise[..., :4], sa, sb, 1.0, 4, 8)
        for i_step, t in enumerate(ts):
            idx = self.get_snippet_indice(i_step, ts, N, snippet_len, start_dilation, 1, 1)
            stride = idx[0][1] - idx[0][0] if snippet_len > 1 else 1
            covered = {f for s in idx for f in s}
            assert len(covered) == N, "refine: every frame must be covered by a snippet"
            lo, hi = _contiguous_range(len(idx), world, rank)
            mine = idx[lo:hi]
            preds = torch.empty((len(mine), snippet_len, h, w, 8), dtype=self.dtype, device=self.device)
            fidx_all = self._device_index([f for s in mine for f in s]) if mine else None
            for b0, b1 in self._snippet_batches(len(mine), snippet_len, h, w):
                sel = mine[b0:b1]
                fidx = fidx_all[b0 * snippet_len:(b0 + len(sel)) * snippet_len]
                x = K.gather_unet_input(rgb_latent, new, fidx, depth_bcast=False)
                pred = self.unet.forward(x, int(t), num_view=snippet_len)
                self.scheduler.step_(pred, int(t), x[..., 4:8], 1.0, channels=4,
                                     out=preds[b0:b0 + len(sel)].view(len(sel) * snippet_len, h, w, 8))
            _progress(f"refine step {i_step + 1}/{len(ts)}: {len(mine)} snippets")
            if world == 1:
                new = K.snippet_average(preds, stride, N)
            else:
                from .shard import _all_reduce
                sums = K.snippet_accumulate(preds, lo, stride, N)
                _all_reduce(sums, group=group)
                new = K.snippet_finish(sums, len(idx), snippet_len, stride, (h, w), 8, dtype=self.dtype)
        return new

    # ------------------------------------------------------------------ entry points
    @torch.no_grad()
    def __call__(self, input_video_path=None, start_frame: int = 0, frame_count: int = 0, processing_res: int = 1024,
                 resample_method: str = "BILINEAR", dilations: List[int] = [1, 25], cap_dilation: bool = True,
                 snippet_lengths: List[int] = [3], init_infer_steps: List[int] = [1], strides: List[int] = [1],
                 coalign_kwargs: Union[Dict, None] = None, refine_step: int = 0, refine_snippet_len: int = 3,
                 refine_start_dilation: int = 6, generator: Union[torch.Generator, None] = None,
                 verbose: bool = False, max_vae_bs: int = 4, unload_snippet: bool = False,
                 restore_res: bool = False, input_fg_video_path=None, **kw) -> RollingDepthOutput:
        """rollingdepth_pipeline.py:78-176.  `input_video_path` (or the fork's `input_fg_video_path`):
        a video file (decoding needs PyAV, absent from this image), decoded uint8 rgb24 frames
        [N, H, W, 3] (numpy / torch: resized to processing_res and normalised on the device,
        video_io.load_video_frames), or an already-normalised float [N, 3, H, W] tensor in [-1, 1]
        (used as is: processing_res and restore_res do not apply to it)."""
        assert processing_res >= 0
        if processing_res > 1024:
            logging.warning(f"Procssing at high-resolution ({processing_res}) may lead to suboptimal accuracy.")
        src = input_fg_video_path if input_fg_video_path is not None else input_video_path
        original_res = None
        if isinstance(src, torch.Tensor) and src.is_floating_point():
            frames = src
        else:
            from .video_io import load_video_frames
            frames, original_res = load_video_frames(src, start_frame, frame_count, processing_res, resample_method,
                                                     verbose, device=self.device)
        if restore_res:
            if original_res is None:
                raise ValueError("restore_res needs the original resolution: pass the video or its decoded uint8 "
                                 "frames, not a normalised tensor")
            if max(original_res) > 2048:
                logging.warning(f"Resizing back to large resolution ({list(original_res)}) may result in significant "
                                "memory usage.")
        kw.pop("input_bg_video_path", None)  # fork CLI (run_video.py:563): IC-Light background, unused here
        out = self.forward(frames[None] if frames.dim() == 4 else frames, dilations, cap_dilation, snippet_lengths,
                           init_infer_steps, strides, coalign_kwargs, refine_step, refine_snippet_len,
                           refine_start_dilation, generator, verbose, max_vae_bs, unload_snippet, **kw)
        if restore_res:  # rollingdepth_pipeline.py:155-173 (torchvision resize, antialias=True), on the device
            for name in ("input_rgb", "depth_pred"):
                t = getattr(out, name)
                r = K.resize(t.to(self.device, torch.float32), original_res, resample_method.upper())
                setattr(out, name, r.to(t.dtype).cpu())
        if input_fg_video_path is not None:
            rgb = out.depth_pred.float() * 0.5 + 0.5
            out.R_pred = out.G_pred = out.B_pred = rgb
            out.aligned_snippet_pred_ls = [out.depth_coaligned.float().expand(-1, 3, -1, -1)]
        return out

    def _forward_sharded(self, input_frames, dilations, snippet_lengths, init_infer_steps, coalign_kwargs, refine_step,
                         refine_snippet_len, refine_start_dilation, init_noise, record, generator=None):
        """forward() over W ranks (shard.sharded_forward), outputs assembled on every rank.  Dilations
        arrive already capped (forward's checks ran); the snippets are all-gathered at full
        resolution only here, to honour the snippet_ls contract (bench.py keeps them distributed)."""
        import torch.distributed as dist
        from .shard import gather_rows_by_dilation, sharded_forward

        world = dist.get_world_size(self._group)
        so = sharded_forward(self, input_frames, list(dilations), False, list(snippet_lengths), coalign_kwargs,
                             init_noise=init_noise, group=self._group, refine_step=refine_step,
                             refine_snippet_len=refine_snippet_len, refine_start_dilation=refine_start_dilation,
                             gather=True, record=record, generator=generator,
                             init_infer_steps=list(init_infer_steps))
        snips = gather_rows_by_dilation([r.to(self.dtype) for r in so.snippet_rows], so.snippet_counts, world,
                                        self._group)
        H, W = so.depth_pred_full.shape[-2:]
        d2h = torch.cuda.Stream(self.device)
        snip_host = [self._to_host_async(s.view(s.shape[0], s.shape[1], 1, H, W), d2h) for s in snips]
        rgb = input_frames[0].to(self.device, self.dtype) / 2.0 + 0.5
        outs = [self._to_host_async(t, d2h) for t in (rgb, so.depth_pred_full, so.depth_coaligned_full)]
        d2h.synchronize()
        return RollingDepthOutput(input_rgb=outs[0], depth_pred=outs[1], snippet_ls=snip_host,
                                  depth_coaligned=outs[2])

    @torch.no_grad()
    def forward(self, input_frames: torch.Tensor, dilations: List[int], cap_dilation: bool,
                snippet_lengths: List[int], init_infer_steps: List[int], strides: List[int],
                coalign_kwargs: Union[Dict, None], refine_step: int, refine_snippet_len: int,
                refine_start_dilation: int, generator: Union[torch.Generator, None], verbose: bool,
                max_vae_bs: int, unload_snippet: bool, init_noise: Optional[torch.Tensor] = None,
                record: Optional[dict] = None) -> RollingDepthOutput:
        # ----------------- checks (rollingdepth_pipeline.py:214-252)
        assert 1 in dilations, "dilations should include 1"
        assert len(snippet_lengths) == len(set(snippet_lengths)), f"Repeated values found in {snippet_lengths = }"
        if len(snippet_lengths) > 1:
            assert len(snippet_lengths) == len(dilations)
        else:
            snippet_lengths = snippet_lengths * len(dilations)
        if len(init_infer_steps) > 1:
            assert len(init_infer_steps) == len(dilations)
        else:
            init_infer_steps = init_infer_steps * len(dilations)
        assert min(init_infer_steps) > 0, "Minimum inference step is 1"
        if len(strides) > 1:
            assert len(strides) == len(dilations)
        else:
            strides = strides * len(dilations)
        if [1] * len(dilations) != strides:
            raise NotImplementedError("Only implemented for stride 1")
        seq_len = input_frames.shape[1]
        if cap_dilation:
            for i, d in enumerate(dilations):
                dilations[i] = self.cap_max_dilation(seq_len, snippet_lengths[i], d, verbose)
            refine_start_dilation = self.cap_max_dilation(seq_len, refine_snippet_len, refine_start_dilation, verbose)
        if input_frames.shape[0] != 1:
            raise NotImplementedError("Layered inference is only implemented for B=1")
        # the aligner's row layout / kernel limits, before any inference (the reference fails there
        # only at its first optimisation step, after all snippets are denoised)
        check_row_layout(snippet_lengths, int((coalign_kwargs or {}).get("num_iterations", 2000)))
        if self._group is not None:
            import torch.distributed as dist
            if dist.get_world_size(self._group) > 1:
                return self._forward_sharded(input_frames, dilations, snippet_lengths, init_infer_steps, coalign_kwargs,
                                             refine_step, refine_snippet_len, refine_start_dilation, init_noise,
                                             record, generator)
        # ----------------- encode (H2D boundary :263)
        frames = input_frames[0].to(self.device)
        # input_rgb = frames / 2 + 0.5 in f16 as the reference computes it on the host (x/2 is exact,
        # the +0.5 rounds identically), evaluated on the device; its D2H copy is queued now so that it
        # runs under the denoising instead of at the end of the call
        d2h = torch.cuda.Stream(self.device)
        rgb_host = self._to_host_async(frames.to(self.dtype) / 2.0 + 0.5, d2h)
        rgb_latent = self.encode_rgb(frames)
        N, h, w, _ = rgb_latent.shape
        # ----------------- shared init noise (:282-288)
        if init_noise is None:
            init_noise = torch.randn((1, 4, h, w), device=self.device, dtype=self.dtype, generator=generator)
        noise = self._noise_nhwc(init_noise, h, w)
        snippets = self.init_snippet_infer(rgb_latent, noise, dilations, snippet_lengths, init_infer_steps, strides,
                                           record=record)
        # snippet_ls D2H (the reference returns it on the host) overlaps the aligner's kernels
        H, W = snippets[0].shape[-2:]
        snip_host = [self._to_host_async(s.to(self.dtype).view(s.shape[0], s.shape[1], 1, H, W), d2h)
                     for s in snippets]
        # ----------------- co-alignment + renormalisation (:306-318)
        aligner = DepthAligner(device=self.device, verbose=verbose, **(coalign_kwargs or {}))
        merged, scales, trans, hist = aligner.run([s.view(s.shape[0], s.shape[1], 1, H, W) for s in snippets],
                                                  dilations, merged_f32=self.merge_f32)
        d = merged.float().contiguous()
        K.renormalize_(d, K.minmax(d))
        coaligned = d.to(self.dtype)
        _progress("co-alignment done")
        if record is not None:
            record.update(rgb_latent=rgb_latent, scales=scales, translations=trans, loss_history=hist,
                          dilations=list(dilations))
        # ----------------- refinement (:323-343, full/paper presets)
        if refine_step > 0:
            dlat = self.encode_rgb(coaligned.expand(-1, 3, -1, -1))
            new = self.refine(rgb_latent, dlat, noise, refine_step, refine_snippet_len, refine_start_dilation)
            if record is not None:
                record["refined_latent"] = new
            z = K.ddim_combine(new[..., :4], new[..., :4], 1.0 / self.depth_latent_scale_factor, 0.0, 1.0, 4, 8)
            dec = torch.empty((N, H, W, 1), dtype=self.depth_dtype, device=self.device)
            self.decode_depth(z, dec)
            depth = dec.view(N, 1, H, W).to(self.dtype)
        else:
            depth = coaligned
        # ----------------- outputs (:345-353, D2H boundary; pinned, async, one sync)
        outs = [self._to_host_async(t, d2h) for t in (depth, coaligned)]
        d2h.synchronize()
        return RollingDepthOutput(input_rgb=rgb_host, depth_pred=outs[0], snippet_ls=snip_host,
                                  depth_coaligned=outs[1])
