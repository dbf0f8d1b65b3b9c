"""Video ingest and egress — rollingdepth/video_io.py.

Decoding and encoding need PyAV (absent from this image): `load_video_frames` on a path and
`write_video_from_numpy` raise ImportError saying so (the PyAV calls themselves are written and
exercised against a stand-in module in tests/test_host_cpu.py).  Everything after the decode runs on the
device: given decoded rgb24 frames (what PyAV's `frame.to_ndarray(format="rgb24")` returns,
uint8 [N, H, W, 3] — numpy or torch), `load_video_frames` uploads the uint8 frames (a quarter of
the PCIe bytes of the reference's float frames) and resizes + normalises them in one librdmi pass
(`rdmi_resize`: torchvision resize(antialias=True) then (x / 255)·2 − 1, video_io.py:104-123).
`resize_max_res` is video_io.py:38-67 on the device."""
from __future__ import annotations

import os
from typing import Tuple, Union

import numpy as np
import torch

from . import kernels as K


def _target_size(h: int, w: int, max_edge_resolution: int) -> Tuple[int, int]:
    """video_io.py:58-65 (Python float arithmetic, int() truncation)."""
    downscale_factor = min(max_edge_resolution / w, max_edge_resolution / h)
    return int(h * downscale_factor), int(w * downscale_factor)


def resize_max_res(img: torch.Tensor, max_edge_resolution: int, resample_method: str = "BILINEAR") -> torch.Tensor:
    """video_io.py:38-67: [B, C, H, W] (float32 or uint8, on the device) resized so that the longer edge
    is max_edge_resolution, aspect ratio kept → f32 [B, C, h, w]."""
    assert 4 == img.dim(), f"Invalid input shape {img.shape}"
    h, w = _target_size(img.shape[-2], img.shape[-1], max_edge_resolution)
    return K.resize(img, (h, w), str(resample_method).upper().split(".")[-1])


def frames_from_rgb24(frames: Union[np.ndarray, torch.Tensor], processing_res: int = 0,
                      resample_method: str = "BILINEAR", device="cuda") -> Tuple[torch.Tensor, Tuple[int, int]]:
    """Decoded uint8 [N, H, W, 3] frames → (f32 [N, 3, h, w] in [-1, 1] on the device, (H, W)):
    video_io.py:104-123 for every frame at once."""
    if isinstance(frames, np.ndarray):
        frames = torch.from_numpy(np.ascontiguousarray(frames))
    if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3:
        raise ValueError(f"expected uint8 [N, H, W, 3] rgb24 frames, got {frames.dtype} {tuple(frames.shape)}")
    if frames.shape[0] == 0:
        raise RuntimeError("No frame is loaded")
    n, h0, w0, _ = frames.shape
    dev = frames.to(device, non_blocking=True)
    h, w = _target_size(h0, w0, processing_res) if processing_res > 0 else (h0, w0)
    out = K.resize(dev, (h, w), str(resample_method).upper().split(".")[-1], normalize=True, channels_last=True)
    return out, (h0, w0)


def load_video_frames(input_path, start_frame: int = 0, frame_count: int = 0, processing_res: int = 0,
                      resample_method: str = "BILINEAR", verbose: bool = False, device="cuda"):
    """video_io.py:71-137.  `input_path`: a video file (needs PyAV) or already-decoded uint8 rgb24
    frames [N, H, W, 3] (numpy / torch).  Returns (f32 [N, 3, h, w] in [-1, 1] on `device`, (H, W))."""
    assert start_frame >= 0
    if isinstance(input_path, (np.ndarray, torch.Tensor)):
        frames = input_path
        end = start_frame + frame_count if frame_count > 0 else frames.shape[0]
        frames = frames[start_frame:end]
        if frames.shape[0] == 0:
            raise RuntimeError("No frame is loaded from the given frames")
        return frames_from_rgb24(frames, processing_res, resample_method, device)
    if not isinstance(input_path, (str, os.PathLike)):
        raise TypeError(f"load_video_frames: a path or uint8 [N, H, W, 3] frames, got {type(input_path)}")
    try:
        import av
    except ImportError as e:
        raise ImportError("video decoding needs PyAV, which is not installed in this image; decode the video "
                          "elsewhere and pass the uint8 [N, H, W, 3] rgb24 frames instead") from e
    container = av.open(input_path)  # pragma: no cover — PyAV absent here
    try:
        stream = container.streams.video[0]
        stream.thread_type = "AUTO"
        end_before = start_frame + frame_count if frame_count > 0 else np.inf
        frame_ls = []
        for i, frame in enumerate(container.decode(stream)):
            if i >= end_before:
                break
            if i >= start_frame:
                frame_ls.append(frame.to_ndarray(format="rgb24"))
    finally:
        container.close()
    if not frame_ls:
        raise RuntimeError(f"No frame is loaded from {input_path}")
    return frames_from_rgb24(np.stack(frame_ls), processing_res, resample_method, device)


def write_video_from_numpy(frames: np.ndarray, output_path, fps: int = 30, codec=None, crf: int = 23,
                           preset: str = "medium", verbose: bool = False) -> None:
    """video_io.py:140-208: uint8 rgb24 frames [n, H, W, 3] → a video file through PyAV (absent from
    this image: ImportError).  Codec: the given one, else the first of libx264 / h264 / mpeg4 / mjpeg
    that PyAV knows (ValueError when none does); yuv420p; crf / preset only for the x264 codecs; one
    rgb24 frame per input frame, then the encoder flushed."""
    if len(frames.shape) != 4 or frames.shape[-1] != 3:
        raise ValueError(f"Expected shape [n, height, width, 3], got {frames.shape}")
    if frames.dtype != np.uint8:
        raise ValueError(f"Expected dtype uint8, got {frames.dtype}")
    try:
        import av
    except ImportError as e:
        raise ImportError("video encoding needs PyAV, which is not installed in this image") from e
    n, height, width, _ = frames.shape
    candidates = [codec] if codec is not None else ["libx264", "h264", "mpeg4", "mjpeg"]
    container = stream = chosen = None
    for c in candidates:
        container = av.open(output_path, mode="w")
        try:
            stream = container.add_stream(c, rate=fps)
        except av.codec.codec.UnknownCodecError:
            container.close()
            continue
        chosen = c
        break
    if chosen is None:
        raise ValueError(f"No working codec found. Tried: {candidates}. Please install ffmpeg with necessary codecs.")
    if verbose:
        import logging

        logging.info(f"Using codec: {chosen}")
    try:
        stream.width, stream.height, stream.pix_fmt = width, height, "yuv420p"
        if chosen in ("libx264", "h264"):
            stream.options = {"crf": str(crf), "preset": preset}
        for i in range(n):
            vf = av.VideoFrame.from_ndarray(np.ascontiguousarray(frames[i]), format="rgb24")
            for packet in stream.encode(vf):
                container.mux(packet)
        for packet in stream.encode(None):  # flush the encoder
            container.mux(packet)
    finally:
        container.close()


def get_video_fps(video_path) -> float:
    """video_io.py:211-224 — reading the container needs PyAV (absent from this image)."""
    try:
        import av
    except ImportError as e:
        raise ImportError("get_video_fps needs PyAV, which is not installed in this image") from e
    container = av.open(video_path)  # pragma: no cover — PyAV absent here
    try:
        return float(container.streams.video[0].average_rate)
    finally:
        container.close()


def concatenate_videos_horizontally_torch(video1, video2, gap: int = 0, gap_color=None) -> torch.Tensor:
    """video_io.py:227-265: video2 resized (antialiased bilinear, rdmi_resize) to video1's [H1, W1] and
    concatenated to its right along the width.  As in the reference, the gap strip is built but the
    returned tensor is the concatenation WITHOUT it (:259-263 overwrite the gapped result), so `gap`
    and `gap_color` do not change the output.  [N, 3, H, W] numpy or torch, float or uint8; a host
    tensor is resized on the default device and returned on the host.  uint8 frames are resized in
    f32 and rounded half-to-even (torchvision's float path for uint8 tensors)."""
    if isinstance(video1, np.ndarray):
        video1 = torch.from_numpy(video1)
    if isinstance(video2, np.ndarray):
        video2 = torch.from_numpy(video2)
    N, C, H1, W1 = video1.shape
    dev = video2.device if video2.is_cuda else torch.device("cuda")
    r = K.resize(video2.to(dev), (H1, W1), "BILINEAR")
    if video2.dtype == torch.uint8:
        r = r.round_().clamp_(0, 255)
    r = r.to(video1.dtype)
    return torch.cat([video1, r.to(video1.device)], dim=3)
