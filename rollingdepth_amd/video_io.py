"""Video ingest (rollingdepth/video_io.py:71-137) — needs PyAV, which is not installed in this image.
Kept as an explicit, loud boundary: the pipeline accepts frame tensors directly."""


def load_video_frames(input_path, start_frame=0, frame_count=0, processing_res=0, resample_method="BILINEAR",
                      verbose=False):
    try:
        import av  # noqa: F401
    except ImportError as e:
        raise ImportError("video decoding needs PyAV (absent); pass a [N,3,H,W] tensor in [-1,1] instead") from e
    raise NotImplementedError("video ingest is SURVEY.md §8f rank 3 (next rounds)")
