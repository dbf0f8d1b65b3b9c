"""rollingdepth_amd — RollingDepth's snippet-denoise hot path on AMD MI355X (gfx950).

Public surface mirrors the reference: RollingDepthPipeline / RollingDepthOutput
(rollingdepth/rollingdepth_pipeline.py), DepthAligner (rollingdepth/depth_aligner.py) and the
modified diffusers attention processor (CrossFrameAttnProcessor).  All arithmetic runs in
librdmi.so (HIP); importing the compute modules without the built library raises.
"""
__version__ = "0.1.0"


def __getattr__(name):
    if name in ("RollingDepthPipeline", "RollingDepthOutput"):
        from . import pipeline
        return getattr(pipeline, name)
    if name == "DepthAligner":
        from .aligner import DepthAligner
        return DepthAligner
    if name == "CrossFrameAttnProcessor":
        from .attention_processor import CrossFrameAttnProcessor
        return CrossFrameAttnProcessor
    raise AttributeError(name)
