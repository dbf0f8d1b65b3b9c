"""Depth colourisation — src/util/colorize.py:12-93 (`colorize_depth`, `colorize_depth_multi_thread`)
with the per-pixel work on the device (rdmi_colorize: one HBM pass, 2-4 B in / 3 B out per pixel).

The colormap table is a host constant built once per name from matplotlib (the reference's own
colormap source); the index arithmetic in the kernel follows matplotlib's Colormap.__call__ for
floats, evaluated in the depth's dtype as numpy evaluates the reference's normalisation.  The 8-bit
output is (table · 255).astype(uint8) of that entry — the bytes the reference's
`(chunk * 255).astype(np.uint8)` produces."""
from __future__ import annotations

from typing import Dict, Optional, Union

import numpy as np
import torch

from . import kernels as K
from ._native import check, lib

_LUTS: Dict[tuple, tuple] = {}


def _cmap(name: str):
    import matplotlib

    cm = matplotlib.colormaps[name]
    if not cm._isinit:
        cm._init()
    return cm


def _lut_u8(name: str, device):
    key = (name, str(device))
    if key not in _LUTS:
        cm = _cmap(name)
        lut = (cm._lut[:, :3] * 255).astype(np.uint8)  # N entries + under, over, bad
        _LUTS[key] = (torch.from_numpy(np.ascontiguousarray(lut)).to(device), cm.N)
    return _LUTS[key]


def _np_dtype(d: torch.Tensor):
    return np.float16 if d.dtype == torch.float16 else np.float32


def _launch(d: torch.Tensor, mn_rng, name: str, index: bool) -> torch.Tensor:
    """mn_rng: (min, max − min) as numpy scalars of the depth's dtype."""
    lut, n = _lut_u8(name, d.device)
    d = d.contiguous()
    mmd = torch.from_numpy(np.array(mn_rng, dtype=_np_dtype(d))).to(d.device)
    if index:
        out = torch.empty(d.shape, dtype=torch.int32, device=d.device)
        rc = lib.rdmi_colorize(d.data_ptr(), K._dtype_code(d), d.numel(), mmd.data_ptr(), None, n, None,
                               out.data_ptr(), K._stream())
    else:
        out = torch.empty((*d.shape, 3), dtype=torch.uint8, device=d.device)
        rc = lib.rdmi_colorize(d.data_ptr(), K._dtype_code(d), d.numel(), mmd.data_ptr(), lut.data_ptr(), n,
                               out.data_ptr(), None, K._stream())
    check(rc, "rdmi_colorize")
    return out


def _as_device(depth, device) -> torch.Tensor:
    """The device path evaluates the reference's index arithmetic in the depth's own dtype, f16 or
    f32 (what the pipeline outputs).  Other dtypes are rejected rather than converted: the reference
    computes (d − min) / (max − min) in float64 for float64 input, and an f32 evaluation could pick a
    different colormap entry at a bin edge."""
    if isinstance(depth, np.ndarray):
        depth = torch.from_numpy(np.ascontiguousarray(depth))
    if depth.dtype not in (torch.float16, torch.float32):
        raise TypeError(f"colorize: depth dtype {depth.dtype} unsupported (float16 / float32; convert explicitly)")
    return depth.to(device)


def colorize_depth(depth: Union[np.ndarray, torch.Tensor], min_depth: float, max_depth: float,
                   cmap: str = "Spectral_r", valid_mask=None, device="cuda") -> np.ndarray:
    """colorize.py:12-38 → float64 RGB [B, H, W, 3] in [0, 1] (the colormap table entry of every pixel).
    The reference's valid_mask branch indexes the [B, H, W, 3] image with a [B, 3, H, W] mask and
    raises; masks enter only through colorize_depth_multi_thread's min / max, as the reference uses
    them."""
    if valid_mask is not None:
        raise NotImplementedError("colorize_depth: valid_mask (see docstring)")
    d = _as_device(depth, device)
    if d.dim() < 3:
        d = d[None]
    # Python-float bounds: their difference is a Python float, rounded to the depth dtype by numpy
    nt = _np_dtype(d)
    idx = _launch(d, (nt(min_depth), nt(max_depth - min_depth)), cmap, index=True).cpu().numpy()
    return _cmap(cmap)._lut[idx][..., :3]


def colorize_depth_multi_thread(depth: Union[np.ndarray, torch.Tensor], valid_mask: Optional[np.ndarray] = None,
                                chunk_size: int = 4, num_threads: int = 4, color_map: str = "Spectral",
                                verbose: bool = False, device="cuda") -> np.ndarray:
    """colorize.py:41-93: depth [N, 1, H, W] → uint8 [N, H, W, 3], normalised by the min / max over the
    valid pixels (all pixels without a mask).  chunk_size / num_threads / verbose are accepted for the
    reference's signature; the whole video is one device launch."""
    d = _as_device(depth, device).squeeze(1)
    assert d.dim() == 3
    nt = _np_dtype(d)
    if valid_mask is None:
        mn, mx = (nt(v) for v in K.minmax(d).tolist())  # exact: min / max are values of the depth dtype
    else:  # the reference reduces the masked pixels with numpy on the host (colorize.py:54-59)
        v = d.cpu().numpy()[np.asarray(valid_mask).reshape(d.shape).astype(bool)]
        mn, mx = v.min(), v.max()
    return _launch(d, (mn, mx - mn), color_map, index=False).cpu().numpy()
