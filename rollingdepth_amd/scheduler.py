"""DDIMScheduler surface used by the depth pipeline (diffusers/schedulers/scheduling_ddim.py).

The α-bar table and the timestep schedule are host-side constants (as in the reference, :180-230,
:297-340); `step` with η = 0 is an affine map of (sample, model_output) whose two coefficients
are computed here in f64 and applied on the device by rdmi_ddim_combine (optionally fused with
the 1/0.18215 latent scale the decoder input needs, rollingdepth_pipeline.py:716).
"""
from __future__ import annotations

import math
from typing import List, Tuple

import numpy as np
import torch

from . import kernels as K
from .config import validate_scheduler_config


class DDIMScheduler:
    def __init__(self, num_train_timesteps: int = 1000, beta_start: float = 0.0001, beta_end: float = 0.02,
                 beta_schedule: str = "linear", set_alpha_to_one: bool = True, steps_offset: int = 0,
                 prediction_type: str = "epsilon", timestep_spacing: str = "leading",
                 rescale_betas_zero_snr: bool = False, clip_sample: bool = False, **unused):
        validate_scheduler_config(unused)
        if clip_sample:
            raise NotImplementedError("clip_sample=True is not used by the RollingDepth checkpoints")
        self.config = dict(num_train_timesteps=num_train_timesteps, beta_start=beta_start, beta_end=beta_end,
                           beta_schedule=beta_schedule, set_alpha_to_one=set_alpha_to_one,
                           steps_offset=steps_offset, prediction_type=prediction_type,
                           timestep_spacing=timestep_spacing, rescale_betas_zero_snr=rescale_betas_zero_snr)
        T = num_train_timesteps
        if beta_schedule == "scaled_linear":
            betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, T, dtype=torch.float32) ** 2
        elif beta_schedule == "linear":
            betas = torch.linspace(beta_start, beta_end, T, dtype=torch.float32)
        else:
            raise NotImplementedError(beta_schedule)
        if rescale_betas_zero_snr:
            a = torch.cumprod(1.0 - betas, 0).sqrt()
            a0, aT = a[0].clone(), a[-1].clone()
            a = (a - aT) * (a0 / (a0 - aT))
            ab = a ** 2
            betas = 1 - torch.cat([ab[0:1], ab[1:] / ab[:-1]])
        self.alphas_cumprod = torch.cumprod(1.0 - betas, dim=0)
        self.final_alpha_cumprod = torch.tensor(1.0) if set_alpha_to_one else self.alphas_cumprod[0]
        self.num_inference_steps = None
        self.timesteps = torch.tensor([], dtype=torch.int64)

    @classmethod
    def from_config(cls, cfg: dict) -> "DDIMScheduler":
        return cls(**{k: v for k, v in cfg.items() if not k.startswith("_")})

    def set_timesteps(self, num_inference_steps: int, device=None) -> None:
        T = self.config["num_train_timesteps"]
        if num_inference_steps > T:
            raise ValueError(f"num_inference_steps {num_inference_steps} > num_train_timesteps {T}")
        self.num_inference_steps = num_inference_steps
        sp = self.config["timestep_spacing"]
        if sp == "linspace":
            ts = np.linspace(0, T - 1, num_inference_steps).round()[::-1].copy().astype(np.int64)
        elif sp == "leading":
            r = T // num_inference_steps
            ts = (np.arange(0, num_inference_steps) * r).round()[::-1].copy().astype(np.int64)
            ts += self.config["steps_offset"]
        elif sp == "trailing":
            r = T / num_inference_steps
            ts = np.round(np.arange(T, 0, -r)).astype(np.int64) - 1
        else:
            raise ValueError(sp)
        self.timesteps = torch.from_numpy(ts)

    def step_coefficients(self, t: int) -> Tuple[float, float]:
        """prev_sample = ca·sample + cb·model_output for η = 0 (scheduling_ddim.py:399-448)."""
        prev = t - self.config["num_train_timesteps"] // self.num_inference_steps
        a = float(self.alphas_cumprod[t])
        ap = float(self.alphas_cumprod[prev]) if prev >= 0 else float(self.final_alpha_cumprod)
        b = 1.0 - a
        sa, sb, sap, sbp = math.sqrt(a), math.sqrt(b), math.sqrt(ap), math.sqrt(1.0 - ap)
        pt = self.config["prediction_type"]
        if pt == "v_prediction":
            return sap * sa + sbp * sb, sbp * sa - sap * sb
        if pt == "epsilon":
            return sap / sa, sbp - sap * sb / sa
        if pt == "sample":
            return sbp / sb, sap - sbp * sa / sb
        raise ValueError(pt)

    def step_(self, model_output: torch.Tensor, t: int, sample: torch.Tensor, out_scale: float = 1.0,
              out: torch.Tensor = None, channels: int = 4) -> torch.Tensor:
        """Device step on NHWC latents: out[..., :channels] = (ca·sample + cb·model_output)·out_scale."""
        ca, cb = self.step_coefficients(int(t))
        cpad = out.shape[-1] if out is not None else sample.shape[-1]
        return K.ddim_combine(sample, model_output, ca, cb, out_scale, channels, cpad, out=out)

    def add_noise_coefficients(self, t: int) -> Tuple[float, float]:
        a = float(self.alphas_cumprod[int(t)])
        return math.sqrt(a), math.sqrt(1.0 - a)
