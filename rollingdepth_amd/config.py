"""Model / scheduler configurations (diffusers `config.json` key names).

The real rollingdepth-v1-0 checkpoint is not in this image (SURVEY.md §8 preamble;
script/download_weight.sh:9-15 fetches it), so the SD2-shaped configs below restate the
architecture the reference loads: UNet2DConditionModel with an 8-channel conv_in (rgb latent +
depth latent, rollingdepth_pipeline.py:650-651) and SD2 KL-f8 AutoencoderKL.  `from_pretrained`
in pipeline.py reads the checkpoint's own JSON files when a checkpoint directory is given.
"""
from __future__ import annotations

import copy

SD2_UNET = {
    "in_channels": 8,
    "out_channels": 4,
    "block_out_channels": [320, 640, 1280, 1280],
    "layers_per_block": 2,
    "attention_head_dim": [5, 10, 20, 20],  # diffusers SD2 quirk: these are head COUNTS (d=64)
    "cross_attention_dim": 1024,
    "norm_num_groups": 32,
    "norm_eps": 1e-5,
    "down_block_types": ["CrossAttnDownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D", "DownBlock2D"],
    "up_block_types": ["UpBlock2D", "CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "CrossAttnUpBlock2D"],
    "flip_sin_to_cos": True,
    "freq_shift": 0,
    "use_linear_projection": True,
    "upcast_attention": False,
    "sample_size": 96,
}

SD2_VAE = {
    "in_channels": 3,
    "out_channels": 3,
    "block_out_channels": [128, 256, 512, 512],
    "layers_per_block": 2,
    "latent_channels": 4,
    "norm_num_groups": 32,
    "down_block_types": ["DownEncoderBlock2D"] * 4,
    "up_block_types": ["UpDecoderBlock2D"] * 4,
    "act_fn": "silu",
    "sample_size": 768,
    "scaling_factor": 0.18215,
}

# DDIM config of the RollingDepth checkpoint family (v-prediction, trailing spacing).
RD_SCHEDULER = {
    "num_train_timesteps": 1000,
    "beta_start": 0.00085,
    "beta_end": 0.012,
    "beta_schedule": "scaled_linear",
    "clip_sample": False,
    "set_alpha_to_one": False,
    "steps_offset": 1,
    "prediction_type": "v_prediction",
    "timestep_spacing": "trailing",
    "rescale_betas_zero_snr": False,
}

# Tiny configs for fast fixture-pinned parity runs (same block types, head_dim 64).
TINY_UNET = dict(copy.deepcopy(SD2_UNET), block_out_channels=[64, 128], attention_head_dim=[1, 2],
                 cross_attention_dim=96,
                 down_block_types=["CrossAttnDownBlock2D", "DownBlock2D"],
                 up_block_types=["UpBlock2D", "CrossAttnUpBlock2D"], sample_size=16)
TINY_VAE = dict(copy.deepcopy(SD2_VAE), block_out_channels=[32, 64], layers_per_block=1,
                down_block_types=["DownEncoderBlock2D"] * 2, up_block_types=["UpDecoderBlock2D"] * 2,
                sample_size=32)


def unet_heads(cfg) -> list:
    nh = cfg.get("num_attention_heads") or cfg["attention_head_dim"]
    n = len(cfg["block_out_channels"])
    return list(nh) if isinstance(nh, (list, tuple)) else [nh] * n


def vae_downscale(cfg) -> int:
    return 2 ** (len(cfg["block_out_channels"]) - 1)
