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


# ----------------------------------------------------------------------------- config validation
# A diffusers config value the native models do not implement must raise, not run as if it were the
# SD2 value (a checkpoint with, e.g., resnet_time_scale_shift="scale_shift" would otherwise load and
# compute the wrong network).  Each entry: key → (diffusers default, accepted predicate, what runs).
def _one_or_all_ones(v) -> bool:
    return v == 1 or (isinstance(v, (list, tuple)) and all(_one_or_all_ones(x) for x in v))


def _falsy_all(v) -> bool:
    return not v if not isinstance(v, (list, tuple)) else not any(v)


# unet_2d_condition.py:171-225 (defaults as there)
_UNET_RULES = {
    "center_input_sample": (False, lambda v: not v, "center_input_sample=False"),
    "mid_block_type": ("UNetMidBlock2DCrossAttn", lambda v: v == "UNetMidBlock2DCrossAttn",
                       "a UNetMidBlock2DCrossAttn mid block"),
    "only_cross_attention": (False, _falsy_all, "only_cross_attention=False"),
    "downsample_padding": (1, lambda v: v == 1, "downsample_padding=1"),
    "mid_block_scale_factor": (1, lambda v: v == 1, "mid_block_scale_factor=1"),
    "act_fn": ("silu", lambda v: v == "silu", "act_fn='silu'"),
    "transformer_layers_per_block": (1, _one_or_all_ones, "one transformer block per Transformer2DModel"),
    "reverse_transformer_layers_per_block": (None, lambda v: v is None or _one_or_all_ones(v),
                                             "one transformer block per Transformer2DModel"),
    "encoder_hid_dim": (None, lambda v: v is None, "no encoder_hid_proj"),
    "encoder_hid_dim_type": (None, lambda v: v is None, "no encoder_hid_proj"),
    "dual_cross_attention": (False, lambda v: not v, "dual_cross_attention=False"),
    "class_embed_type": (None, lambda v: v is None, "no class embedding"),
    "addition_embed_type": (None, lambda v: v is None, "no addition embedding"),
    "num_class_embeds": (None, lambda v: v is None, "no class embedding"),
    "resnet_time_scale_shift": ("default", lambda v: v == "default", "resnet_time_scale_shift='default'"),
    "resnet_skip_time_act": (False, lambda v: not v, "resnet_skip_time_act=False"),
    "resnet_out_scale_factor": (1.0, lambda v: v == 1, "resnet_out_scale_factor=1"),
    "time_embedding_type": ("positional", lambda v: v == "positional", "positional time embedding"),
    "time_embedding_dim": (None, lambda v: v is None, "time_embedding_dim = 4·block_out_channels[0]"),
    "time_embedding_act_fn": (None, lambda v: v is None, "no time_embedding_act_fn"),
    "timestep_post_act": (None, lambda v: v is None, "no timestep_post_act"),
    "time_cond_proj_dim": (None, lambda v: v is None, "no time_cond_proj"),
    "conv_in_kernel": (3, lambda v: v == 3, "a 3×3 conv_in"),
    "conv_out_kernel": (3, lambda v: v == 3, "a 3×3 conv_out"),
    "attention_type": ("default", lambda v: v == "default", "attention_type='default'"),
    "class_embeddings_concat": (False, lambda v: not v, "class_embeddings_concat=False"),
    "mid_block_only_cross_attention": (None, lambda v: not v, "mid_block_only_cross_attention unset"),
    "cross_attention_norm": (None, lambda v: v is None, "no cross_attention_norm"),
}
_UNET_DOWN = {"CrossAttnDownBlock2D", "DownBlock2D"}
_UNET_UP = {"CrossAttnUpBlock2D", "UpBlock2D"}

# autoencoder_kl.py:75-95
_VAE_RULES = {
    "act_fn": ("silu", lambda v: v == "silu", "act_fn='silu'"),
    "use_quant_conv": (True, lambda v: bool(v), "use_quant_conv=True"),
    "use_post_quant_conv": (True, lambda v: bool(v), "use_post_quant_conv=True"),
    "mid_block_add_attention": (True, lambda v: bool(v), "the mid-block attention"),
}

# scheduling_ddim.py:148-190 (keys the η = 0 step of the pipeline depends on; clip_sample is checked
# by DDIMScheduler itself)
_SCHED_RULES = {
    "trained_betas": (None, lambda v: v is None, "betas from beta_schedule"),
    "thresholding": (False, lambda v: not v, "thresholding=False"),
}


def _check(kind: str, cfg: dict, rules: dict) -> None:
    for key, (default, ok, what) in rules.items():
        v = cfg.get(key, default)
        if not ok(v):
            raise NotImplementedError(f"{kind} config {key}={v!r}: the native {kind} implements {what} only")


def validate_unet_config(cfg: dict) -> None:
    """Raise for UNet2DConditionModel config values the native UNet does not implement; diffusers'
    own ValueError for num_attention_heads (unet_2d_condition.py:230-233).  use_linear_projection
    needs no check: proj_in / proj_out as 1×1 convs (the diffusers default, False) are the same
    per-pixel linear map and are loaded as such (unet._Lin)."""
    if cfg.get("num_attention_heads") is not None:
        raise ValueError("At the moment it is not possible to define the number of attention heads via "
                         "`num_attention_heads` (unet_2d_condition.py:230)")
    _check("UNet", cfg, _UNET_RULES)
    bad = [b for b in cfg.get("down_block_types", ()) if b not in _UNET_DOWN] + \
          [b for b in cfg.get("up_block_types", ()) if b not in _UNET_UP]
    if bad:
        raise NotImplementedError(f"UNet block types {bad}: the native UNet implements {sorted(_UNET_DOWN | _UNET_UP)}")
    if not isinstance(cfg.get("layers_per_block", 2), int):
        raise NotImplementedError(f"UNet layers_per_block={cfg['layers_per_block']!r}: one count for every block")
    if isinstance(cfg.get("cross_attention_dim", 1280), (list, tuple)):
        raise NotImplementedError("UNet cross_attention_dim per block: one context width for every block")


def validate_vae_config(cfg: dict) -> None:
    """Raise for AutoencoderKL config values the native VAE does not implement."""
    _check("VAE", cfg, _VAE_RULES)
    bad = [b for b in cfg.get("down_block_types", ()) if b != "DownEncoderBlock2D"] + \
          [b for b in cfg.get("up_block_types", ()) if b != "UpDecoderBlock2D"]
    if bad:
        raise NotImplementedError(f"VAE block types {bad}: the native VAE implements DownEncoderBlock2D / "
                                  "UpDecoderBlock2D")


def validate_scheduler_config(cfg: dict) -> None:
    """Raise for DDIMScheduler config values the device step does not implement."""
    _check("DDIMScheduler", cfg, _SCHED_RULES)
