"""Checkpoint configs are validated at load: a diffusers config value the native
UNet / VAE / DDIM scheduler does not implement raises NotImplementedError in the constructor, before
any weight is read, instead of running the SD2 network under another checkpoint's name.  Reference:
unet_2d_condition.py:171-233, autoencoder_kl.py:75-95, scheduling_ddim.py:148-190."""
import copy

import pytest
import torch

from rollingdepth_amd import config as C

UNET_REJECT = [
    ("center_input_sample", True),
    ("transformer_layers_per_block", 2),
    ("transformer_layers_per_block", [1, 2, 1, 1]),
    ("reverse_transformer_layers_per_block", [[2], [1]]),
    ("resnet_time_scale_shift", "scale_shift"),
    ("only_cross_attention", True),
    ("only_cross_attention", [False, True, False, False]),
    ("class_embed_type", "timestep"),
    ("num_class_embeds", 10),
    ("addition_embed_type", "text_time"),
    ("encoder_hid_dim", 1024),
    ("encoder_hid_dim_type", "text_proj"),
    ("conv_in_kernel", 1),
    ("conv_out_kernel", 1),
    ("mid_block_type", "UNetMidBlock2DSimpleCrossAttn"),
    ("mid_block_type", None),
    ("dual_cross_attention", True),
    ("resnet_skip_time_act", True),
    ("resnet_out_scale_factor", 2.0),
    ("time_embedding_type", "fourier"),
    ("time_embedding_act_fn", "silu"),
    ("timestep_post_act", "silu"),
    ("time_cond_proj_dim", 256),
    ("downsample_padding", 0),
    ("mid_block_scale_factor", 2.0),
    ("act_fn", "gelu"),
    ("attention_type", "gated"),
    ("cross_attention_norm", "layer_norm"),
    ("layers_per_block", [2, 2, 2, 2]),
    ("cross_attention_dim", [1024, 1024, 1024, 1024]),
    ("down_block_types", ["CrossAttnDownBlock2D", "SimpleCrossAttnDownBlock2D"]),
    ("up_block_types", ["UpBlock2D", "AttnUpBlock2D"]),
]


@pytest.mark.parametrize("key,value", UNET_REJECT, ids=[f"{k}={v}" for k, v in UNET_REJECT])
def test_unet_rejects_unimplemented_config(key, value):
    from rollingdepth_amd.unet import UNet

    cfg = copy.deepcopy(C.SD2_UNET)
    cfg[key] = value
    with pytest.raises(NotImplementedError, match=key.split("_")[0] if "block_types" not in key else "block types"):
        UNet(cfg, {}, "cpu")


def test_unet_num_attention_heads_is_diffusers_value_error():
    from rollingdepth_amd.unet import UNet

    cfg = dict(C.SD2_UNET, num_attention_heads=[5, 10, 20, 20])
    with pytest.raises(ValueError, match="num_attention_heads"):
        UNet(cfg, {}, "cpu")


def test_unet_accepts_the_sd2_config_and_explicit_defaults():
    cfg = dict(C.SD2_UNET, center_input_sample=False, transformer_layers_per_block=[1, 1, 1, 1],
               resnet_time_scale_shift="default", only_cross_attention=[False] * 4, conv_in_kernel=3,
               mid_block_type="UNetMidBlock2DCrossAttn", class_embed_type=None, addition_embed_type=None,
               use_linear_projection=False, upcast_attention=True, _class_name="UNet2DConditionModel")
    C.validate_unet_config(cfg)
    C.validate_unet_config(C.SD2_UNET)
    C.validate_unet_config(C.TINY_UNET)


VAE_REJECT = [("mid_block_add_attention", False), ("use_quant_conv", False), ("use_post_quant_conv", False),
              ("act_fn", "relu"), ("down_block_types", ["DownEncoderBlock2D", "AttnDownEncoderBlock2D"]),
              ("up_block_types", ["AttnUpDecoderBlock2D"])]


@pytest.mark.parametrize("key,value", VAE_REJECT, ids=[f"{k}={v}" for k, v in VAE_REJECT])
def test_vae_rejects_unimplemented_config(key, value):
    from rollingdepth_amd.vae import VAE

    cfg = dict(C.SD2_VAE, **{key: value})
    with pytest.raises(NotImplementedError):
        VAE(cfg, {}, "cpu")
    C.validate_vae_config(dict(C.SD2_VAE, shift_factor=None, force_upcast=True, mid_block_add_attention=True))


@pytest.mark.parametrize("key,value", [("thresholding", True), ("trained_betas", [0.1] * 1000),
                                       ("clip_sample", True), ("beta_schedule", "squaredcos_cap_v2")])
def test_scheduler_rejects_unimplemented_config(key, value):
    from rollingdepth_amd.scheduler import DDIMScheduler

    with pytest.raises(NotImplementedError):
        DDIMScheduler.from_config(dict(C.RD_SCHEDULER, **{key: value}))
    DDIMScheduler.from_config(dict(C.RD_SCHEDULER, thresholding=False, trained_betas=None, clip_sample_range=1.0,
                                   _diffusers_version="0.25.0"))


def test_linear_projection_false_loads_1x1_conv_weights():
    """use_linear_projection=False (the diffusers default): proj_in / proj_out are [C, C, 1, 1] convs,
    loaded as the same per-pixel linear map."""
    from rollingdepth_amd import kernels as K
    from rollingdepth_amd.unet import _Lin

    w = torch.randn(64, 64, 1, 1)
    sd = {"p.weight": w, "p.bias": torch.randn(64)}
    lin = _Lin(sd, "p", "cpu")
    assert (lin.n, lin.k) == (64, 64)
    assert torch.equal(lin.w, K.pack_linear(w[:, :, 0, 0], "cpu"))
