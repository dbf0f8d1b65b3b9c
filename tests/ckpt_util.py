"""Write a diffusers-format RollingDepth checkpoint directory from synthesised weights — the layout
`RollingDepthPipeline.from_pretrained` reads (diffusers/pipelines/pipeline_utils.py:480;
model_index.json, unet/, vae/, scheduler/, text_encoder/, tokenizer/), so tests can replay
run_video.py's load sequence without network access or the real checkpoint."""
import json
import os

from safetensors.torch import save_file

from rollingdepth_amd import text_encoder as TE
from rollingdepth_amd import weights as W


def write_text_encoder(root: str, te_cfg: dict, vocab: dict, seed: int = 0):
    te = os.path.join(root, "text_encoder")
    tok = os.path.join(root, "tokenizer")
    os.makedirs(te, exist_ok=True)
    os.makedirs(tok, exist_ok=True)
    json.dump({"architectures": ["CLIPTextModel"], "model_type": "clip_text_model", **te_cfg},
              open(os.path.join(te, "config.json"), "w"))
    sd = W.synth_state_dict(TE.text_encoder_param_shapes(te_cfg), seed)
    save_file({k: v.contiguous() for k, v in sd.items()}, os.path.join(te, "model.safetensors"))
    json.dump(vocab, open(os.path.join(tok, "vocab.json"), "w"))
    open(os.path.join(tok, "merges.txt"), "w").write("#version: 0.2\n")
    json.dump({"bos_token": "<|startoftext|>", "eos_token": "<|endoftext|>", "unk_token": "<|endoftext|>",
               "model_max_length": 77, "tokenizer_class": "CLIPTokenizer"},
              open(os.path.join(tok, "tokenizer_config.json"), "w"))


def write_checkpoint(root: str, unet_cfg: dict, vae_cfg: dict, sched_cfg: dict, te_cfg: dict, vocab: dict,
                     seed: int = 0):
    os.makedirs(root, exist_ok=True)
    json.dump({"_class_name": "RollingDepthPipeline", "_diffusers_version": "0.30.0",
               "unet": ["diffusers", "UNet2DConditionModel"], "vae": ["diffusers", "AutoencoderKL"],
               "scheduler": ["diffusers", "DDIMScheduler"], "text_encoder": ["transformers", "CLIPTextModel"],
               "tokenizer": ["transformers", "CLIPTokenizer"]}, open(os.path.join(root, "model_index.json"), "w"))
    for sub, cfg, shapes in (("unet", unet_cfg, W.unet_param_shapes(unet_cfg)),
                             ("vae", vae_cfg, W.vae_param_shapes(vae_cfg))):
        d = os.path.join(root, sub)
        os.makedirs(d, exist_ok=True)
        json.dump(cfg, open(os.path.join(d, "config.json"), "w"))
        sd = W.synth_state_dict(shapes, seed)
        save_file({k: v.contiguous() for k, v in sd.items()}, os.path.join(d, "diffusion_pytorch_model.safetensors"))
    os.makedirs(os.path.join(root, "scheduler"), exist_ok=True)
    json.dump({"_class_name": "DDIMScheduler", **sched_cfg},
              open(os.path.join(root, "scheduler", "scheduler_config.json"), "w"))
    write_text_encoder(root, te_cfg, vocab, seed)
