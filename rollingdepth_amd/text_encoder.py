"""Empty-prompt text embedding from a diffusers checkpoint's text_encoder/ + tokenizer/ folders —
RollingDepthPipeline.encode_empty_text (rollingdepth_pipeline.py:178-191) without the transformers
stack: `tokenizer("", padding="do_not_pad", truncation=True)` is exactly [BOS, EOS], and
`CLIPTextModel(ids)[0]` (transformers CLIPTextTransformer: token + position embedding, pre-LN
encoder layers with causal self-attention and an MLP, final LayerNorm) is restated below for those
two tokens.

The embedding is a constant of the checkpoint (every UNet cross-attention reads it, and
unet.Transformer folds it into the attn2 weights once), so it is computed once at load time, like
weight packing: in f64 on the host from the checkpoint's f32 weights, then cast to the pipeline
dtype (the reference casts the text encoder output with `.to(self.dtype)`).  Only the two token
rows of the embedding table are read.  Pinned by tests/test_host_cpu.py against
transformers.CLIPTextModel, and end to end by the tiny_clip_pipeline reference fixture.
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, List, Tuple

import torch

_ACTS = {
    "gelu": lambda x: torch.nn.functional.gelu(x),
    "quick_gelu": lambda x: x * torch.sigmoid(1.702 * x),
    "gelu_new": lambda x: torch.nn.functional.gelu(x, approximate="tanh"),
    "relu": torch.relu,
}


def special_token_ids(tok_dir: str) -> Tuple[int, int]:
    """(BOS, EOS) ids of a CLIP tokenizer folder (vocab.json + tokenizer_config.json /
    special_tokens_map.json) — what tokenizing "" without padding returns."""
    vocab = json.load(open(os.path.join(tok_dir, "vocab.json"), encoding="utf-8"))
    names = {"bos_token": "<|startoftext|>", "eos_token": "<|endoftext|>"}
    for fn in ("special_tokens_map.json", "tokenizer_config.json"):
        p = os.path.join(tok_dir, fn)
        if os.path.exists(p):
            cfg = json.load(open(p, encoding="utf-8"))
            for k in names:
                v = cfg.get(k)
                if isinstance(v, dict):
                    v = v.get("content")
                if isinstance(v, str):
                    names[k] = v
    return int(vocab[names["bos_token"]]), int(vocab[names["eos_token"]])


def _open_weights(te_dir: str):
    """A key → tensor getter over the text encoder's weights (safetensors, lazily per key; or a
    torch .bin loaded with weights_only=True)."""
    st = os.path.join(te_dir, "model.safetensors")
    if os.path.exists(st):
        from safetensors import safe_open

        f = safe_open(st, framework="pt")
        keys = set(f.keys())

        def get(k, rows=None):
            if rows is not None:
                sl = f.get_slice(k)
                return torch.stack([sl[r] for r in rows])
            return f.get_tensor(k)

        return get, keys
    b = os.path.join(te_dir, "pytorch_model.bin")
    sd = torch.load(b, map_location="cpu", weights_only=True)
    return (lambda k, rows=None: sd[k][list(rows)] if rows is not None else sd[k]), set(sd)


def clip_text_forward(get, cfg: dict, ids: List[int], prefix: str = "text_model.") -> torch.Tensor:
    """CLIPTextTransformer forward (last_hidden_state) for one short token sequence, f64.
    `get(key, rows=None)` returns checkpoint tensors; `prefix` is the checkpoint's key prefix
    ("text_model." in transformers-4 checkpoints such as SD2's, "" in transformers-5 saves)."""
    d = int(cfg["hidden_size"])
    nh = int(cfg["num_attention_heads"])
    nl = int(cfg["num_hidden_layers"])
    eps = float(cfg.get("layer_norm_eps", 1e-5))
    act = _ACTS[cfg.get("hidden_act", "quick_gelu")]
    hd = d // nh
    L = len(ids)
    P = prefix
    g = lambda k: get(P + k).double()  # noqa: E731
    h = get(P + "embeddings.token_embedding.weight", rows=ids).double() + \
        get(P + "embeddings.position_embedding.weight", rows=range(L)).double()
    causal = torch.full((L, L), float("-inf"), dtype=torch.float64).triu(1)

    def ln(x, k):
        return torch.nn.functional.layer_norm(x, (d,), g(k + ".weight"), g(k + ".bias"), eps)

    def lin(x, k):
        return x @ g(k + ".weight").t() + g(k + ".bias")

    for i in range(nl):
        p = f"encoder.layers.{i}."
        r = h
        x = ln(h, p + "layer_norm1")
        q = lin(x, p + "self_attn.q_proj").view(L, nh, hd).transpose(0, 1)
        k = lin(x, p + "self_attn.k_proj").view(L, nh, hd).transpose(0, 1)
        v = lin(x, p + "self_attn.v_proj").view(L, nh, hd).transpose(0, 1)
        a = torch.softmax(q @ k.transpose(1, 2) / math.sqrt(hd) + causal, dim=-1) @ v
        h = r + lin(a.transpose(0, 1).reshape(L, d), p + "self_attn.out_proj")
        r = h
        x = ln(h, p + "layer_norm2")
        h = r + lin(act(lin(x, p + "mlp.fc1")), p + "mlp.fc2")
    return ln(h, "final_layer_norm")


def empty_text_embedding(ckpt_dir: str, dtype=torch.float32) -> torch.Tensor:
    """[1, 2, hidden] — encode_empty_text of the checkpoint at ckpt_dir (text_encoder/, tokenizer/)."""
    te = os.path.join(ckpt_dir, "text_encoder")
    tok = os.path.join(ckpt_dir, "tokenizer")
    cfg = json.load(open(os.path.join(te, "config.json")))
    if cfg.get("text_config"):  # a full CLIPModel config: the text tower's part
        cfg = cfg["text_config"]
    bos, eos = special_token_ids(tok)
    get, keys = _open_weights(te)
    prefix = "text_model." if "text_model.final_layer_norm.weight" in keys else ""
    out = clip_text_forward(get, cfg, [bos, eos], prefix)
    return out[None].to(dtype)


def text_encoder_param_shapes(cfg: dict) -> Dict[str, tuple]:
    """Key → shape of transformers' CLIPTextModel state dict (for synthesised test checkpoints)."""
    d, ff, nl = int(cfg["hidden_size"]), int(cfg["intermediate_size"]), int(cfg["num_hidden_layers"])
    P = "text_model."
    s = {P + "embeddings.token_embedding.weight": (int(cfg["vocab_size"]), d),
         P + "embeddings.position_embedding.weight": (int(cfg["max_position_embeddings"]), d)}
    for i in range(nl):
        p = f"{P}encoder.layers.{i}."
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            s[p + f"self_attn.{n}.weight"] = (d, d)
            s[p + f"self_attn.{n}.bias"] = (d,)
        s[p + "layer_norm1.weight"] = s[p + "layer_norm1.bias"] = (d,)
        s[p + "mlp.fc1.weight"] = (ff, d)
        s[p + "mlp.fc1.bias"] = (ff,)
        s[p + "mlp.fc2.weight"] = (d, ff)
        s[p + "mlp.fc2.bias"] = (d,)
        s[p + "layer_norm2.weight"] = s[p + "layer_norm2.bias"] = (d,)
    s[P + "final_layer_norm.weight"] = s[P + "final_layer_norm.bias"] = (d,)
    return s
