"""Weight sources: random init (default; the GPU box has no network) or HF safetensors on disk.

SURVEY.md §5.4: "The weight loader reads safetensors from HF_HOME/PVC when present. Otherwise it
random-initialises from a built-in config registry with a deterministic seed."  The reference mounts
the HF cache PVC at `/home/dynamo/.cache/huggingface` with `HF_HOME` (disagg_cache.yaml:29-34).
"""
from __future__ import annotations

import glob
import os
from typing import Optional

import torch

from .config import ModelConfig, find_local_model_dir


def random_full_state(cfg: ModelConfig, seed: int = 0, std: float = 0.02,
                      dtype: torch.dtype = torch.float32) -> dict[str, torch.Tensor]:
    """Unsharded random weights on the host in our naming (small models / tests only)."""
    g = torch.Generator().manual_seed(seed)
    H, D, I = cfg.hidden_size, cfg.head_dim, cfg.intermediate_size

    def rnd(*shape):
        return (torch.randn(*shape, generator=g) * std).to(dtype)

    def norm(n):
        return (1.0 + 0.1 * torch.randn(n, generator=g)).to(dtype)

    sd = {"embed": rnd(cfg.vocab_size, H), "norm": norm(H)}
    if not cfg.tie_word_embeddings:
        sd["lm_head"] = rnd(cfg.vocab_size, H)
    for i in range(cfg.num_layers):
        p = f"l{i}."
        sd[p + "in_norm"] = norm(H)
        sd[p + "post_norm"] = norm(H)
        sd[p + "qkv"] = rnd((cfg.num_heads + 2 * cfg.num_kv_heads) * D, H)
        sd[p + "o"] = rnd(H, cfg.num_heads * D)
        if cfg.qk_norm:
            sd[p + "q_norm"] = norm(D)
            sd[p + "k_norm"] = norm(D)
        if cfg.is_moe:
            sd[p + "gate"] = rnd(cfg.num_experts, H) * 10
            sd[p + "w13"] = rnd(cfg.num_experts, 2 * I, H)
            sd[p + "w2"] = rnd(cfg.num_experts, H, I)
        else:
            sd[p + "gate_up"] = rnd(2 * I, H)
            sd[p + "down"] = rnd(H, I)
    return sd


def hf_to_internal(cfg: ModelConfig, hf: dict[str, torch.Tensor]) -> dict[str, torch.Tensor]:
    """Map HF checkpoint names (Llama/Qwen3/Mixtral) to our fused layout."""
    sd = {"embed": hf["model.embed_tokens.weight"], "norm": hf["model.norm.weight"]}
    if "lm_head.weight" in hf and not cfg.tie_word_embeddings:
        sd["lm_head"] = hf["lm_head.weight"]
    for i in range(cfg.num_layers):
        a, p = f"model.layers.{i}.", f"l{i}."
        sd[p + "in_norm"] = hf[a + "input_layernorm.weight"]
        sd[p + "post_norm"] = hf[a + "post_attention_layernorm.weight"]
        sd[p + "qkv"] = torch.cat([hf[a + f"self_attn.{n}_proj.weight"] for n in "qkv"])
        sd[p + "o"] = hf[a + "self_attn.o_proj.weight"]
        if cfg.qk_norm:
            sd[p + "q_norm"] = hf[a + "self_attn.q_norm.weight"]
            sd[p + "k_norm"] = hf[a + "self_attn.k_norm.weight"]
        if cfg.is_moe:
            m = a + "block_sparse_moe."
            sd[p + "gate"] = hf[m + "gate.weight"]
            sd[p + "w13"] = torch.stack([torch.cat([hf[m + f"experts.{e}.w1.weight"],
                                                    hf[m + f"experts.{e}.w3.weight"]])
                                         for e in range(cfg.num_experts)])
            sd[p + "w2"] = torch.stack([hf[m + f"experts.{e}.w2.weight"] for e in range(cfg.num_experts)])
        else:
            sd[p + "gate_up"] = torch.cat([hf[a + "mlp.gate_proj.weight"], hf[a + "mlp.up_proj.weight"]])
            sd[p + "down"] = hf[a + "mlp.down_proj.weight"]
    return sd


def load_safetensors_state(cfg: ModelConfig, model_dir: Optional[str] = None) -> Optional[dict]:
    model_dir = model_dir or find_local_model_dir(cfg.name)
    if model_dir is None:
        return None
    files = sorted(glob.glob(os.path.join(model_dir, "*.safetensors")))
    if not files:
        return None
    from safetensors.torch import load_file
    hf = {}
    for f in files:
        hf.update(load_file(f))
    return hf_to_internal(cfg, hf)


def load_weights(model, load_format: str = "auto", seed: int = 0) -> str:
    """Populate `model` (TransformerLM).  Returns the source used: 'safetensors' | 'random'."""
    if load_format == "random_full":  # unsharded host init, then shard: identical model for any TP size
        model.load_full_state(random_full_state(model.cfg, seed=seed, std=0.05, dtype=torch.float32))
        return "random_full"
    if load_format in ("auto", "safetensors"):
        sd = load_safetensors_state(model.cfg)
        if sd is not None:
            model.load_full_state(sd)
            return "safetensors"
        if load_format == "safetensors":
            raise FileNotFoundError(f"no safetensors for {model.cfg.name}")
    model.init_random(seed=seed)
    return "random"
