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
                      dtype: torch.dtype = torch.float32, device="cpu") -> dict[str, torch.Tensor]:
    """Unsharded random weights in our naming (small models / tests; device="cuda" generates big
    shapes on the GPU, identically in every process with the same seed)."""
    g = torch.Generator(device=device).manual_seed(seed)
    H, D, I = cfg.hidden_size, cfg.head_dim, cfg.intermediate_size

    def rnd(*shape):
        return (torch.randn(*shape, generator=g, device=device) * std).to(dtype)

    def norm(n):
        return (1.0 + 0.1 * torch.randn(n, generator=g, device=device)).to(dtype)

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


class ShardedCheckpoint:
    """Read THIS rank's slices straight out of HF safetensors files (memory-mapped; only the
    sliced bytes are read), one tensor at a time onto the device.  A Llama-3-70B rank at TP=8 reads
    ~17.6 GB instead of materialising all 141 GB on every rank."""

    def __init__(self, model_dir: str):
        from safetensors import safe_open
        self.files = sorted(glob.glob(os.path.join(model_dir, "*.safetensors")))
        self._open = {f: safe_open(f, framework="pt") for f in self.files}
        self.where: dict[str, str] = {}
        for f, h in self._open.items():
            for k in h.keys():
                self.where[k] = f
        self.bytes_read = 0

    def __contains__(self, name: str) -> bool:
        return name in self.where

    def get(self, name: str, rows: Optional[tuple] = None, cols: Optional[tuple] = None) -> torch.Tensor:
        sl = self._open[self.where[name]].get_slice(name)
        if rows is not None and cols is not None:
            t = sl[rows[0]:rows[1], cols[0]:cols[1]]
        elif rows is not None:
            t = sl[rows[0]:rows[1]]
        elif cols is not None:
            t = sl[:, cols[0]:cols[1]]
        else:
            t = sl[:]
        self.bytes_read += t.numel() * t.element_size()
        return t


def _span(n: int, rank: int, size: int) -> tuple:
    k = n // size
    return rank * k, (rank + 1) * k


def load_sharded_safetensors(model, model_dir: str) -> int:
    """Populate `model` with its own TP/EP shard (same layout as TransformerLM.load_full_state, but
    without the full tensors ever existing on the host).  Returns the bytes read."""
    c = model.cfg
    ck = ShardedCheckpoint(model_dir)
    r, s = model.tp_rank, model.tp_size
    D, I = c.head_dim, c.intermediate_size
    dev, dt = model.device, model.dtype
    kr = r // model.kv_replicas if model.kv_replicas > 1 else r
    ksz = s // model.kv_replicas if model.kv_replicas > 1 else s
    out: dict[str, torch.Tensor] = {}

    def put(name: str, t: torch.Tensor) -> None:
        out[name] = t.to(device=dev, dtype=dt).contiguous()

    put("embed", ck.get("model.embed_tokens.weight"))
    put("norm", ck.get("model.norm.weight"))
    if not c.tie_word_embeddings and "lm_head.weight" in ck:
        vl = model.vocab_local
        lo, hi = r * vl, min((r + 1) * vl, c.vocab_size)
        t = ck.get("lm_head.weight", rows=(lo, hi))
        if t.shape[0] < vl:  # last rank of a vocab that does not divide: zero rows
            t = torch.cat([t, t.new_zeros(vl - t.shape[0], t.shape[1])])
        put("lm_head", t)
    for i in range(c.num_layers):
        a, p = f"model.layers.{i}.", f"l{i}."
        put(p + "in_norm", ck.get(a + "input_layernorm.weight"))
        put(p + "post_norm", ck.get(a + "post_attention_layernorm.weight"))
        q = ck.get(a + "self_attn.q_proj.weight", rows=_span(c.num_heads * D, r, s))
        k = ck.get(a + "self_attn.k_proj.weight", rows=_span(c.num_kv_heads * D, kr, ksz))
        v = ck.get(a + "self_attn.v_proj.weight", rows=_span(c.num_kv_heads * D, kr, ksz))
        put(p + "qkv", torch.cat([q, k, v]))
        put(p + "o", ck.get(a + "self_attn.o_proj.weight", cols=_span(c.num_heads * D, r, s)))
        if c.qk_norm:
            put(p + "q_norm", ck.get(a + "self_attn.q_norm.weight"))
            put(p + "k_norm", ck.get(a + "self_attn.k_norm.weight"))
        if c.is_moe:
            m = a + "block_sparse_moe."
            put(p + "gate", ck.get(m + "gate.weight"))
            es = range(model.e_offset, model.e_offset + model.e_local)
            put(p + "w13", torch.stack([torch.cat([ck.get(m + f"experts.{e}.w1.weight"),
                                                   ck.get(m + f"experts.{e}.w3.weight")]) for e in es]))
            put(p + "w2", torch.stack([ck.get(m + f"experts.{e}.w2.weight") for e in es]))
        else:
            g = ck.get(a + "mlp.gate_proj.weight", rows=_span(I, r, s))
            u = ck.get(a + "mlp.up_proj.weight", rows=_span(I, r, s))
            put(p + "gate_up", torch.cat([g, u]))
            put(p + "down", ck.get(a + "mlp.down_proj.weight", cols=_span(I, r, s)))
    model.w = out
    return ck.bytes_read


def load_weights(model, load_format: str = "auto", seed: int = 0) -> str:
    """Populate `model` (TransformerLM).  Returns the source used: 'safetensors' | 'random'."""
    if load_format == "random_full":  # unsharded host init, then shard: identical model for any TP size
        model.load_full_state(random_full_state(model.cfg, seed=seed, std=0.05, dtype=torch.float32))
        return "random_full"
    if load_format in ("auto", "safetensors"):
        model_dir = find_local_model_dir(model.cfg.name)
        if model_dir is not None and glob.glob(os.path.join(model_dir, "*.safetensors")):
            load_sharded_safetensors(model, model_dir)
            return "safetensors"
        if load_format == "safetensors":
            raise FileNotFoundError(f"no safetensors for {model.cfg.name}")
    model.init_random(seed=seed)
    return "random"
