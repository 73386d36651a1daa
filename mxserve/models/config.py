"""Model architecture configs and the built-in model registry.

The reference never ships model code; it names models in its manifests
(`examples/deploy/vllm/agg.yaml:35` Llama-3.2-1B-Instruct, `examples/dgdr/trtllm/dgdr.yaml:11`
Qwen3-0.6B) and BASELINE.json names Llama-3-8B, Llama-3-70B and Mixtral-8x7B.  The GPU box has no
network, so every model can be instantiated from the shapes below with random weights; if a
`config.json` is found on disk (HF_HOME / a local path) it overrides the built-in entry.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class ModelConfig:
    name: str
    arch: str  # "llama" | "qwen3" | "mixtral"
    hidden_size: int
    intermediate_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    vocab_size: int
    rope_theta: float = 10000.0
    rms_norm_eps: float = 1e-5
    tie_word_embeddings: bool = False
    max_position_embeddings: int = 8192
    # llama3 rope scaling (factor, low_freq_factor, high_freq_factor, original_max_pos) or None
    rope_scaling: Optional[dict] = None
    qk_norm: bool = False
    # MoE
    num_experts: int = 0
    num_experts_per_tok: int = 0
    # tokenizer / chat
    bos_token_id: Optional[int] = None
    eos_token_ids: list = field(default_factory=list)
    chat_template: str = "llama3"

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return self.num_layers * 2 * self.num_kv_heads * self.head_dim * dtype_bytes

    def num_params(self) -> int:
        h, i, L = self.hidden_size, self.intermediate_size, self.num_layers
        attn = h * (self.q_size + 2 * self.kv_size) + self.q_size * h
        if self.is_moe:
            mlp = self.num_experts * 3 * h * i + h * self.num_experts
        else:
            mlp = 3 * h * i
        per_layer = attn + mlp + 2 * h + (2 * self.head_dim if self.qk_norm else 0)
        emb = self.vocab_size * h
        return L * per_layer + emb + (0 if self.tie_word_embeddings else emb) + h

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


_LLAMA3_EOS = [128001, 128008, 128009]
_LLAMA31_ROPE = {"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                 "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}

# Shapes: public HF config.json of each model.
REGISTRY: dict[str, ModelConfig] = {}


def _reg(cfg: ModelConfig, *aliases: str) -> None:
    REGISTRY[cfg.name.lower()] = cfg
    for a in aliases:
        REGISTRY[a.lower()] = cfg


_reg(ModelConfig(
    name="meta-llama/Llama-3.2-1B-Instruct", arch="llama", hidden_size=2048, intermediate_size=8192,
    num_layers=16, num_heads=32, num_kv_heads=8, head_dim=64, vocab_size=128256, rope_theta=500000.0,
    rms_norm_eps=1e-5, tie_word_embeddings=True, max_position_embeddings=131072,
    rope_scaling=dict(_LLAMA31_ROPE), bos_token_id=128000, eos_token_ids=list(_LLAMA3_EOS),
    chat_template="llama3"), "llama-3.2-1b", "meta-llama/Llama-3.2-1B", "llama-3.2-1b-instruct")

_reg(ModelConfig(
    name="Qwen/Qwen3-0.6B", arch="qwen3", hidden_size=1024, intermediate_size=3072, num_layers=28,
    num_heads=16, num_kv_heads=8, head_dim=128, vocab_size=151936, rope_theta=1000000.0,
    rms_norm_eps=1e-6, tie_word_embeddings=True, max_position_embeddings=40960, qk_norm=True,
    bos_token_id=None, eos_token_ids=[151645, 151643], chat_template="chatml"), "qwen3-0.6b")

_reg(ModelConfig(
    name="meta-llama/Meta-Llama-3-8B-Instruct", arch="llama", hidden_size=4096, intermediate_size=14336,
    num_layers=32, num_heads=32, num_kv_heads=8, head_dim=128, vocab_size=128256, rope_theta=500000.0,
    rms_norm_eps=1e-5, max_position_embeddings=8192, bos_token_id=128000,
    eos_token_ids=[128001, 128009], chat_template="llama3"),
    "llama-3-8b", "meta-llama/Meta-Llama-3-8B", "meta-llama/Llama-3.1-8B-Instruct")

_reg(ModelConfig(
    name="meta-llama/Meta-Llama-3-70B-Instruct", arch="llama", hidden_size=8192, intermediate_size=28672,
    num_layers=80, num_heads=64, num_kv_heads=8, head_dim=128, vocab_size=128256, rope_theta=500000.0,
    rms_norm_eps=1e-5, max_position_embeddings=8192, bos_token_id=128000,
    eos_token_ids=[128001, 128009], chat_template="llama3"),
    "llama-3-70b", "meta-llama/Meta-Llama-3-70B", "meta-llama/Llama-3.1-70B-Instruct")

_reg(ModelConfig(
    name="mistralai/Mixtral-8x7B-Instruct-v0.1", arch="mixtral", hidden_size=4096, intermediate_size=14336,
    num_layers=32, num_heads=32, num_kv_heads=8, head_dim=128, vocab_size=32000, rope_theta=1000000.0,
    rms_norm_eps=1e-5, max_position_embeddings=32768, num_experts=8, num_experts_per_tok=2,
    bos_token_id=1, eos_token_ids=[2], chat_template="mistral"),
    "mixtral-8x7b", "mistralai/Mixtral-8x7B-v0.1")

# Tiny configs with the same code paths, used by CPU tests.
_reg(ModelConfig(
    name="tiny-llama", arch="llama", hidden_size=128, intermediate_size=256, num_layers=2, num_heads=4,
    num_kv_heads=2, head_dim=32, vocab_size=512, rope_theta=10000.0, tie_word_embeddings=True,
    max_position_embeddings=2048, rope_scaling=dict(_LLAMA31_ROPE, original_max_position_embeddings=64),
    bos_token_id=1, eos_token_ids=[2], chat_template="llama3"))
_reg(ModelConfig(
    name="tiny-qwen3", arch="qwen3", hidden_size=128, intermediate_size=256, num_layers=2, num_heads=4,
    num_kv_heads=2, head_dim=64, vocab_size=512, rope_theta=1000000.0, rms_norm_eps=1e-6,
    tie_word_embeddings=True, max_position_embeddings=2048, qk_norm=True, eos_token_ids=[2],
    chat_template="chatml"))
_reg(ModelConfig(
    name="tiny-mixtral", arch="mixtral", hidden_size=128, intermediate_size=192, num_layers=2, num_heads=4,
    num_kv_heads=2, head_dim=32, vocab_size=512, rope_theta=1000000.0, max_position_embeddings=2048,
    num_experts=4, num_experts_per_tok=2, bos_token_id=1, eos_token_ids=[2], chat_template="mistral"))
_reg(ModelConfig(
    name="tiny-qwen3-gpu", arch="qwen3", hidden_size=256, intermediate_size=512, num_layers=2, num_heads=4,
    num_kv_heads=2, head_dim=128, vocab_size=1024, rope_theta=1000000.0, rms_norm_eps=1e-6,
    tie_word_embeddings=True, max_position_embeddings=4096, qk_norm=True, eos_token_ids=[2],
    chat_template="chatml"))
_reg(ModelConfig(
    name="tiny-mixtral-gpu", arch="mixtral", hidden_size=256, intermediate_size=512, num_layers=2, num_heads=8,
    num_kv_heads=2, head_dim=64, vocab_size=1024, rope_theta=1000000.0, max_position_embeddings=4096,
    num_experts=4, num_experts_per_tok=2, bos_token_id=1, eos_token_ids=[2], chat_template="mistral"))
# A GPU-test config: real head dims (64/128) and GQA ratios, few layers.
_reg(ModelConfig(
    name="small-llama", arch="llama", hidden_size=1024, intermediate_size=2816, num_layers=4, num_heads=16,
    num_kv_heads=4, head_dim=64, vocab_size=32000, rope_theta=500000.0, tie_word_embeddings=True,
    max_position_embeddings=8192, bos_token_id=1, eos_token_ids=[2], chat_template="llama3"))


def _from_hf_json(name: str, d: dict) -> ModelConfig:
    arch_list = d.get("architectures") or []
    mt = d.get("model_type", "")
    if "qwen3" in mt or any("Qwen3" in a for a in arch_list):
        arch = "qwen3"
    elif "mixtral" in mt or d.get("num_local_experts"):
        arch = "mixtral"
    else:
        arch = "llama"
    nh = d["num_attention_heads"]
    hd = d.get("head_dim") or d["hidden_size"] // nh
    eos = d.get("eos_token_id")
    eos = eos if isinstance(eos, list) else ([eos] if eos is not None else [])
    rs = d.get("rope_scaling")
    if rs is not None and rs.get("rope_type", rs.get("type")) != "llama3":
        rs = None
    return ModelConfig(
        name=name, arch=arch, hidden_size=d["hidden_size"], intermediate_size=d["intermediate_size"],
        num_layers=d["num_hidden_layers"], num_heads=nh, num_kv_heads=d.get("num_key_value_heads", nh),
        head_dim=hd, vocab_size=d["vocab_size"], rope_theta=float(d.get("rope_theta", 10000.0)),
        rms_norm_eps=float(d.get("rms_norm_eps", 1e-5)),
        tie_word_embeddings=bool(d.get("tie_word_embeddings", False)),
        max_position_embeddings=int(d.get("max_position_embeddings", 8192)), rope_scaling=rs,
        qk_norm=(arch == "qwen3"), num_experts=int(d.get("num_local_experts", 0) or 0),
        num_experts_per_tok=int(d.get("num_experts_per_tok", 0) or 0), bos_token_id=d.get("bos_token_id"),
        eos_token_ids=eos,
        chat_template={"qwen3": "chatml", "mixtral": "mistral"}.get(arch, "llama3"))


def find_local_model_dir(name: str) -> Optional[str]:
    """Locate a HF snapshot for `name` on disk (a path, or HF_HOME hub cache). No network."""
    if os.path.isdir(name) and os.path.exists(os.path.join(name, "config.json")):
        return name
    home = os.environ.get("HF_HOME") or os.path.join(os.path.expanduser("~"), ".cache", "huggingface")
    repo_dir = os.path.join(home, "hub", "models--" + name.replace("/", "--"), "snapshots")
    if os.path.isdir(repo_dir):
        for snap in sorted(os.listdir(repo_dir)):
            p = os.path.join(repo_dir, snap)
            if os.path.exists(os.path.join(p, "config.json")):
                return p
    return None


def get_model_config(name: str) -> ModelConfig:
    """`name@layers=N` keeps a model's real shapes with only its first N layers (tests and probes of
    big models on one GPU, e.g. Llama-3-70B TP=8 with 8 ranks sharing the test box's GPU)."""
    if "@layers=" in name:
        base, n = name.split("@layers=", 1)
        cfg = get_model_config(base)
        return dataclasses.replace(cfg, num_layers=int(n), name=name)
    local = find_local_model_dir(name)
    if local is not None:
        with open(os.path.join(local, "config.json")) as f:
            return _from_hf_json(name, json.load(f))
    key = name.lower()
    if key in REGISTRY:
        cfg = REGISTRY[key]
        return dataclasses.replace(cfg, name=name if "/" in name else cfg.name)
    # tolerate org-less or path-like names ("/models/Llama-3.2-1B-Instruct")
    base = os.path.basename(key.rstrip("/"))
    for k, cfg in REGISTRY.items():
        if k.split("/")[-1] == base:
            return dataclasses.replace(cfg, name=name)
    raise KeyError(f"unknown model {name!r}; known: {sorted(set(c.name for c in REGISTRY.values()))}")
