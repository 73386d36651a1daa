"""Typed engine configuration (one dataclass tree, populated from the vLLM / SGLang /
TRT-LLM flag dialects, `--extra-engine-args` YAML and MXS_* env; precedence CLI > YAML > env >
defaults)."""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class EngineArgs:
    model: str = "meta-llama/Llama-3.2-1B-Instruct"
    served_model_name: Optional[str] = None
    device: str = "auto"  # "auto" | "cuda" | "cpu"
    dtype: str = "bfloat16"
    tensor_parallel_size: int = 1
    # MoE expert parallelism over the TP ranks: "allreduce" (each rank runs its experts over the
    # replicated batch, partial outputs summed by the TP all-reduce) or "a2a" (token slices
    # dispatched to expert owners with all-to-all, mxserve/parallel/expert.py)
    moe_dispatch: str = "allreduce"
    block_size: int = 16
    # KV cache storage: "auto" (= the model dtype, bf16) or "fp8" / "fp8_e4m3" (OCP e4m3fn, the
    # gfx950 fp8 format: half the bytes per token, so twice the tokens per GB and half the decode
    # attention traffic; attention math stays bf16/fp32)
    kv_cache_dtype: str = "auto"
    max_model_len: int = 8192
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    enable_chunked_prefill: bool = True
    # decode-aware prefill chunking: cap each step's prefill chunks so the step's predicted time
    # (online step-time model, engine/pacing.py) stays under this inter-token latency (0 = off)
    itl_target_ms: float = 0.0
    enable_prefix_caching: bool = True
    gpu_memory_utilization: float = 0.90
    num_gpu_blocks: Optional[int] = None  # override the memory-derived count
    enforce_eager: bool = False  # disable hipGraph capture of decode steps
    # largest decode batch captured as a hipGraph; 0 = follow max_num_seqs (up to the 512 bucket), so a
    # larger --max-num-seqs never leaves its big decode batches to eager launches
    cuda_graph_max_bs: int = 0
    # schedule + launch step N+1 before waiting for step N's sampled tokens (host work overlaps
    # the GPU; decode inputs are read on the device from the last sampled token of each row)
    async_scheduling: bool = True
    load_format: str = "auto"  # auto | safetensors | random
    seed: int = 0
    # disaggregation role: "agg" | "prefill" | "decode"
    disagg_mode: str = "agg"
    kv_transfer_backend: str = "xgmi"  # xgmi (hipIpc peer copy) | host (staged) | nixl (alias of xgmi)
    bootstrap_port: int = 12345
    trust_remote_code: bool = False
    skip_tokenizer_init: bool = False
    cpu_num_blocks: int = 2048

    @property
    def name(self) -> str:
        return self.served_model_name or self.model

    def replace(self, **kw) -> "EngineArgs":
        return dataclasses.replace(self, **kw)

    def resolved_device(self) -> str:
        if self.device != "auto":
            return self.device
        import torch
        return "cuda" if torch.cuda.is_available() else "cpu"


def env_overrides() -> dict:
    """MXS_* environment overrides (lowest precedence above defaults)."""
    out = {}
    for f in dataclasses.fields(EngineArgs):
        v = os.environ.get("MXS_" + f.name.upper())
        if v is None:
            continue
        t = f.type if isinstance(f.type, type) else str(f.type)
        if "bool" in str(t):
            out[f.name] = v.lower() in ("1", "true", "yes", "on")
        elif "int" in str(t) and "Optional" not in str(t):
            out[f.name] = int(v)
        elif "float" in str(t):
            out[f.name] = float(v)
        elif "Optional[int]" in str(t):
            out[f.name] = int(v)
        else:
            out[f.name] = v
    return out
