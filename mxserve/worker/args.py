"""Worker CLI: accepts the vLLM, SGLang and TRT-LLM flag dialects used by the reference manifests
 and maps them onto one EngineArgs.

  vLLM   (examples/deploy/vllm/*.yaml):   --model, --is-decode-worker, --is-prefill-worker, ...
  SGLang (examples/deploy/sglang/*.yaml): --model-path, --served-model-name, --page-size, --tp,
         --trust-remote-code, --skip-tokenizer-init, --disaggregation-mode,
         --disaggregation-transfer-backend, --disaggregation-bootstrap-port, --host
  TRT-LLM (examples/deploy/trtllm, dgdr): --model-path, --served-model-name, --disaggregation-mode,
         --extra-engine-args <yaml>
Precedence: CLI > --extra-engine-args YAML > MXS_* env > defaults.
"""
from __future__ import annotations

import argparse
import logging
import os
from dataclasses import dataclass, field
from typing import Optional

import yaml

from ..config import EngineArgs, env_overrides


@dataclass
class WorkerArgs:
    engine: EngineArgs
    host: str = "0.0.0.0"
    port: int = 0  # 0 = pick DYN_SYSTEM_PORT / 8081
    frontend_url: Optional[str] = None
    advertise_host: Optional[str] = None
    dialect: str = "vllm"
    worker_id: Optional[str] = None
    # configuration problems the worker started with anyway (reported by /health "config_warnings")
    warnings: list = field(default_factory=list)


log = logging.getLogger("mxserve.worker.args")
# the checkout / image root: the reference runs its workers from /workspace (examples/deploy/vllm/
# agg.yaml:28) and points --extra-engine-args at ./examples/backends/... inside the NVIDIA image
# (examples/dgdr/trtllm/disagg.yaml:29,39-40); the same relative paths exist under this root
PACKAGE_ROOT = os.environ.get("MXS_EXAMPLES_ROOT") or os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))


def _parser(dialect: str) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog=f"python -m dynamo.{dialect}", allow_abbrev=False)
    # model identity
    ap.add_argument("--model", "--model-path", dest="model", default=None)
    ap.add_argument("--served-model-name", default=None)
    ap.add_argument("--tokenizer", default=None)
    ap.add_argument("--trust-remote-code", action="store_true")
    ap.add_argument("--skip-tokenizer-init", action="store_true")
    ap.add_argument("--dtype", default=None)
    ap.add_argument("--load-format", default=None)
    ap.add_argument("--seed", type=int, default=None)
    # parallelism
    ap.add_argument("--tensor-parallel-size", "--tp", "--tp-size", dest="tp", type=int, default=None)
    ap.add_argument("--moe-dispatch", choices=["allreduce", "a2a"], default=None,
                    help="MoE expert parallelism: partial sums + all-reduce, or all-to-all token dispatch")
    # memory / batching (vLLM names, then SGLang / TRT-LLM aliases)
    ap.add_argument("--block-size", "--page-size", "--tokens-per-block", dest="block_size", type=int, default=None)
    ap.add_argument("--max-model-len", "--context-length", "--max-seq-len", dest="max_model_len", type=int,
                    default=None)
    ap.add_argument("--max-num-seqs", "--max-running-requests", "--max-batch-size", dest="max_num_seqs", type=int,
                    default=None)
    ap.add_argument("--max-num-batched-tokens", "--chunked-prefill-size", "--max-num-tokens",
                    dest="max_num_batched_tokens", type=int, default=None)
    ap.add_argument("--itl-target-ms", dest="itl_target_ms", type=float, default=None,
                    help="decode-aware prefill chunking: keep each step's predicted time under this ITL")
    ap.add_argument("--gpu-memory-utilization", "--mem-fraction-static", "--free-gpu-memory-fraction",
                    dest="gpu_memory_utilization", type=float, default=None)
    ap.add_argument("--num-gpu-blocks-override", dest="num_gpu_blocks", type=int, default=None)
    ap.add_argument("--kv-cache-dtype", dest="kv_cache_dtype", default=None,
                    help="auto (bf16) | fp8 | fp8_e4m3 (vLLM / SGLang flag; TRT-LLM: kv_cache_config.dtype)")
    ap.add_argument("--enforce-eager", "--disable-cuda-graph", dest="enforce_eager", action="store_true",
                    default=None)
    ap.add_argument("--enable-prefix-caching", dest="enable_prefix_caching", action="store_true", default=None)
    ap.add_argument("--async-scheduling", dest="async_scheduling", action="store_true", default=None)
    ap.add_argument("--no-async-scheduling", dest="async_scheduling", action="store_false")
    ap.add_argument("--no-enable-prefix-caching", "--disable-radix-cache", dest="enable_prefix_caching",
                    action="store_false")
    ap.add_argument("--no-enable-chunked-prefill", dest="enable_chunked_prefill", action="store_false",
                    default=None)
    ap.add_argument("--device", default=None)
    # disaggregation
    ap.add_argument("--is-decode-worker", action="store_true")
    ap.add_argument("--is-prefill-worker", action="store_true")
    ap.add_argument("--disaggregation-mode", choices=["null", "prefill", "decode", "prefill_and_decode"],
                    default=None)
    ap.add_argument("--disaggregation-transfer-backend", default=None)
    ap.add_argument("--disaggregation-bootstrap-port", type=int, default=None)
    ap.add_argument("--extra-engine-args", default=None)
    # serving
    ap.add_argument("--host", default=os.environ.get("MXS_WORKER_HOST", "0.0.0.0"))
    ap.add_argument("--port", type=int, default=int(os.environ.get("DYN_SYSTEM_PORT", os.environ.get("MXS_WORKER_PORT",
                                                                                                       "8081"))))
    ap.add_argument("--frontend-url", default=os.environ.get("MXS_FRONTEND_URL", os.environ.get("DYN_FRONTEND_URL")))
    ap.add_argument("--advertise-host", default=os.environ.get("POD_IP", os.environ.get("MXS_ADVERTISE_HOST")))
    ap.add_argument("--worker-id", default=os.environ.get("MXS_WORKER_ID"))
    return ap


# TRT-LLM engine-config YAML keys (--extra-engine-args) -> EngineArgs fields
_YAML_MAP = {
    "tensor_parallel_size": "tensor_parallel_size", "max_batch_size": "max_num_seqs",
    "max_num_tokens": "max_num_batched_tokens", "max_seq_len": "max_model_len",
    "enable_chunked_prefill": "enable_chunked_prefill", "tokens_per_block": "block_size",
    "max_model_len": "max_model_len", "max_num_seqs": "max_num_seqs", "block_size": "block_size",
    "gpu_memory_utilization": "gpu_memory_utilization", "enforce_eager": "enforce_eager",
    "moe_dispatch": "moe_dispatch", "itl_target_ms": "itl_target_ms",
}


def resolve_engine_args_path(path: str) -> Optional[str]:
    """The file an --extra-engine-args path names: as given (relative to the working directory), else
    the same path under PACKAGE_ROOT (a reference path like ./examples/backends/trtllm/engine_configs/
    qwen3/prefill.yaml or /workspace/examples/... resolves to this image's copy).  None if neither."""
    if not path:
        return None
    if os.path.exists(path):
        return path
    rel = os.path.normpath(path)
    for prefix in ("/workspace/", "workspace/"):
        if rel.startswith(prefix):
            rel = rel[len(prefix):]
    rel = rel.lstrip("/")
    cand = os.path.join(PACKAGE_ROOT, rel)
    return cand if os.path.exists(cand) else None


def load_extra_engine_args(path: str, warnings: Optional[list] = None) -> dict:
    """Parse a TRT-LLM/vLLM engine YAML into EngineArgs overrides.  The path is resolved against the
    image layout (resolve_engine_args_path); a file that is still missing is NOT silently dropped: it
    is logged and appended to `warnings` (the worker reports them in /health), and the worker starts
    with its other settings."""
    found = resolve_engine_args_path(path)
    if found is None:
        if path:
            msg = (f"--extra-engine-args {path!r} not found (cwd {os.getcwd()!r}, image root {PACKAGE_ROOT!r}); "
                   "starting without it")
            log.warning(msg)
            if warnings is not None:
                warnings.append(msg)
        return {}
    if found != path:
        log.info("--extra-engine-args %s resolved to %s", path, found)
    with open(found) as f:
        d = yaml.safe_load(f) or {}
    out = {}
    for k, v in d.items():
        if k in _YAML_MAP:
            out[_YAML_MAP[k]] = v
    kvc = d.get("kv_cache_config") or {}
    if "free_gpu_memory_fraction" in kvc:
        out["gpu_memory_utilization"] = float(kvc["free_gpu_memory_fraction"])
    if "enable_block_reuse" in kvc:
        out["enable_prefix_caching"] = bool(kvc["enable_block_reuse"])
    if kvc.get("dtype"):
        out["kv_cache_dtype"] = str(kvc["dtype"])
    if d.get("cuda_graph_config") is None and "cuda_graph_config" in d:
        out["enforce_eager"] = True
    return out


def parse_worker_args(argv: list[str], dialect: str = "vllm") -> WorkerArgs:
    a = _parser(dialect).parse_args(argv)
    kw = env_overrides()
    warnings: list = []
    if a.extra_engine_args:
        kw.update(load_extra_engine_args(a.extra_engine_args, warnings))
    cli = {
        "model": a.model, "served_model_name": a.served_model_name, "dtype": a.dtype, "load_format": a.load_format,
        "seed": a.seed, "tensor_parallel_size": a.tp, "block_size": a.block_size, "max_model_len": a.max_model_len,
        "max_num_seqs": a.max_num_seqs, "max_num_batched_tokens": a.max_num_batched_tokens,
        "itl_target_ms": a.itl_target_ms, "gpu_memory_utilization": a.gpu_memory_utilization, "num_gpu_blocks": a.num_gpu_blocks,
        "enforce_eager": a.enforce_eager, "enable_prefix_caching": a.enable_prefix_caching,
        "enable_chunked_prefill": a.enable_chunked_prefill, "device": a.device,
        "async_scheduling": a.async_scheduling, "moe_dispatch": a.moe_dispatch,
        "trust_remote_code": a.trust_remote_code or None, "skip_tokenizer_init": a.skip_tokenizer_init or None,
        "bootstrap_port": a.disaggregation_bootstrap_port, "kv_cache_dtype": a.kv_cache_dtype,
    }
    kw.update({k: v for k, v in cli.items() if v is not None})
    mode = "agg"
    if a.is_prefill_worker or a.disaggregation_mode == "prefill":
        mode = "prefill"
    elif a.is_decode_worker or a.disaggregation_mode == "decode":
        mode = "decode"
    kw["disagg_mode"] = mode
    if a.disaggregation_transfer_backend:
        kw["kv_transfer_backend"] = {"nixl": "xgmi", "mooncake": "xgmi"}.get(a.disaggregation_transfer_backend,
                                                                           a.disaggregation_transfer_backend)
    if kw.get("block_size", 16) != 16:
        raise ValueError("only --page-size/--block-size 16 is supported (the kernels' block shape)")
    eng = EngineArgs(**kw)
    if eng.model is None:
        raise SystemExit("--model / --model-path is required")
    return WorkerArgs(engine=eng, host=a.host, port=a.port, frontend_url=a.frontend_url,
                      advertise_host=a.advertise_host, dialect=dialect, worker_id=a.worker_id, warnings=warnings)
