"""One capacity model for both disaggregation planners: bench.py's P:D split (disagg_plan) and the
DGDR profiler's replica counts (profiler/sla.py plan).

Capacity of one MI355X in a role, in requests per second of the workload (model, ISL, OSL):
  * prefill: prompt tokens a prefill GPU processes per second (large batched prefill steps) / ISL;
  * decode: running requests a decode GPU holds within the ITL target, / (OSL x ITL at that batch)
    -- every step streams each running request's KV, so the ITL target caps the batch.
Measured values live in capacity_mi355x.json next to this file (scripts/prefill_capacity_probe.py
and scripts/decode_capacity_probe.py write them); a workload without an entry gets the roofline of
sla.py with the efficiencies this engine measures (prefill ~1.1 PF/s dense-equivalent, decode KV
streaming at ~97 % of achievable HBM bandwidth).

Reference: the SLA the reference sizes for (ISL 4000 / OSL 500, TTFT 600 ms, ITL 25 ms),
/root/reference/examples/dgdr/trtllm/dgdr.yaml:22-26, and its independent prefill / decode replica
counts, /root/reference/examples/deploy/vllm/disagg.yaml:22,42.
"""
from __future__ import annotations

import json
import os
from typing import Optional

TABLE_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "capacity_mi355x.json")
# the highest utilisation a role is planned at: Poisson arrivals queue visibly above it
PLAN_UTIL = 0.85


def _key(model: str, isl: int, osl: int) -> str:
    return f"{model}|{int(isl)}|{int(osl)}"


def load_table(path: str = TABLE_PATH) -> dict:
    try:
        with open(path) as f:
            return json.load(f).get("entries", {})
    except (OSError, ValueError):
        return {}


def lookup(model: str, isl: int, osl: int) -> Optional[dict]:
    """The measured entry of a workload, or None."""
    return load_table().get(_key(model, isl, osl))


def roofline(model: str, isl: int, osl: int, itl_ms: float = 25.0, system: str = "mi355x") -> dict:
    """Per-GPU role capacities (TP 1) from sla.py's roofline."""
    from ..models.config import get_model_config
    from . import sla
    cfg = get_model_config(model)
    s = sla.SYSTEMS.get(system.lower(), sla.SYSTEMS["mi355x"])
    flops = 2 * sla._active_params(cfg) * isl + 2 * cfg.num_layers * cfg.num_heads * cfg.head_dim * isl * isl
    prefill = s.bf16_flops * s.prefill_eff / flops
    ctx = isl + osl // 2
    b = sla.max_decode_batch(cfg, s, ctx, 1, itl_ms / 1e3)
    decode = b / (osl * sla.decode_itl(cfg, s, b, ctx, 1)) if b else 0.0
    return {"prefill_rps": prefill, "decode_rps": decode, "decode_batch": b, "source": f"roofline:{s.name}"}


def capacity(model: str, isl: int, osl: int, itl_ms: float = 25.0, system: str = "mi355x") -> dict:
    """{"prefill_rps", "decode_rps", "source", ...}: the measured entry on MI355X when the table
    has the workload, else the roofline.  The measured decode capacity holds for ITL targets at least
    as loose as the one it was measured at (decode_itl_target_ms): a tighter target caps the decode
    batch lower, so the decode side then scales the measurement by the roofline's ratio between the
    two targets (the prefill side does not depend on the ITL)."""
    if system.lower() == "mi355x":
        e = lookup(model, isl, osl)
        if e is not None and e.get("prefill_rps") and e.get("decode_rps"):
            out = dict(e, source=e.get("source", "measured"))
            at = float(e.get("decode_itl_target_ms") or itl_ms)
            if itl_ms < at:
                tight, loose = roofline(model, isl, osl, itl_ms), roofline(model, isl, osl, at)
                ratio = tight["decode_rps"] / loose["decode_rps"] if loose["decode_rps"] else 0.0
                out["decode_rps"] = e["decode_rps"] * ratio
                out["decode_source"] = f"measured at ITL {at:g} ms x roofline ratio for ITL {itl_ms:g} ms"
            return out
    return roofline(model, isl, osl, itl_ms, system)


def pd_split(world: int, prefill_rps: float, decode_rps: float, util: float = PLAN_UTIL) -> tuple:
    """(prefill GPUs, decode GPUs, node request rate) for `world` GPUs: the split whose tighter role
    carries the most, and the rate that loads that role to `util`."""
    if world < 2:
        raise ValueError("a prefill / decode split needs at least 2 GPUs")
    p = max(range(1, world), key=lambda k: (min(k * prefill_rps, (world - k) * decode_rps), -k))
    d = world - p
    return p, d, util * min(p * prefill_rps, d * decode_rps)
