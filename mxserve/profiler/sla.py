"""SLA profiler for DynamoGraphDeploymentRequests (replaces the reference's AIConfigurator sweep,
examples/dgdr/trtllm/dgdr.yaml:14-31: `useAiConfigurator`, `aicSystem: a100_sxm`).

Given a model, ISL/OSL and TTFT/ITL targets it estimates, per tensor-parallel degree, the prefill
latency and the largest decode batch that meets the ITL target, then sizes prefill and decode
replica counts for the GPUs of one node.  The estimate is a roofline with efficiencies calibrated
on this framework's own MI355X measurements (profiles/r1_*: prefill linear layers ~0.67 PF/s
effective at 8k-token chunks, decode attention 5.1 TB/s, decode weights ~2.5 TB/s at batch 256).

`--measure` (a DGDR with `useAiConfigurator: false`, run by the operator as a profiling Job on one
GPU) replaces both halves of the model with live timings of this engine on the local GPU: the
time to first token of an ISL-token prompt, and decode step time (graph replay, forward + logits +
sampling) at a sweep of batch sizes over KV contexts of ISL + OSL/2 tokens.  The plan then uses the
measured TTFT (divided by TP for TP > 1, plus the all-reduce term) and the measured ITL(batch) curve
(scaled the same way).  `--output-configmap` stores the result in a ConfigMap for the operator.
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
    # MI355X: 2.5 PF bf16 dense, 8 TB/s spec (6.3 measured), 288 GB, 7 xGMI links x ~153 GB/s.
    # Efficiencies this engine measures (round 3-4): batched prefill ~1.1 PF/s (0.44 of dense peak,
    # profiles/r3/s3/prefill_capacity), decode KV streaming 6.1-6.4 TB/s (0.97 of achievable)
    "mi355x": System("mi355x", 2.5e15, 6.3e12, 288e9, 8, 153e9, 0.44, 0.97, 0.6e-3),
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


class Measured:
    """Live timings on the local GPU (TP = 1), used in place of the roofline terms."""

    def __init__(self, d: dict):
        self.d = d
        self.ttft_s = d["ttft_ms"] / 1e3
        self.batches = [int(b) for b in d["decode_itl_ms"]]
        self.itls = [d["decode_itl_ms"][str(b)] / 1e3 for b in self.batches]

    def itl(self, batch: int) -> float:
        """Piecewise-linear in batch through the measured points (linear extrapolation past them)."""
        bs, ts = self.batches, self.itls
        if batch <= bs[0]:
            return ts[0]
        for (b0, t0), (b1, t1) in zip(zip(bs, ts), zip(bs[1:], ts[1:])):
            if batch <= b1:
                return t0 + (t1 - t0) * (batch - b0) / (b1 - b0)
        b0, b1, t0, t1 = bs[-2], bs[-1], ts[-2], ts[-1]
        return t1 + (t1 - t0) * (batch - b1) / max(1, b1 - b0)


def measure(model: str, isl: int, osl: int, batches=(1, 8, 32, 64, 128, 256), seed: int = 0) -> dict:
    """Time this engine on the local GPU at TP = 1 (random-init weights of the real shapes)."""
    import math as _m
    import time as _t

    import torch

    from ..config import EngineArgs
    from ..engine.engine import LLMEngine
    from ..engine.request import SamplingParams
    from ..models.llama import AttnMetadata
    from .. import ops
    ctx = isl + osl // 2
    bmax = max(batches)
    nb_seq = _m.ceil((ctx + 1) / 16)
    eng = LLMEngine(EngineArgs(model=model, device="cuda", num_gpu_blocks=max(bmax * nb_seq + 64, 4096),
                               max_model_len=max(8192, isl + osl + 16), max_num_seqs=max(16, bmax),
                               enforce_eager=True, seed=seed))
    cfg = eng.model_config
    # TTFT: one ISL-token prompt through the engine (chunked prefill + first sample), median of 3
    ttfts = []
    for i in range(4):
        prompt = torch.randint(100, cfg.vocab_size - 100, (isl,), generator=torch.Generator().manual_seed(i)).tolist()
        torch.cuda.synchronize()
        t0 = _t.perf_counter()
        eng.generate([prompt], SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
        torch.cuda.synchronize()
        ttfts.append(_t.perf_counter() - t0)
        eng.kv.pool.reset_prefix_cache()
    ttft = sorted(ttfts[1:])[1]
    # decode: one step (forward + logits + sampling) for B sequences of ctx tokens of (random) KV
    m, kv, dev = eng.runner.model, eng.runner.kv_cache, eng.runner.device
    itl = {}
    for b in batches:
        bt = torch.arange(b * nb_seq, dtype=torch.int32, device=dev).view(b, nb_seq)
        pos = torch.full((b,), ctx, dtype=torch.int64, device=dev)
        sl = torch.full((b,), ctx + 1, dtype=torch.int32, device=dev)
        md = AttnMetadata(positions=pos, slot_mapping=bt[:, -1].long() * 16 + ctx % 16, block_tables=bt, seq_lens=sl,
                          query_start_loc=torch.arange(b + 1, dtype=torch.int32, device=dev),
                          logits_indices=torch.arange(b, device=dev), num_decodes=b, num_prefills=0,
                          num_prefill_tokens=0, max_query_len=1, max_seq_len=ctx + 1)
        ids = torch.randint(100, cfg.vocab_size - 100, (b,), device=dev)
        zeros = torch.zeros(b, device=dev)
        ones = torch.ones(b, device=dev)
        ks = torch.zeros(b, dtype=torch.int32, device=dev)
        seeds = torch.arange(b, device=dev)

        def step():
            logits = m.compute_logits(m.forward(ids, md, kv))
            return ops.sample(logits, zeros, ones, ks, seeds, seeds)

        with torch.inference_mode():
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            itl[str(b)] = round(e0.elapsed_time(e1) / 10, 4)
        del g
    dev_name = torch.cuda.get_device_name(dev)
    eng.close()
    return {"model": model, "isl": isl, "osl": osl, "ctx": ctx, "tp": 1, "device": dev_name,
            "ttft_ms": round(ttft * 1e3, 3), "decode_itl_ms": itl}


def b1_rps(max_batch, dec_itl, osl: int) -> float:
    """Decode requests/s of one TP-1 replica under the ITL model in use (the scale that maps the
    capacity model's per-GPU decode rate onto other TP degrees)."""
    b = max_batch(1)
    return b / (osl * dec_itl(b, 1)) if b else 0.0


def plan(model: str, isl: int, osl: int, ttft_ms: float, itl_ms: float, system: str = "mi355x",
         gpus: int | None = None, measured: dict | None = None) -> dict:
    """Choose prefill/decode TP and replica counts meeting the SLA on one node.  With `measured`
    (see measure()) the TTFT and ITL terms come from live timings instead of the roofline."""
    cfg = get_model_config(model)
    sys = SYSTEMS.get(system.lower(), SYSTEMS["mi355x"])
    ctx = isl + osl // 2
    if measured is not None:
        meas = Measured(measured)

        def pre_lat(tp):  # measured at TP 1; compute splits over TP, all-reduces added
            t = meas.ttft_s / tp
            if tp > 1:
                t += 2 * cfg.num_layers * 2 * isl * cfg.hidden_size * 2 * (tp - 1) / tp / sys.link_bw
            return t

        def dec_itl(b, tp):
            t = meas.itl(b) / tp
            if tp > 1:
                t += 2 * cfg.num_layers * (8e-6 + 2 * b * cfg.hidden_size * 2 / sys.link_bw)
            return t
    else:
        def pre_lat(tp):
            return prefill_latency(cfg, sys, isl, tp)

        def dec_itl(b, tp):
            return decode_itl(cfg, sys, b, ctx, tp)
    gpus = gpus or sys.gpus_per_node
    tps = [t for t in (1, 2, 4, 8) if t <= gpus and cfg.num_heads % t == 0]

    def max_batch(tp: int, cap: int = 1024) -> int:
        """Largest decode batch meeting the ITL target that fits in HBM next to the weights."""
        mem = tp * sys.hbm_bytes * 0.9 - _weights_bytes(cfg)
        lo, hi = 0, min(cap, int(mem // max(1, ctx * cfg.kv_bytes_per_token())) if mem > 0 else 0)
        while lo < hi:
            mid = (lo + hi + 1) // 2
            if dec_itl(mid, tp) <= itl_ms / 1e3:
                lo = mid
            else:
                hi = mid - 1
        return lo
    fits = [t for t in tps if _weights_bytes(cfg) / t < sys.hbm_bytes * 0.8]
    # per-GPU role capacities at TP 1: the one capacity model bench.py's split uses too
    # (profiler/capacity.py: this engine's measured MI355X table, else the roofline); a --measure run
    # replaces them with its own live throughputs
    from . import capacity as capm
    cap = capm.capacity(model, isl, osl, itl_ms, system)
    if measured is not None and measured.get("prefill_rps"):
        cap = dict(cap, prefill_rps=measured["prefill_rps"], source="measured")
    if measured is not None:
        b1 = max_batch(1)
        if b1:
            cap = dict(cap, decode_rps=b1 / (osl * dec_itl(b1, 1)), source="measured")
    d1 = b1_rps(max_batch, dec_itl, osl)
    cands = []
    for tp_p in fits:
        ttft = pre_lat(tp_p)
        if ttft * 1e3 > ttft_ms:
            continue
        # requests/s one prefill replica sustains: batched prompts, not one prompt at a time; TP
        # splits the compute and adds the all-reduces (the latency ratio prices them)
        pre_rps = cap["prefill_rps"] * pre_lat(1) / pre_lat(tp_p)
        for tp_d in fits:
            b = max_batch(tp_d)
            if b == 0:
                continue
            itl = dec_itl(b, tp_d)
            # the per-GPU capacity at TP 1, scaled to this TP degree by the ITL model's own ratio
            dec_rps = cap["decode_rps"] * (b / (osl * itl)) / d1 if d1 > 0 else b / (osl * itl)
            # split the node: prefill replicas r_p, decode replicas r_d, r_p*tp_p + r_d*tp_d <= gpus;
            # ties go to fewer prefill replicas (capm.pd_split's rule)
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
        b = max_batch(tp)
        ttft = pre_lat(tp)
        if b == 0 or ttft * 1e3 > ttft_ms:
            continue
        itl = dec_itl(b, tp)
        per = 1.0 / (osl * itl / b + ttft)
        r = gpus // tp
        cand = {"tp": tp, "replicas": r, "batch": b, "requests_per_s": round(r * per, 3),
                "output_tok_per_s": round(r * per * osl, 1), "ttft_ms": round(ttft * 1e3, 2),
                "itl_ms": round(itl * 1e3, 3)}
        if agg is None or cand["requests_per_s"] > agg["requests_per_s"]:
            agg = cand
    best = max(cands, key=lambda c: (c["requests_per_s"], -c["gpus_used"])) if cands else None
    return {"model": cfg.name, "capacity": {k: cap[k] for k in ("prefill_rps", "decode_rps", "source") if k in cap}, "system": sys.name, "gpus": gpus, "sla": {"isl": isl, "osl": osl, "ttft_ms": ttft_ms,
                                                                           "itl_ms": itl_ms},
            "disagg": best, "agg": agg, "feasible": best is not None or agg is not None,
            "source": "measured" if measured is not None else "roofline", "measurements": measured,
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
    ap.add_argument("--measure", action="store_true", help="time the engine on the local GPU (TP 1)")
    ap.add_argument("--output-configmap", default=None,
                    help="store the result as ConfigMap NAME (key results.json) in --namespace")
    ap.add_argument("--namespace", default=None)
    a = ap.parse_args(argv)
    meas = measure(a.model, a.isl, a.osl) if a.measure else None
    res = plan(a.model, a.isl, a.osl, a.ttft, a.itl, a.system, a.gpus, measured=meas)
    out = json.dumps(res, indent=2)
    print(out, flush=True)
    if a.output_configmap:
        import os

        from ..k8s.client import KubeClient
        KubeClient(os.environ.get("MXS_KUBE_SERVER")).apply({"apiVersion": "v1", "kind": "ConfigMap",
                            "metadata": {"name": a.output_configmap, "namespace": a.namespace or "default",
                                         "labels": {"app.kubernetes.io/managed-by": "mxserve-profiler"}},
                            "data": {"results.json": out}})


if __name__ == "__main__":
    main()
