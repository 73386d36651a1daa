#!/usr/bin/env python3
"""Headline benchmark: output tok/s (node) + p50 TTFT at a fixed QPS, Llama-3.2-1B-Instruct,
aggregated serving (BASELINE.json metric / config 2).

Each rank (one per GPU, launched by torch.distributed.run) runs an independent engine replica -
the reference scales Llama-3.2-1B by `replicas:` of single-GPU workers behind the frontend router
 - and drives it with an open-loop Poisson arrival process at --qps requests/s
per GPU (weak scaling).  Workload shape: ISL 4000 / OSL 500, the only request shape the reference
quantifies (examples/dgdr/trtllm/dgdr.yaml:22-26).  Prompts are synthetic random token ids and the
weights are random-init of the real architecture (no network on the GPU box); every request
generates exactly OSL tokens (ignore_eos).

A "step" is one engine iteration (continuous batching: decodes + chunked prefill under the token
budget).  W warmup steps fill the pipeline; then exactly K steps are timed between a barrier +
device sync on both sides.  value = output tokens produced in the timed window summed over ranks
/ the slowest rank's window.  TTFT is measured from each request's scheduled Poisson arrival
(queueing included) for requests whose first token lands in the window.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

BASELINE_METRIC = "output tok/s (node) + p50 TTFT at fixed QPS, Llama-3.2-1B agg vs disagg"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--warmup", type=int, default=1500)
    ap.add_argument("--model", default="meta-llama/Llama-3.2-1B-Instruct")
    ap.add_argument("--isl", type=int, default=4000)
    ap.add_argument("--osl", type=int, default=500)
    ap.add_argument("--qps", type=float, default=float(os.environ.get("MXS_BENCH_QPS", "36")),
                    help="Poisson arrival rate per GPU (requests/s)")
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-num-batched-tokens", type=int, default=8192)
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--enforce-eager", action="store_true")
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default="auto")
    return ap.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    on_gpu = torch.cuda.is_available() and a.device != "cpu"
    if on_gpu:
        torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl" if on_gpu else "gloo")

    from mxserve.config import EngineArgs
    from mxserve.engine.engine import LLMEngine
    from mxserve.engine.request import SamplingParams

    args = EngineArgs(model=a.model, device="cuda" if on_gpu else "cpu", max_num_seqs=a.max_num_seqs,
                      max_num_batched_tokens=a.max_num_batched_tokens, max_model_len=a.max_model_len,
                      enforce_eager=a.enforce_eager, seed=a.seed)
    if not on_gpu:  # plumbing run only (CPU container): keep it tiny
        args = args.replace(model="tiny-llama", max_model_len=1024, cpu_num_blocks=4096)
        a.isl, a.osl = min(a.isl, 200), min(a.osl, 20)
    eng = LLMEngine(args)
    vocab = eng.model_config.vocab_size

    # open-loop Poisson arrivals, identical stream shape on every rank but distinct prompts
    rng = np.random.default_rng(1234 + rank)
    horizon = 4096
    gaps = rng.exponential(1.0 / a.qps, size=horizon)
    arrivals = np.cumsum(gaps)
    prompts = rng.integers(100, vocab - 100, size=(horizon, a.isl), dtype=np.int64)
    sp = SamplingParams(max_tokens=a.osl, temperature=a.temperature, ignore_eos=True)

    sync = torch.cuda.synchronize if on_gpu else (lambda: None)

    def barrier():
        if world > 1:
            dist.barrier()
        sync()

    arrival_of: dict[str, float] = {}
    first_tok: dict[str, float] = {}
    last_tok: dict[str, float] = {}
    itls: list[float] = []
    nxt = 0
    t_start = None

    def admit(now_rel: float):
        nonlocal nxt
        while nxt < horizon and arrivals[nxt] <= now_rel:
            rid = f"r{rank}-{nxt}"
            eng.add_request(prompts[nxt].tolist(), sp, request_id=rid)
            arrival_of[rid] = t_start + arrivals[nxt]
            nxt += 1

    def run_step(record: bool, counters: dict):
        admit(time.perf_counter() - t_start)
        if not eng.has_unfinished() and nxt < horizon:  # idle: wait for the next arrival
            time.sleep(max(0.0, t_start + arrivals[nxt] - time.perf_counter()))
            admit(time.perf_counter() - t_start)
        outs = eng.step()
        now = time.perf_counter()
        for o in outs:
            rid = o.request_id
            if rid not in first_tok:
                first_tok[rid] = now
                if record:
                    counters["ttft"].append(now - arrival_of[rid])
            elif record:
                itls.append(now - last_tok[rid])
            last_tok[rid] = now
            if record:
                counters["tokens"] += 1

    barrier()
    t_start = time.perf_counter()
    junk = {"ttft": [], "tokens": 0}
    for _ in range(a.warmup):
        run_step(False, junk)
    barrier()
    c = {"ttft": [], "tokens": 0}
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run_step(True, c)
    barrier()
    dt = time.perf_counter() - t0

    ttft = np.array(c["ttft"]) if c["ttft"] else np.array([float("nan")])
    itl = np.array(itls) if itls else np.array([float("nan")])
    local_stats = torch.tensor([dt, float(c["tokens"]), float(np.nanmedian(ttft)), float(np.nanmedian(itl)),
                                float(len(c["ttft"]))], dtype=torch.float64)
    if world > 1:
        gathered = [torch.zeros_like(local_stats) for _ in range(world)]
        dist.all_gather_object(gathered, local_stats)
        allst = torch.stack(gathered)
    else:
        allst = local_stats.unsqueeze(0)
    if rank == 0:
        t_max = float(allst[:, 0].max())
        tokens = float(allst[:, 1].sum())
        value = tokens / t_max
        col = allst.numpy()
        ttft_p50 = float(np.median(col[:, 2][~np.isnan(col[:, 2])])) * 1e3 if np.any(~np.isnan(col[:, 2])) else None
        itl_p50 = float(np.median(col[:, 3][~np.isnan(col[:, 3])])) * 1e3 if np.any(~np.isnan(col[:, 3])) else None
        st = eng.stats()
        line = {
            "metric": BASELINE_METRIC,
            "value": round(value, 2),
            "unit": "tok/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(t_max / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if on_gpu else "fp32",
            "data": "synthetic (random prompt token ids, random-init weights, Poisson arrivals)",
            "config": {"model": args.model if on_gpu else "tiny-llama (CPU plumbing run)",
                       "global_batch": int(world * a.max_num_seqs), "seq_len": a.isl + a.osl,
                       "parallelism": f"dp{world}", "mode": "agg", "isl": a.isl, "osl": a.osl,
                       "qps_per_gpu": a.qps, "qps_node": a.qps * world},
            "ttft_p50_ms": None if ttft_p50 is None else round(ttft_p50, 2),
            "itl_p50_ms": None if itl_p50 is None else round(itl_p50, 3),
            "requests_with_first_token": int(allst[:, 4].sum()),
            "sla_isl4000_osl500": {"ttft_ms<=600": ttft_p50 is not None and ttft_p50 <= 600,
                                   "itl_ms<=25": itl_p50 is not None and itl_p50 <= 25},
            "engine": {"kv_blocks": st["num_blocks"], "running_at_end": st["num_running"],
                       "waiting_at_end": st["num_waiting"], "preemptions": st["num_preemptions"],
                       "graphs": sorted(eng.runner.graphs) if on_gpu else []},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
