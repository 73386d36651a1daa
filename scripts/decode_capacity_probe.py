#!/usr/bin/env python3
"""Decode-role capacity of one MI355X: requests enter the way a disaggregated
decode worker receives them -- blocks reserved for the prompt (engine.reserve_remote_prefill), the KV
taken as landed (a prefill GPU would have pushed it; the blocks hold a synthetic fill, which the
attention kernels stream exactly like real KV), first token delivered (complete_remote_prefill) --
at a swept Poisson rate; the engine then decodes OSL - 1 tokens per request with its CUDA graphs.

For each rate: ITL p50 / p90 over the steady window and the running batch.  The capacity is the
highest rate whose ITL p90 stays within --itl-ms.  With --write the result is stored in
mxserve/profiler/capacity_mi355x.json (decode_rps) for bench.py's split and the DGDR profiler.

  python scripts/decode_capacity_probe.py --rates 60,70,80,90 --itl-ms 25 --write
"""
import argparse
import json
import os
import sys
import time
import uuid

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_rate(eng, rate: float, isl: int, osl: int, seconds: float, warm_s: float, seed: int) -> dict:
    from mxserve.engine.request import SamplingParams
    rng = np.random.default_rng(seed)
    sp = SamplingParams(max_tokens=osl, temperature=1.0, ignore_eos=True)
    t0 = time.perf_counter()
    next_t = t0 + rng.exponential(1.0 / rate)
    last_tok: dict = {}
    itl: list = []
    running: list = []
    refused = 0
    while True:
        now = time.perf_counter()
        if now - t0 > warm_s + seconds:
            break
        while next_t <= now:
            rid = uuid.uuid4().hex
            prompt = rng.integers(100, 120000, size=isl).tolist()
            if eng.reserve_remote_prefill(prompt, sp, rid) is None:
                refused += 1
            else:
                eng.complete_remote_prefill(rid, int(rng.integers(100, 120000)))
                last_tok[rid] = time.perf_counter()
            next_t += rng.exponential(1.0 / rate)
        outs = eng.step()
        t = time.perf_counter()
        steady = t - t0 > warm_s
        for o in outs:
            p = last_tok.get(o.request_id)
            if p is not None and steady:
                itl.append(t - p)
            if o.finished:
                last_tok.pop(o.request_id, None)
            else:
                last_tok[o.request_id] = t
        if steady:
            running.append(len(eng.scheduler.running))
    # drain
    for rid in list(last_tok):
        eng.abort(rid)
    while eng.has_unfinished():
        eng.step()
    a = np.array(itl) * 1e3
    return {"rate": rate, "itl_p50_ms": round(float(np.percentile(a, 50)), 3) if len(a) else None,
            "itl_p90_ms": round(float(np.percentile(a, 90)), 3) if len(a) else None,
            "running_mean": round(float(np.mean(running)), 1) if running else 0, "tokens": int(len(a)),
            "refused": refused}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="meta-llama/Llama-3.2-1B-Instruct")
    ap.add_argument("--isl", type=int, default=4000)
    ap.add_argument("--osl", type=int, default=500)
    ap.add_argument("--rates", default="60,70,80,90")
    ap.add_argument("--itl-ms", type=float, default=25.0)
    ap.add_argument("--seconds", type=float, default=12.0)
    ap.add_argument("--max-num-seqs", type=int, default=1024)
    ap.add_argument("--write", action="store_true")
    a = ap.parse_args()
    from mxserve.config import EngineArgs
    from mxserve.engine.engine import LLMEngine
    eng = LLMEngine(EngineArgs(model=a.model, device="cuda", max_num_seqs=a.max_num_seqs,
                               max_model_len=max(8192, a.isl + a.osl + 16), load_format="random",
                               disagg_mode="decode", cuda_graph_max_bs=512))
    # a synthetic fill of the whole pool: every reserved block holds finite, non-trivial values
    with torch.inference_mode():
        kv = eng.runner.kv_cache
        kv.view(-1)[:] = 0.01
    warm = a.osl * 0.012 + 2.0  # one request lifetime at ~12 ms per step
    rows = []
    for i, r in enumerate(float(x) for x in a.rates.split(",")):
        row = run_rate(eng, r, a.isl, a.osl, a.seconds, warm, seed=i)
        rows.append(row)
        print(json.dumps(row), flush=True)
    ok = [r for r in rows if r["itl_p90_ms"] is not None and r["itl_p90_ms"] <= a.itl_ms and not r["refused"]]
    cap = max((r["rate"] for r in ok), default=0.0)
    res = {"model": a.model, "isl": a.isl, "osl": a.osl, "itl_target_ms": a.itl_ms, "decode_rps": cap,
           "sweep": rows, "device": torch.cuda.get_device_name(0)}
    print(json.dumps(res), flush=True)
    if a.write and cap > 0:
        from mxserve.profiler import capacity
        path = os.environ.get("MXS_CAPACITY_OUT", capacity.TABLE_PATH)
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            d = {"entries": {}}
        key = f"{a.model}|{a.isl}|{a.osl}"
        e = d["entries"].setdefault(key, {})
        e.update({"decode_rps": cap, "decode_itl_target_ms": a.itl_ms,
                  "decode_source": "scripts/decode_capacity_probe.py (measured)"})
        with open(path, "w") as f:
            json.dump(d, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
