#!/usr/bin/env python3
"""Decode-role capacity of one MI355X: requests enter the way a disaggregated
decode worker receives them -- blocks reserved for the prompt (engine.reserve_remote_prefill), the KV
taken as landed (a prefill GPU would have pushed it; the blocks hold a synthetic fill, which the
attention kernels stream exactly like real KV), first token delivered (complete_remote_prefill) --
and the engine decodes OSL - 1 tokens per request with its CUDA graphs.

Closed loop per batch size R: R requests are kept running (a finished one is replaced at once), so
after one request lifetime the contexts are spread uniformly over [ISL, ISL + OSL] as under an open
load, and the step time measured is the ITL at that batch.  A decode GPU at batch R completes
R / (OSL x ITL(R)) requests per second; its capacity is the largest of those whose ITL p90 stays
within --itl-ms.  (An open-loop rate sweep cannot measure this in seconds: near capacity the running
set relaxes over many request lifetimes -- Little's law with an ITL that grows with the batch -- so a
short window under-reports the batch and the ITL and over-reports the rate; r4 dec1 did exactly
that, profiles/r4/decode_capacity_open_loop_misleading.jsonl.)  With --write the result is stored in
mxserve/profiler/capacity_mi355x.json (decode_rps) for bench.py's split and the DGDR profiler.

  python scripts/decode_capacity_probe.py --batches 256,384,512,640,768 --itl-ms 25 --write
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


def run_batch(eng, R: int, isl: int, osl: int, seconds: float, seed: int) -> dict:
    from mxserve.engine.request import SamplingParams
    rng = np.random.default_rng(seed)
    sp = SamplingParams(max_tokens=osl, temperature=1.0, ignore_eos=True)
    live: set = set()
    refused = 0

    def top_up(n: int):
        nonlocal refused
        while len(live) < n:
            rid = uuid.uuid4().hex
            if eng.reserve_remote_prefill(rng.integers(100, 120000, size=isl).tolist(), sp, rid) is None:
                refused += 1
                return
            eng.complete_remote_prefill(rid, int(rng.integers(100, 120000)))
            live.add(rid)

    # stagger: the first R requests start over one lifetime (R / OSL per step), not all at once, so
    # their contexts and finish times spread like an open load's
    steps, t_steps, running = 0, [], []
    warm_steps = osl + 50
    t_end = None
    while True:
        top_up(min(R, max(1, (steps + 1) * R // osl)))
        t0 = time.perf_counter()
        outs = eng.step()
        t1 = time.perf_counter()
        for o in outs:
            if o.finished:
                live.discard(o.request_id)
        steps += 1
        if steps > warm_steps:
            t_steps.append(t1 - t0)
            running.append(len(eng.scheduler.running))
            if t_end is None:
                t_end = t1 + seconds
            elif t1 > t_end:
                break
    for rid in list(live):
        eng.abort(rid)
    while eng.has_unfinished():
        eng.step()
    a = np.array(t_steps) * 1e3
    itl = float(np.mean(a))
    rmean = float(np.mean(running))
    return {"batch": R, "running_mean": round(rmean, 1), "itl_mean_ms": round(itl, 3),
            "itl_p50_ms": round(float(np.percentile(a, 50)), 3), "itl_p90_ms": round(float(np.percentile(a, 90)), 3),
            "rps": round(rmean / (osl * itl / 1e3), 2), "steps": len(a), "refused": refused}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="meta-llama/Llama-3.2-1B-Instruct")
    ap.add_argument("--isl", type=int, default=4000)
    ap.add_argument("--osl", type=int, default=500)
    ap.add_argument("--batches", default="256,384,512,640,768")
    ap.add_argument("--itl-ms", type=float, default=25.0)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--max-num-seqs", type=int, default=1024)
    ap.add_argument("--write", action="store_true")
    a = ap.parse_args()
    from mxserve.config import EngineArgs
    from mxserve.engine.engine import LLMEngine
    eng = LLMEngine(EngineArgs(model=a.model, device="cuda", max_num_seqs=a.max_num_seqs,
                               max_model_len=max(8192, a.isl + a.osl + 16), load_format="random",
                               disagg_mode="decode",
                               cuda_graph_max_bs=max(int(x) for x in a.batches.split(","))))
    # a synthetic fill of the whole pool: every reserved block holds finite, non-trivial values
    with torch.inference_mode():
        kv = eng.runner.kv_cache
        kv.view(-1)[:] = 0.01
    rows = []
    for i, r in enumerate(int(x) for x in a.batches.split(",")):
        row = run_batch(eng, r, a.isl, a.osl, a.seconds, seed=i)
        rows.append(row)
        print(json.dumps(row), flush=True)
    ok = [r for r in rows if r["itl_p90_ms"] <= a.itl_ms and not r["refused"]]
    cap = max((r["rps"] for r in ok), default=0.0)
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
        best = max(ok, key=lambda r: r["rps"])
        e.update({"decode_rps": cap, "decode_itl_target_ms": a.itl_ms, "decode_batch": best["batch"],
                  "decode_itl_p90_ms": best["itl_p90_ms"],
                  "decode_source": "scripts/decode_capacity_probe.py (measured, closed-loop batch sweep)"})
        with open(path, "w") as f:
            json.dump(d, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
