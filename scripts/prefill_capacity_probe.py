#!/usr/bin/env python3
"""Prefill-only capacity of one MI355X for the headline workload (Llama-3.2-1B, 4000-token prompts,
1 output token): the rate a disaggregated prefill GPU sustains, for bench.py's P:D split."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from mxserve.config import EngineArgs
    from mxserve.engine.engine import LLMEngine
    from mxserve.engine.request import SamplingParams
    mnbt = int(os.environ.get("MNBT", "8192"))
    eng = LLMEngine(EngineArgs(model="meta-llama/Llama-3.2-1B-Instruct", device="cuda", max_num_seqs=64,
                               max_num_batched_tokens=mnbt, max_model_len=max(8192, mnbt), load_format="random",
                               enforce_eager=os.environ.get("EAGER", "1") == "1"))
    rng = np.random.default_rng(0)
    sp = SamplingParams(max_tokens=int(os.environ.get("OSL", "1")), temperature=0, ignore_eos=True)
    for n in (32,) + (256,) * int(os.environ.get("ROUNDS", "1")):  # warm-up round, then measured ones
        for i in range(n):
            eng.add_request(rng.integers(100, 120000, size=4000).tolist(), sp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        slow = []
        while eng.has_unfinished():
            before = dict(eng.step_times) if eng.step_times is not None else None
            ts = time.perf_counter()
            eng.step()
            w = time.perf_counter() - ts
            if w > float(os.environ.get("SLOW_S", "0.08")):  # a stalled step: which host phase took the time
                slow.append({"step": eng.num_steps, "wall_ms": round(w * 1e3, 1),
                             **({k: round((eng.step_times[k] - before[k]) * 1e3, 1) for k in before
                                 if k != "steps"} if before else {})})
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if True:
            print(json.dumps({"n": n, "round_s": round(dt, 3), "slow_steps": slow}), flush=True)
        if n == 32 and eng.step_times is not None:
            eng.step_times.update({k: 0.0 for k in eng.step_times})
    print(json.dumps({"max_num_batched_tokens": mnbt, "prompts": 256, "isl": 4000, "seconds": round(dt, 3), "req_per_s": round(256 / dt, 1),
                      "prefill_tok_per_s": round(256 * 4000 / dt), "slow_steps": slow,
                      "host_ms_per_step": ({k: round(v / max(1, eng.step_times["steps"]) * 1e3, 3)
                                            for k, v in eng.step_times.items() if k != "steps"}
                                           if eng.step_times else None)}), flush=True)


if __name__ == "__main__":
    main()
