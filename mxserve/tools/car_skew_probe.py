"""Arrival skew of the ranks at their first custom all-reduce, with and without the arming barrier
(diagnosis of the round-4 driver failure: GPUTEST_r04.json, tests/test_c_tp8_gpu.py).

Runs the exact start-up of test_c_tp8_gpu's 70B TP-8 ranks (8 processes sharing GPU 0: gloo group,
custom all-reduce, per-rank random 70B@layers=2 state generated on the GPU, model build, one 40-token
forward) with a 60 s wait budget, so nothing times out, then reads every rank's device timestamp of
its first collective (custom_allreduce.hip kSigFirst; one GPU = one clock) and each rank's host time
at its first collective.  MXS_CAR_ARM=0 skips the synchronize + barrier in CustomAllReduce._arm.

  python -m mxserve.tools.car_skew_probe [--world 8] [--arm 0|1] [--out path.json]
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import socket
import sys
import time
import traceback


def _rank(rank, world, port, q, arm):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          MXS_CAR_ARM=str(arm), MXS_CAR_TIMEOUT_MS="60000")
        import torch
        torch.cuda.set_device(0)
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
        from mxserve.models.config import get_model_config
        from mxserve.models.llama import build_model
        from mxserve.models.weights import random_full_state
        from mxserve.parallel import comm
        from tests.test_c_tp8_gpu import _md
        t_start = time.time()
        st = comm.init_distributed(world, backend="gloo", device=torch.device("cuda:0"))
        t_init = time.time()
        cfg = get_model_config("meta-llama/Meta-Llama-3-70B-Instruct@layers=2")
        full = random_full_state(cfg, seed=4, std=0.02, dtype=torch.bfloat16, device="cuda:0")
        m = build_model(cfg, torch.device("cuda:0"), torch.bfloat16, "allreduce")
        m.load_full_state(full)
        n = 40
        ids = torch.randint(3, cfg.vocab_size, (n,), generator=torch.Generator().manual_seed(2)).to("cuda:0")
        kv = torch.zeros(4, cfg.num_layers, 2, m.nkv, 16, cfg.head_dim, dtype=torch.bfloat16, device="cuda:0")
        t_fwd = time.time()
        with torch.inference_mode():
            m.compute_logits(m.forward(ids, _md(n, "cuda:0"), kv))
        torch.cuda.synchronize()
        car = st.custom_ar
        healthy = car.check()
        diag = car.diagnose() if rank == 0 else None
        torch.distributed.barrier()
        q.put((rank, {"t_start": t_start, "t_init_done": t_init, "t_forward_enqueue": t_fwd,
                      "t_first_collective_host": car.first_host_time, "healthy": healthy}, diag, None))
    except BaseException:  # noqa: BLE001
        q.put((rank, None, None, traceback.format_exc()))


def run(world: int, arm: int) -> dict:
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q, arm)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, host, diag, err = q.get(timeout=400)
            res[r] = (host, diag, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = {r: v[2] for r, v in res.items() if v[2]}
    if errs:
        return {"arm": arm, "errors": errs}
    hosts = {r: v[0] for r, v in res.items()}
    t0 = min(h["t_first_collective_host"] for h in hosts.values())
    f0 = min(h["t_forward_enqueue"] for h in hosts.values())
    diag = res[0][1]
    return {"arm": arm, "world": world,
            "device_first_collective_skew_ms": {d["rank"]: round(d.get("first_collective_skew_ms", float("nan")), 3)
                                                for d in diag},
            "host_first_collective_skew_ms": {r: round(1e3 * (h["t_first_collective_host"] - t0), 3)
                                              for r, h in sorted(hosts.items())},
            "host_forward_enqueue_skew_ms": {r: round(1e3 * (h["t_forward_enqueue"] - f0), 3)
                                             for r, h in sorted(hosts.items())},
            "healthy": all(h["healthy"] for h in hosts.values()), "error_words": [d["err"] for d in diag]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--arm", type=int, default=None, help="1 / 0; default: both")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    out = [run(a.world, arm) for arm in ([a.arm] if a.arm is not None else [0, 1])]
    txt = json.dumps(out, indent=1)
    print(txt, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
