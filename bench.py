#!/usr/bin/env python3
"""Headline benchmark: output tok/s (node) + p50 TTFT at a fixed QPS, Llama-3.2-1B-Instruct,
aggregated vs disaggregated serving (BASELINE.json metric / configs 2-3).

--mode agg (default): each rank (one per GPU, launched by torch.distributed.run) runs an
  independent engine replica -- the reference scales Llama-3.2-1B by `replicas:` of single-GPU
  workers behind the frontend router -- driven by an open-loop Poisson arrival
  process at --qps requests/s per GPU (weak scaling).
--mode disagg (N even): ranks [0, N/2) are prefill workers, ranks [N/2, N) decode workers, paired
  1P:1D (the reference's vllm/disagg.yaml graph).  Requests arrive at the decode rank (2 x --qps per
  pair, so the per-GPU rate matches agg); it reserves KV blocks and hands the prompt to its prefill
  rank, which computes it, pushes the blocks straight into the decode rank's pool with the IPC copy
  kernel (xGMI between GPUs; mxserve/disagg/kv_transfer.py) and returns the first token.  TTFT
  there includes the KV transfer.

Workload shape: ISL 4000 / OSL 500, the only request shape the reference quantifies
(examples/dgdr/trtllm/dgdr.yaml:22-26).  Prompts are synthetic random token ids and the weights are
random-init of the real architecture (no network on the GPU box); every request generates exactly
OSL tokens (ignore_eos).

A "step" is one engine iteration (continuous batching: decodes + chunked prefill under the token
budget) of a rank that owns requests (every rank in agg, the decode ranks in disagg).  W warmup
steps fill the pipeline; then exactly K steps are timed between a barrier + device sync on both
sides.  value = output tokens produced in the timed window summed over ranks / the slowest rank's
window.  TTFT is measured from each request's scheduled Poisson arrival (queueing included) for
requests whose first token lands in the window.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

BASELINE_METRIC = "output tok/s (node) + p50 TTFT at fixed QPS, Llama-3.2-1B agg vs disagg"
_VERBOSE = os.environ.get("MXS_BENCH_VERBOSE", "0") == "1"
_T0 = time.perf_counter()


if _VERBOSE:  # stacks of every thread once a minute: where a stalled rank is waiting
    import faulthandler
    faulthandler.dump_traceback_later(45, repeat=True)


def vlog(msg: str) -> None:
    if _VERBOSE:
        print(f"[bench r{os.environ.get('RANK', '0')} {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr,
              flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--warmup", type=int, default=1500)
    ap.add_argument("--mode", choices=["agg", "disagg"], default=os.environ.get("MXS_BENCH_MODE", "agg"))
    ap.add_argument("--model", default="meta-llama/Llama-3.2-1B-Instruct")
    ap.add_argument("--isl", type=int, default=4000)
    ap.add_argument("--osl", type=int, default=500)
    ap.add_argument("--qps", type=float, default=float(os.environ.get("MXS_BENCH_QPS", "42")),
                    help="Poisson arrival rate per GPU (requests/s)")
    ap.add_argument("--max-num-seqs", type=int, default=384)
    ap.add_argument("--max-num-batched-tokens", type=int, default=8192)
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--enforce-eager", action="store_true")
    ap.add_argument("--kv-cache-dtype", default=os.environ.get("MXS_BENCH_KV_DTYPE", "auto"),
                    help="auto (bf16, the headline) | fp8 (e4m3fn KV cache: a separate, labelled data point)")
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--max-warmup-s", type=float, default=120.0,
                    help="cap on the extra warmup that waits for the first finished request")
    return ap.parse_args()


class Driver:
    """Open-loop Poisson load on one request-owning rank + latency bookkeeping."""

    def __init__(self, a, rank: int, vocab: int, qps: float):
        rng = np.random.default_rng(1234 + rank)
        self.horizon = 4096
        self.arrivals = np.cumsum(rng.exponential(1.0 / qps, size=self.horizon))
        self.prompts = rng.integers(100, vocab - 100, size=(self.horizon, a.isl), dtype=np.int64)
        self.rank = rank
        self.nxt = 0
        self.t_start = 0.0
        self.arrival_of: dict = {}
        self.first_tok: dict = {}
        self.last_tok: dict = {}
        self.itls: list = []
        self.record = False
        self.finished = 0
        self.warmup_steps = 0
        self.c = {"ttft": [], "tokens": 0}

    def due(self) -> list:
        """(request_id, prompt) for every arrival whose time has come."""
        out = []
        now_rel = time.perf_counter() - self.t_start
        while self.nxt < self.horizon and self.arrivals[self.nxt] <= now_rel:
            rid = f"r{self.rank}-{self.nxt}"
            self.arrival_of[rid] = self.t_start + self.arrivals[self.nxt]
            out.append((rid, self.prompts[self.nxt].tolist()))
            self.nxt += 1
        return out

    def wait_next(self) -> None:
        if self.nxt < self.horizon:
            time.sleep(max(0.0, self.t_start + self.arrivals[self.nxt] - time.perf_counter()))

    def token(self, rid: str, now: float, finished: bool = False) -> None:
        self.finished += finished
        if rid not in self.first_tok:
            self.first_tok[rid] = now
            if self.record:
                self.c["ttft"].append(now - self.arrival_of[rid])
        elif self.record:
            self.itls.append(now - self.last_tok[rid])
        self.last_tok[rid] = now
        if self.record:
            self.c["tokens"] += 1

    def stats(self, dt: float) -> list:
        ttft = np.array(self.c["ttft"]) if self.c["ttft"] else np.array([np.nan])
        itl = np.array(self.itls) if self.itls else np.array([np.nan])
        return [dt, float(self.c["tokens"]), float(np.nanmedian(ttft)), float(np.nanmedian(itl)),
                float(len(self.c["ttft"])), float(self.warmup_steps)]


def timed_phases(a, step, barrier, drv, on_phase=lambda phase: None) -> float:
    """W untimed steps, then exactly K steps between barrier + device sync; returns the window."""
    on_phase("warmup")
    barrier()
    vlog("warmup")
    drv.t_start = time.perf_counter()
    i = 0
    while i < a.warmup or (drv.finished == 0 and time.perf_counter() - drv.t_start < a.max_warmup_s):
        step()
        if i % 200 == 0:
            vlog(f"warmup step {i}: {drv.nxt} arrivals, {len(drv.first_tok)} first tokens")
        i += 1
    drv.warmup_steps = i
    on_phase("timed")
    barrier()
    vlog("timed")
    drv.record = True
    t0 = time.perf_counter()
    for i in range(a.steps):
        step()
        if i % 200 == 0:
            vlog(f"timed step {i}: {drv.c['tokens']} tokens")
    on_phase("stop")
    barrier()
    vlog("done")
    return time.perf_counter() - t0


def run_agg(a, eng, sp, drv, barrier) -> float:
    def step():
        for rid, toks in drv.due():
            eng.add_request(toks, sp, request_id=rid)
        if not eng.has_unfinished():  # idle: wait for the next arrival
            drv.wait_next()
            for rid, toks in drv.due():
                eng.add_request(toks, sp, request_id=rid)
        t0 = time.perf_counter()
        outs = eng.step()
        now = time.perf_counter()
        for o in outs:
            drv.token(o.request_id, now, o.finished)
        if eng.step_times is not None:
            eng.step_times["engine_step"] = eng.step_times.get("engine_step", 0.0) + now - t0
            eng.step_times["loop"] = eng.step_times.get("loop", 0.0) + time.perf_counter() - t_loop[0]
        t_loop[0] = time.perf_counter()

    t_loop = [time.perf_counter()]
    return timed_phases(a, step, barrier, drv)


def _pair_conn(rank: int, world: int, is_decode: bool):
    """Host control channel between a prefill rank and its decode rank (same node)."""
    from multiprocessing.connection import Client, Listener
    half = world // 2
    pair = rank - half if is_decode else rank
    port = int(os.environ.get("MASTER_PORT", "29500")) + 101 + pair
    if is_decode:
        lst = Listener(("127.0.0.1", port), authkey=b"mxs-bench")
        conn = lst.accept()
        lst.close()
        return conn
    for _ in range(1200):
        try:
            return Client(("127.0.0.1", port), authkey=b"mxs-bench")
        except OSError:
            time.sleep(0.1)
    raise RuntimeError("could not reach the decode rank")


def run_disagg_decode(a, eng, sp, drv, barrier, conn) -> float:
    from mxserve.disagg.kv_transfer import KVTransferAgent
    agent = KVTransferAgent(eng.runner, "xgmi")
    conn.send(("desc", agent.descriptor()))
    # the prefill rank maps the pool now, while this rank idles in a plain socket wait
    ack = conn.recv()
    assert ack[0] == "mapped", ack
    vlog("decode pool mapped by the prefill rank")
    bs = eng.args.block_size
    backlog: list = []
    inflight: dict = {}

    def step():
        backlog.extend(drv.due())
        if not eng.has_unfinished() and not backlog and not inflight:
            drv.wait_next()
            backlog.extend(drv.due())
        while backlog:
            rid, toks = backlog[0]
            req = eng.reserve_remote_prefill(toks, sp, rid)
            if req is None:  # decode pool full: retry next step
                break
            backlog.pop(0)
            skip = req.num_cached_tokens // bs
            dst = list(req.block_ids[skip:-(-len(toks) // bs)])
            start = agent.acquire(len(dst))  # None: host-staged transfer for this request
            conn.send(("prefill", rid, toks, dst, skip, start))
            inflight[rid] = (dst, start)
        now = time.perf_counter()
        while conn.poll():
            _, rid, tok, data = conn.recv()
            dst, start = inflight.pop(rid)
            if start is not None:  # staging extent -> pool blocks, ordered before the next step
                agent.land(start, dst)
            elif data is not None:  # host-staged transfer (CPU plumbing runs)
                agent.write_blocks(dst, data)
            eng.complete_remote_prefill(rid, tok)
            drv.token(rid, now)
        if eng.has_unfinished():
            outs = eng.step()
            now = time.perf_counter()
            for o in outs:
                drv.token(o.request_id, now, o.finished)
        elif inflight:  # nothing to decode yet: block until a prefill lands (or an arrival is due)
            conn.poll(0.05)

    return timed_phases(a, step, barrier, drv, on_phase=lambda ph: conn.send(("phase", ph)))


def run_disagg_prefill(eng, temperature: float, barrier, conn) -> int:
    """Serve the paired decode rank until it says stop, joining its barriers; returns blocks moved."""
    from mxserve.disagg.kv_transfer import KVTransferAgent
    from mxserve.engine.request import SamplingParams
    agent = KVTransferAgent(eng.runner, "xgmi")
    kind, target = conn.recv()
    assert kind == "desc", kind
    if agent.backend == "xgmi" and target["backend"] == "xgmi":
        agent.connect(target)
    conn.send(("mapped",))
    vlog(f"prefill rank serving (decode pool backend {target['backend']})")
    pending: dict = {}
    moved = 0
    while True:
        stop = False
        while conn.poll():
            msg = conn.recv()
            if msg[0] == "phase":
                vlog(f"phase {msg[1]}; {moved} blocks pushed so far")
                barrier()
                stop = msg[1] == "stop"
                continue
            _, rid, toks, dst, skip, start = msg
            eng.add_request(toks, SamplingParams(max_tokens=1, temperature=temperature, ignore_eos=True),
                            request_id=rid, disagg_role="prefill_only")
            vlog(f"prefill {rid}: {len(toks)} tokens -> {len(dst)} blocks")
            pending[rid] = (dst, skip, start)
        if stop:
            return moved
        if not eng.has_unfinished():
            time.sleep(0.0002)
            continue
        for o in eng.step():
            if not o.finished or o.request_id not in pending:
                continue
            dst, skip, start = pending.pop(o.request_id)
            src = list(eng.requests[o.request_id].block_ids[skip:skip + len(dst)])
            data = None
            if start is not None:
                secs = agent.push_xgmi(src, target, start)
                vlog(f"pushed {o.request_id}: {len(src)} blocks in {secs * 1e3:.2f} ms")
            else:
                data = agent.read_blocks(src)
            moved += len(src)
            eng.release_prefill_blocks(o.request_id)
            conn.send(("done", o.request_id, o.token_id, data))


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    on_gpu = torch.cuda.is_available() and a.device != "cpu"
    disagg = a.mode == "disagg"
    if disagg and (world < 2 or world % 2):
        raise SystemExit("--mode disagg needs an even number of ranks (1 prefill : 1 decode pairs)")
    if on_gpu:
        torch.cuda.set_device(local % torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # disagg ranks exchange only host messages + barriers (and may share a GPU in functional runs)
        dist.init_process_group("nccl" if on_gpu and not disagg else "gloo")

    from mxserve.config import EngineArgs
    from mxserve.engine.engine import LLMEngine
    from mxserve.engine.request import SamplingParams

    args = EngineArgs(model=a.model, device="cuda" if on_gpu else "cpu", max_num_seqs=a.max_num_seqs,
                      cuda_graph_max_bs=a.max_num_seqs,
                      max_num_batched_tokens=a.max_num_batched_tokens, max_model_len=a.max_model_len,
                      enforce_eager=a.enforce_eager, seed=a.seed, kv_cache_dtype=a.kv_cache_dtype)
    if not on_gpu:  # plumbing run only (CPU container): keep it tiny
        args = args.replace(model="tiny-llama", max_model_len=1024, cpu_num_blocks=4096)
        a.isl, a.osl = min(a.isl, 200), min(a.osl, 20)
    is_prefill = disagg and rank < world // 2
    if disagg:
        args = args.replace(disagg_mode="prefill" if is_prefill else "decode")
        if on_gpu and torch.cuda.device_count() < world:  # functional run: ranks share a GPU
            args = args.replace(num_gpu_blocks=int(os.environ.get("MXS_BENCH_SHARED_BLOCKS", "40000")))
    vlog("building engine")
    eng = LLMEngine(args)
    vlog(f"engine ready ({eng.runner.num_blocks} KV blocks)")
    sp = SamplingParams(max_tokens=a.osl, temperature=a.temperature, ignore_eos=True)

    sync = torch.cuda.synchronize if on_gpu else (lambda: None)

    def barrier():
        if world > 1:
            dist.barrier()
        sync()

    if not disagg:
        drv = Driver(a, rank, eng.model_config.vocab_size, a.qps)
        local_stats = drv.stats(run_agg(a, eng, sp, drv, barrier))
    else:
        conn = _pair_conn(rank, world, not is_prefill)
        vlog("paired")
        if is_prefill:
            run_disagg_prefill(eng, a.temperature, barrier, conn)
            local_stats = [0.0, 0.0, float("nan"), float("nan"), 0.0, float("nan")]
        else:
            drv = Driver(a, rank, eng.model_config.vocab_size, 2 * a.qps)
            local_stats = drv.stats(run_disagg_decode(a, eng, sp, drv, barrier, conn))
        conn.close()

    local_stats = torch.tensor(local_stats, dtype=torch.float64)
    if world > 1:
        gathered = [torch.zeros_like(local_stats) for _ in range(world)]
        dist.all_gather_object(gathered, local_stats)
        allst = torch.stack(gathered)
    else:
        allst = local_stats.unsqueeze(0)
    if rank == 0:
        col = allst.numpy()
        t_max = float(col[:, 0].max())
        value = float(col[:, 1].sum()) / t_max

        def med(c):
            v = col[:, c][~np.isnan(col[:, c])]
            return float(np.median(v)) * 1e3 if len(v) else None

        ttft_p50, itl_p50 = med(2), med(3)
        st = eng.stats()
        line = {
            "metric": BASELINE_METRIC,
            "value": round(value, 2),
            "unit": "tok/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "warmup_steps_executed": int(np.nanmax(col[:, 5])),
            "ms_per_step": round(t_max / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if on_gpu else "fp32",
            "data": "synthetic (random prompt token ids, random-init weights, Poisson arrivals)",
            "config": {"model": args.model if on_gpu else "tiny-llama (CPU plumbing run)",
                       "global_batch": int(world * a.max_num_seqs), "seq_len": a.isl + a.osl,
                       "parallelism": f"disagg {world // 2}P+{world // 2}D" if disagg else f"dp{world}",
                       "mode": a.mode, "isl": a.isl, "osl": a.osl,
                       "qps_per_gpu": a.qps, "qps_node": a.qps * world,
                       "kv_cache_dtype": "fp8_e4m3fn" if eng.runner.kv_fp8 else ("bf16" if on_gpu else "fp32")},
            "ttft_p50_ms": None if ttft_p50 is None else round(ttft_p50, 2),
            "itl_p50_ms": None if itl_p50 is None else round(itl_p50, 3),
            "requests_with_first_token": int(col[:, 4].sum()),
            "sla_isl4000_osl500": {"ttft_ms<=600": ttft_p50 is not None and ttft_p50 <= 600,
                                   "itl_ms<=25": itl_p50 is not None and itl_p50 <= 25},
            "engine": {"kv_blocks": st["num_blocks"], "running_at_end": st["num_running"],
                       "waiting_at_end": st["num_waiting"], "preemptions": st["num_preemptions"],
                       "graphs": sorted(eng.runner.graphs) if on_gpu else []},
        }
        print(json.dumps(line), flush=True)
        if eng.step_times is not None and eng.step_times["steps"]:
            n = eng.step_times["steps"]
            print(json.dumps({"host_ms_per_step": {k: round(v / n * 1e3, 4) for k, v in eng.step_times.items()
                                                   if k != "steps"}, "steps": n}), file=sys.stderr, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
