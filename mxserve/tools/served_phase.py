"""bench.py's served phase: the same open-loop Poisson stream as the engine-direct
headline, driven through the whole served stack on the same GPU.  The stack is the OpenAI frontend
(`python -m dynamo.frontend`: HTTP + SSE, router, multi-process), the worker with its streamer
process (`python -m dynamo.vllm`, started with the flags a manifest passes), and the engine.  The
client is the reference's benchmark path (/root/reference/run-benchmarks.sh:61-65 points
`benchmarks.utils.benchmark` at `--endpoint-url`).

It runs after the engine-direct phase has released the GPU, at the same QPS, ISL / OSL, engine
limits and temperature.  It also uses the same steady-state window: it is measured from the
engine-direct phase's warm-up length after the first arrival, for the engine-direct timed window's
length.  Output tokens are counted where they land at the client and spread over each request's first
and last token.  TTFT runs from each request's scheduled arrival to its first streamed token, so HTTP,
routing, the request plane and SSE are all inside.  ITL is reported two ways: the gap between
streamed chunks (itl_p50_ms) and each request's mean gap (t_last - t_first) / (tokens - 1)
(itl_req_p50_ms); the client runs in CLIENT_PROCS processes so it reads every stream on time.
"""
from __future__ import annotations

import asyncio
import os
import signal
import socket
import subprocess
import sys
import time
from typing import Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# load-generator processes (benchmarks/utils/benchmark.py run_rate): ~22k streamed tokens/s is more
# than one asyncio reader keeps up with, and a late reader shows up as bursty chunk gaps and TTFT
CLIENT_PROCS = int(os.environ.get("MXS_SERVED_CLIENT_PROCS", "2"))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stop(p: Optional[subprocess.Popen]) -> None:
    if p is None or p.poll() is not None:
        return
    try:
        os.killpg(p.pid, signal.SIGTERM)
        p.wait(timeout=20)
    except (ProcessLookupError, subprocess.TimeoutExpired):
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass


def _registered(url: str, model: str) -> bool:
    import json
    import urllib.request
    try:
        with urllib.request.urlopen(url + "/v1/models", timeout=2) as r:
            return any(m.get("id") == model for m in json.loads(r.read()).get("data", []))
    except (OSError, ValueError):
        return False


def _trace_breakdown(url: str, polls: int = 24, window: Optional[tuple] = None) -> dict:
    """Median per-stage times of the served requests' first tokens (those that arrived inside
    `window`, wall clock), from the frontend processes' trace rings (/debug/traces; each GET reaches one of the frontend processes, so several GETs cover
    them all): frontend spans from the request's arrival at the frontend (tokenized, dispatched: the
    submit POST to the worker's streamer starts, submitted: it returned, first_token) and the worker's spans carried on the first token (inbox: the engine thread's inbox,
    queue: waiting for admission, prefill: admission to the sampled token, delivery: worker emit to the
    frontend's receipt)."""
    import json
    import statistics
    import urllib.request
    seen: dict = {}
    for _ in range(polls):
        try:
            with urllib.request.urlopen(url + "/debug/traces?n=1024", timeout=5) as r:
                for t in json.loads(r.read()).get("traces", []):
                    tu = t.get("t_unix")
                    if window is None or (tu is not None and window[0] <= tu <= window[1]):
                        seen[t.get("request_id")] = t
        except (OSError, ValueError):
            break
    vals: dict = {}
    for t in seen.values():
        for k, v in (t.get("spans_ms") or {}).items():
            if k in ("tokenized", "routed", "dispatched", "submitted", "first_token"):
                vals.setdefault("frontend_" + k, []).append(v)
        for k, v in (t.get("worker_ms") or {}).items():
            if k in ("inbox_ms", "queue_ms", "prefill_ms", "delivery_ms") and isinstance(v, (int, float)):
                vals.setdefault("worker_" + k[:-3], []).append(v)
    out = {k: round(statistics.median(v), 3) for k, v in sorted(vals.items()) if v}
    if out:
        out["requests"] = len(seen)
    return out


def arrival_stream(qps: float, n: int, isl: int, vocab: int, rank: int = 0) -> tuple:
    """The engine-direct phase's exact Poisson stream (bench.py Driver, rank 0): the same generator
    draws the 65,536 inter-arrival gaps first, then each prompt in arrival order -- so both phases
    see the same arrival realisation (at the capacity point a few % more realised load is the
    difference between a flat and a growing queue)."""
    import numpy as np
    rng = np.random.default_rng(1234 + rank)
    gaps = rng.exponential(1.0 / qps, size=65536)
    prompts = [rng.integers(100, vocab - 100, size=isl, dtype=np.int64).tolist() for _ in range(n)]
    return gaps[:n], prompts


def run(model: str, qps: float, isl: int, osl: int, warmup_s: float, window_s: float, engine_flags: list,
        vocab: int, seed: int = 0, on_gpu: bool = True, deadline: Optional[float] = None, log_dir: str = "",
        children: Optional[list] = None) -> dict:
    """Start frontend + worker, stream the Poisson load, measure the steady window; stop both."""
    from benchmarks.utils.benchmark import run_rate
    t_setup = time.time()
    fe_port, w_port, s_port = _free_port(), _free_port(), _free_port()
    url = f"http://127.0.0.1:{fe_port}"
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
               HSA_ENABLE_IPC_MODE_LEGACY="0", MXS_STREAM_PORT=str(s_port))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
    out = open(os.path.join(log_dir, "served_frontend.log"), "w") if log_dir else subprocess.DEVNULL
    wout = open(os.path.join(log_dir, "served_worker.log"), "w") if log_dir else subprocess.DEVNULL
    fe = w = None
    try:
        fe = subprocess.Popen([sys.executable, "-m", "dynamo.frontend", "--http-port", str(fe_port), "--num-procs",
                               "4" if on_gpu else "1"], env=env, cwd=ROOT, stdout=out, stderr=subprocess.STDOUT,
                              start_new_session=True)
        w = subprocess.Popen([sys.executable, "-m", "dynamo.vllm", "--model", model, "--frontend-url", url,
                              "--host", "127.0.0.1", "--port", str(w_port), *engine_flags], env=env, cwd=ROOT,
                             stdout=wout, stderr=subprocess.STDOUT, start_new_session=True)
        if children is not None:
            children.extend([fe, w])
        while not _registered(url, model):
            if w.poll() is not None or fe.poll() is not None:
                return {"status": "failed", "error": f"served stack exited (worker {w.poll()}, frontend {fe.poll()})"}
            if deadline is not None and time.time() > deadline - (warmup_s + window_s + 30):
                return {"status": "skipped", "error": "no time left in the bench budget for the served phase"}
            time.sleep(0.5)
        setup_s = time.time() - t_setup
        n = int(qps * (warmup_s + window_s)) + 1
        gaps, prompts = arrival_stream(qps, n, isl, vocab, seed)
        w_url = f"http://127.0.0.1:{w_port}"
        marks: list = []

        clock: dict = {}

        async def main():
            # the worker engine's own counters at both ends of the steady window: engine iterations and
            # tokens generated inside it (separates the engine's rate from the client's view of it);
            # timed from the client's schedule origin (after its processes are up), like its window
            async def sample():
                import aiohttp
                t_wait = time.perf_counter() + 120
                while "t0" not in clock and time.perf_counter() < t_wait:
                    await asyncio.sleep(0.02)
                t0 = clock.get("t0", time.perf_counter())
                async with aiohttp.ClientSession() as sess:
                    for t in (warmup_s, warmup_s + window_s):
                        await asyncio.sleep(max(0.0, t0 + t - time.perf_counter()))
                        try:
                            async with sess.get(w_url + "/stats") as r:
                                st = await r.json()
                            marks.append((time.perf_counter(), st.get("num_steps", 0), st.get("num_generated", 0),
                                          st.get("num_running", 0), st.get("late_admission")))
                        except (aiohttp.ClientError, ValueError):
                            pass
            smp = asyncio.create_task(sample())
            res = await run_rate(url + "/v1/completions", model, qps, n, isl, osl, True, vocab, seed, warmup_s,
                                 gaps=gaps, prompts=prompts, procs=CLIENT_PROCS if on_gpu else 1, clock=clock)
            await smp
            return res
        t_run = time.time()
        s = asyncio.run(main())
        # the steady window's requests only (the trace rings also hold the ramp-up's, which see an
        # emptier engine), from the client's schedule origin
        t_run = clock.get("t0_unix", t_run)
        breakdown = _trace_breakdown(url, window=(t_run + warmup_s, t_run + warmup_s + window_s))
        res = {"status": "ok", "value": s.get("steady_output_tok_per_s"), "unit": "tok/s",
               "ttft_p50_ms": s.get("steady_ttft_ms_p50"), "ttft_p90_ms": s.get("steady_ttft_ms_p90"),
               "itl_p50_ms": s.get("steady_itl_ms_p50"), "itl_p90_ms": s.get("steady_itl_ms_p90"),
               "itl_req_p50_ms": s.get("steady_itl_req_ms_p50"), "itl_req_p90_ms": s.get("steady_itl_req_ms_p90"),
               "client_procs": s.get("client_procs"),
               "steady_window_s": s.get("steady_window_s"), "steady_requests": s.get("steady_requests"),
               "requests": s.get("requests"), "failed": s.get("failed"), "errors": s.get("errors"),
               "stack_start_s": round(setup_s, 1),
               "path": "client -> frontend (dynamo.frontend, 4 processes: HTTP/SSE, router) -> worker "
                       "(dynamo.vllm: streamer process + engine) on the same GPU"}
        if breakdown:
            res["ttft_breakdown_p50_ms"] = breakdown
        if len(marks) == 2:
            (ta, sa, ga, ra, _), (tb, sb, gb, rb, la) = marks
            res["worker_engine"] = {"tok_per_s": round((gb - ga) / (tb - ta), 1),
                                    "iteration_ms": round(1e3 * (tb - ta) / max(1, sb - sa), 3),
                                    "running_at_window_ends": [ra, rb], "late_admission": la}
        for k in ("value", "ttft_p50_ms", "ttft_p90_ms", "itl_p50_ms", "itl_p90_ms", "itl_req_p50_ms",
                  "itl_req_p90_ms", "steady_window_s"):
            if isinstance(res.get(k), float):
                res[k] = round(res[k], 3 if k != "value" else 2)
        return res
    finally:
        _stop(w)
        _stop(fe)
