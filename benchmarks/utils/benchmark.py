"""Load generator for an OpenAI-compatible endpoint.

    python3 -m benchmarks.utils.benchmark --benchmark-name NAME --endpoint-url URL --model M \
        --output-dir DIR [--isl 4000 --osl 500] [--concurrency 1,2,4,...] [--request-rate 8,16,...]

For each concurrency level (closed loop) and each request rate (open loop, Poisson arrivals) it
streams /v1/completions requests with synthetic prompts of ~ISL tokens and exactly OSL output
tokens (ignore_eos), and records TTFT (first streamed token), ITL (gaps between streamed chunks),
end-to-end latency and throughput.  One JSON file per point under DIR/NAME/, plus summary.json.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import time
from typing import Optional

import aiohttp
import numpy as np

WORDS = ("alpha bravo charlie delta echo foxtrot golf hotel india juliet kilo lima mike november oscar papa "
         "quebec romeo sierra tango uniform victor whiskey xray yankee zulu").split()


def synth_prompt(rng: random.Random, isl: int, token_ids: bool, vocab: int):
    if token_ids:
        return [rng.randrange(100, vocab - 100) for _ in range(isl)]
    # ~1 token per word for BPE tokenizers; byte tokenizers see more
    return " ".join(rng.choice(WORDS) for _ in range(isl))


async def one_request(sess, url: str, model: str, prompt, osl: int, t_sched: float) -> dict:
    body = {"model": model, "prompt": prompt, "max_tokens": osl, "ignore_eos": True, "stream": True,
            "temperature": 1.0, "stream_options": {"include_usage": True}}
    t0 = max(time.perf_counter(), t_sched)
    first, last, gaps, n_chunks, usage, err = None, None, [], 0, None, None
    try:
        async with sess.post(url, json=body) as r:
            if r.status != 200:
                return {"ok": False, "error": f"HTTP {r.status}: {(await r.text())[:200]}"}
            async for raw in r.content:
                line = raw.decode().strip()
                if not line.startswith("data: "):
                    continue
                data = line[6:]
                if data == "[DONE]":
                    break
                ch = json.loads(data)
                if "error" in ch:
                    err = ch["error"].get("message")
                    break
                if ch.get("usage"):
                    usage = ch["usage"]
                if ch.get("choices"):
                    now = time.perf_counter()
                    if first is None:
                        first = now
                    else:
                        gaps.append(now - last)
                    last = now
                    n_chunks += 1
    except (aiohttp.ClientError, asyncio.TimeoutError) as e:
        return {"ok": False, "error": repr(e)}
    if err or first is None:
        return {"ok": False, "error": err or "no tokens"}
    out_tokens = usage["completion_tokens"] if usage else n_chunks
    # per-request ITL: the mean gap over the request's own tokens, (last - first) / (tokens - 1).  It
    # does not depend on how chunks were grouped on the way (a reader that falls behind sees several
    # chunks back to back: small chunk gaps, then one large one)
    itl_req = (last - first) / (out_tokens - 1) if out_tokens > 1 else None
    return {"ok": True, "ttft": first - t_sched, "e2e": last - t_sched, "itl": gaps, "out": out_tokens, "chunks": n_chunks,
            "in": usage["prompt_tokens"] if usage else None, "start": t0, "sched": t_sched, "first": first,
            "last": last, "itl_req": itl_req}


def steady_window(results: list, t_a: float, t_b: float) -> dict:
    """Open-loop steady state: output tokens emitted inside [t_a, t_b] (each request's tokens spread
    evenly over [first token, last token]) and TTFT of requests scheduled inside it -- the ramp-up
    before t_a and the drain after the last arrival are excluded, as in bench.py's timed window."""
    ok = [r for r in results if r["ok"]]
    toks = 0.0
    for r in ok:
        if r.get("chunks") == r["out"]:  # one token per streamed chunk: count the chunks that landed inside
            t = r["first"]
            toks += t_a <= t <= t_b
            for g in r["itl"]:
                t += g
                toks += t_a <= t <= t_b
            continue
        lo, hi = max(r["first"], t_a), min(r["last"], t_b)  # chunks carrying several tokens: spread them
        if hi <= lo:
            continue
        span = max(r["last"] - r["first"], 1e-9)
        toks += (r["out"] - 1) * (hi - lo) / span + (1 if t_a <= r["first"] <= t_b else 0)
    ttft = [r["ttft"] for r in ok if t_a <= r["sched"] <= t_b]
    itl = [g for r in ok if t_a <= r["sched"] <= t_b for g in r["itl"]]
    itl_req = [r["itl_req"] for r in ok if t_a <= r["sched"] <= t_b and r.get("itl_req") is not None]
    pct = lambda xs, q: float(np.percentile(xs, q)) * 1e3 if xs else None  # noqa: E731
    return {"steady_window_s": t_b - t_a, "steady_output_tok_per_s": toks / max(t_b - t_a, 1e-9),
            "steady_requests": len(ttft), "steady_ttft_ms_p50": pct(ttft, 50), "steady_ttft_ms_p90": pct(ttft, 90),
            "steady_itl_ms_p50": pct(itl, 50), "steady_itl_ms_p90": pct(itl, 90),
            "steady_itl_req_ms_p50": pct(itl_req, 50), "steady_itl_req_ms_p90": pct(itl_req, 90)}


def summarize(results: list, wall: float, label: dict) -> dict:
    ok = [r for r in results if r["ok"]]
    def pct(xs, q):
        return float(np.percentile(xs, q)) * 1e3 if xs else None
    ttft = [r["ttft"] for r in ok]
    itl = [g for r in ok for g in r["itl"]]
    itl_req = [r["itl_req"] for r in ok if r.get("itl_req") is not None]
    e2e = [r["e2e"] for r in ok]
    out = sum(r["out"] for r in ok)
    return dict(label, requests=len(results), failed=len(results) - len(ok), duration_s=wall,
                output_tok_per_s=out / wall if wall > 0 else 0.0, requests_per_s=len(ok) / wall if wall > 0 else 0.0,
                ttft_ms_p50=pct(ttft, 50), ttft_ms_p90=pct(ttft, 90), ttft_ms_p99=pct(ttft, 99),
                itl_ms_p50=pct(itl, 50), itl_ms_p90=pct(itl, 90), itl_ms_p99=pct(itl, 99),
                itl_req_ms_p50=pct(itl_req, 50), itl_req_ms_p90=pct(itl_req, 90),
                e2e_ms_p50=pct(e2e, 50), errors=[r["error"] for r in results if not r["ok"]][:5])


async def run_concurrency(url, model, conc, n, isl, osl, token_ids, vocab, seed):
    rng = random.Random(seed)
    prompts = [synth_prompt(rng, isl, token_ids, vocab) for _ in range(n)]
    results = []
    it = iter(prompts)
    conn = aiohttp.TCPConnector(limit=0)
    async with aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(total=None)) as sess:
        t0 = time.perf_counter()

        async def worker():
            for p in it:
                results.append(await one_request(sess, url, model, p, osl, time.perf_counter()))
        await asyncio.gather(*(worker() for _ in range(conc)))
        wall = time.perf_counter() - t0
    return summarize(results, wall, {"mode": "concurrency", "concurrency": conc, "isl": isl, "osl": osl})


async def _fire(url, model, osl, sched, prompts) -> list:
    """Send each prompt at its absolute perf_counter time in `sched`; the results in order."""
    conn = aiohttp.TCPConnector(limit=0)
    async with aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(total=None)) as sess:
        tasks = []
        for t, p in zip(sched, prompts):
            await asyncio.sleep(max(0.0, t - time.perf_counter()))
            tasks.append(asyncio.create_task(one_request(sess, url, model, p, osl, t)))
        return list(await asyncio.gather(*tasks))


def _fire_shard(args) -> list:  # a client process (spawned: imports nothing of the caller's GPU state)
    return asyncio.run(_fire(*args))


def _ready(_i: int = 0) -> float:
    return time.perf_counter()


def client_procs() -> int:
    """Client processes for open-loop points (BENCH_CLIENT_PROCS).  At ~20k streamed tokens/s one
    asyncio process reads its sockets late and in bursts -- its chunk gaps and first-token times then
    measure the client, not the server -- so the served bench spreads the streams over several."""
    return max(1, int(os.environ.get("BENCH_CLIENT_PROCS", "1")))


async def run_rate(url, model, rate, n, isl, osl, token_ids, vocab, seed, warmup_s: float = 0.0, gaps=None,
                   prompts=None, procs: int = 0, clock: Optional[dict] = None):
    """Open-loop Poisson arrivals.  gaps / prompts: an explicit arrival stream (bench.py's served
    phase replays the engine-direct phase's exact stream) instead of one drawn from `seed`.
    procs > 1: request i is sent by client process i % procs at the same absolute schedule
    (perf_counter is CLOCK_MONOTONIC, one clock for every process on the host).  clock: filled with the
    schedule's origin once it is fixed ("t0": perf_counter, "t0_unix": wall clock), so a caller can
    align its own measurements with the steady window (t0 + warmup_s)."""
    if prompts is None:
        rng = random.Random(seed)
        prompts = [synth_prompt(rng, isl, token_ids, vocab) for _ in range(n)]
    if gaps is None:
        gaps = np.random.default_rng(seed).exponential(1.0 / rate, size=n)
    procs = procs or client_procs()
    prompts = list(prompts)[:len(gaps)]
    def mark(t0: float) -> None:
        if clock is not None:
            clock["t0"], clock["t0_unix"] = t0, time.time() + (t0 - time.perf_counter())
    if procs <= 1:
        t0 = time.perf_counter()
        mark(t0)
        sched = (t0 + np.cumsum(np.asarray(gaps[:len(prompts)], dtype=np.float64))).tolist()
        results = await _fire(url, model, osl, sched, prompts)
    else:
        import concurrent.futures
        import multiprocessing
        with concurrent.futures.ProcessPoolExecutor(procs, mp_context=multiprocessing.get_context("spawn")) as ex:
            list(ex.map(_ready, range(procs)))  # every client process up (imports done) before t0
            loop = asyncio.get_running_loop()
            t0 = time.perf_counter() + 0.2
            mark(t0)
            sched = (t0 + np.cumsum(np.asarray(gaps[:len(prompts)], dtype=np.float64))).tolist()
            futs = [loop.run_in_executor(ex, _fire_shard, (url, model, osl, sched[k::procs], prompts[k::procs]))
                    for k in range(procs)]
            shards = await asyncio.gather(*futs)
        results = [None] * len(prompts)
        for k, sh in enumerate(shards):
            results[k::procs] = sh
    t_arrivals_end = sched[-1] if sched else t0
    wall = max([r["last"] for r in results if r.get("ok")] + [time.perf_counter() if procs <= 1 else t0]) - t0
    s = summarize(list(results), wall, {"mode": "request_rate", "request_rate": rate, "isl": isl, "osl": osl,
                                        "client_procs": procs})
    if warmup_s > 0 and t0 + warmup_s < t_arrivals_end:
        s.update(steady_window(list(results), t0 + warmup_s, t_arrivals_end))
    return s


def _endpoint(url: str) -> str:
    u = url.rstrip("/")
    if u.endswith("/v1/completions"):
        return u
    if u.endswith("/v1/chat/completions"):
        return u[: -len("/chat/completions")] + "/completions"
    if u.endswith("/v1"):
        return u + "/completions"
    return u + "/v1/completions"


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(prog="python3 -m benchmarks.utils.benchmark")
    ap.add_argument("--benchmark-name", required=True)
    ap.add_argument("--endpoint-url", required=True)
    ap.add_argument("--model", required=True)
    ap.add_argument("--output-dir", required=True)
    ap.add_argument("--isl", type=int, default=int(os.environ.get("BENCH_ISL", "4000")))
    ap.add_argument("--osl", type=int, default=int(os.environ.get("BENCH_OSL", "500")))
    ap.add_argument("--concurrency", default=os.environ.get("BENCH_CONCURRENCY", "1,2,4,8,16,32,64"))
    ap.add_argument("--request-rate", default=os.environ.get("BENCH_REQUEST_RATE", ""))
    ap.add_argument("--num-requests", type=int, default=0, help="per point (default max(4*conc, 16))")
    ap.add_argument("--token-ids", action="store_true", help="send prompts as token-id lists (exact ISL)")
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--warmup-s", type=float, default=float(os.environ.get("BENCH_WARMUP_S", "0")),
                    help="request-rate points: also report steady-state numbers from this many seconds after "
                         "the first arrival to the last one (ramp-up and drain excluded)")
    a = ap.parse_args(argv)
    url = _endpoint(a.endpoint_url)
    out_dir = os.path.join(a.output_dir, a.benchmark_name)
    os.makedirs(out_dir, exist_ok=True)
    points = []
    for c in [int(x) for x in a.concurrency.split(",") if x.strip()]:
        n = a.num_requests or max(4 * c, 16)
        s = asyncio.run(run_concurrency(url, a.model, c, n, a.isl, a.osl, a.token_ids, a.vocab, a.seed + c))
        points.append(s)
        with open(os.path.join(out_dir, f"concurrency_{c}.json"), "w") as f:
            json.dump(s, f, indent=2)
        print(json.dumps({k: v for k, v in s.items() if k != "errors"}), flush=True)
    for r in [float(x) for x in a.request_rate.split(",") if x.strip()]:
        n = a.num_requests or max(int(r * 30), 16)
        s = asyncio.run(run_rate(url, a.model, r, n, a.isl, a.osl, a.token_ids, a.vocab, a.seed + int(r * 100),
                                 a.warmup_s))
        points.append(s)
        with open(os.path.join(out_dir, f"rate_{r:g}.json"), "w") as f:
            json.dump(s, f, indent=2)
        print(json.dumps({k: v for k, v in s.items() if k != "errors"}), flush=True)
    with open(os.path.join(out_dir, "summary.json"), "w") as f:
        json.dump({"benchmark": a.benchmark_name, "endpoint": url, "model": a.model, "points": points}, f, indent=2)


if __name__ == "__main__":
    main()
