#!/usr/bin/env python3
"""Frontend load test without a GPU: synthetic token-emitting workers
behind the real multi-process frontend, driven by lean open-loop streaming clients.

  fake workers  W processes, each one "GPU": the worker's mux request plane (POST /mux, /submit,
                /abort; worker/server.py) on mxserve's own HTTP server, one NDJSON line per 10 ms
                "engine step" carrying a token of every running request; the FIRST token is written
                at /submit time, so a client's TTFT is exactly what the serving path adds
                (HTTP parse, route, the submit round trip, delivery, SSE)
  frontend      `python -m mxserve.frontend --num-procs P` (httpd + push fast path)
  clients       C processes, Poisson arrivals, raw-socket HTTP/1.1 streaming /v1/completions
                (token-id prompts, ISL 100, OSL 500), counting SSE chunks and stamping arrivals

Prints one JSON line: delivered tokens/s, requests completed / dropped, client TTFT p50 / p90 (the
added latency), inter-chunk gap p50 / p90 (10 ms if nothing queues), frontend CPU per 1k tokens.

  python scripts/frontend_load.py --tok-per-s 170000 --workers 8 --procs 4 --clients 4 --duration 20
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MODEL = "meta-llama/Llama-3.2-1B-Instruct"


# ---------------------------------------------------------------------------- fake worker
def fake_worker(port: int, frontend: str, wid: str, step_ms: float) -> None:
    from mxserve.frontend import httpd

    active: dict = {}  # rid -> [remaining, channel conn, n]
    chans: dict = {}

    def line(rid: str, st: list) -> list:
        st[0] -= 1
        st[2] += 1
        fin = st[0] <= 0
        return [rid, {"t": 300 + st[2] % 26, "f": fin, "r": "length" if fin else None, "p": 100, "c": 0}]

    async def stepper():
        nxt = time.perf_counter()
        while True:
            nxt += step_ms / 1e3
            await asyncio.sleep(max(0.0, nxt - time.perf_counter()))
            per: dict = {}
            for rid, st in list(active.items()):
                per.setdefault(id(st[1]), (st[1], []))[1].append(line(rid, st))
                if st[0] <= 0:
                    active.pop(rid, None)
            for conn, b in per.values():
                conn.write_chunk((json.dumps({"b": b}) + "\n").encode())

    async def fast(req, conn) -> bool:
        if req.path == "/mux":
            sid = json.loads(req.body)["sid"]
            chans[sid] = conn
            conn.write_head(200, [(b"content-type", b"application/x-ndjson"), (b"transfer-encoding", b"chunked")])
            conn.write_chunk((json.dumps({"hello": sid}) + "\n").encode())
            return True  # the connection stays a stream
        if req.path == "/submit":
            b = json.loads(req.body)
            ch = chans.get(b["sid"])
            if ch is None:
                conn.write_head(404, [(b"content-length", b"0")])
                conn.finish()
                return True
            st = [int(b["sampling"].get("max_tokens", 16)), ch, 0]
            conn.write_head(200, [(b"content-type", b"application/json"), (b"content-length", b"11")])
            conn.write(b'{"ok":true}')
            conn.finish()
            ch.write_chunk((json.dumps({"b": [line(b["request_id"], st)]}) + "\n").encode())  # first token now
            if st[0] > 0:
                active[b["request_id"]] = st
            return True
        if req.path == "/abort":
            active.pop(json.loads(req.body).get("request_id"), None)
            conn.write_head(200, [(b"content-length", b"2")])
            conn.write(b"{}")
            conn.finish()
            return True
        conn.write_head(404, [(b"content-length", b"0")])
        conn.finish()
        return True

    async def register():
        import aiohttp
        reg = {"worker_id": wid, "url": f"http://127.0.0.1:{port}", "model": MODEL, "role": "agg", "block_size": 16,
               "kv_total_blocks": 500000, "tp": 1, "max_model_len": 8192}
        async with aiohttp.ClientSession() as s:
            while True:
                try:
                    async with s.post(frontend + "/internal/register", json=reg) as r:
                        if r.status == 200:
                            break
                except Exception:  # noqa: BLE001
                    pass
                await asyncio.sleep(0.3)
            while True:
                await asyncio.sleep(1.0)
                try:
                    async with s.post(frontend + "/internal/heartbeat",
                                      json={"worker_id": wid, "load": {"num_running": len(active)}, "stored": [],
                                            "removed": []}) as r:
                        if r.status == 404:
                            async with s.post(frontend + "/internal/register", json=reg) as r2:
                                await r2.read()
                except Exception:  # noqa: BLE001
                    pass

    async def main():
        asyncio.ensure_future(stepper())
        asyncio.ensure_future(register())
        await httpd.Server(None, fast).serve(httpd.listen("127.0.0.1", port))

    asyncio.run(main())


# ---------------------------------------------------------------------------- client
def client(port: int, rate: float, duration: float, osl: int, seed: int, out: str) -> None:
    rng = random.Random(seed)
    res = {"ttft": [], "gaps": [], "done": 0, "dropped": 0, "tokens": 0, "t0": time.perf_counter(), "t1": 0.0,
           "per_s": {}, "drop_reasons": {}}

    def drop(reason: str) -> None:
        res["dropped"] += 1
        res["drop_reasons"][reason] = res["drop_reasons"].get(reason, 0) + 1

    class Stream(asyncio.Protocol):
        """One streaming request on its own connection; data_received counts SSE chunks (no
        StreamReader / task wakeup per read: the client must be cheaper than what it measures)."""
        __slots__ = ("t_sched", "n", "first", "last", "tail", "done", "fut", "tr", "status", "err", "lost")

        def __init__(self, t_sched: float, body: bytes, fut):
            self.t_sched, self.n, self.first, self.last, self.tail, self.done = t_sched, 0, None, None, b"", False
            self.fut = fut
            self.tr = body
            self.status = None  # HTTP status of the response
            self.err = None  # the stream's SSE error message, if it sent one
            self.lost = None  # repr of the connection_lost exception

        def connection_made(self, tr):
            body, self.tr = self.tr, tr
            tr.write(b"POST /v1/completions HTTP/1.1\r\nhost: x\r\ncontent-type: application/json\r\n"
                     b"content-length: %d\r\nconnection: close\r\n\r\n%b" % (len(body), body))

        def data_received(self, data):
            now = time.perf_counter()
            if self.status is None and data.startswith(b"HTTP/1.1 "):
                self.status = int(data[9:12])
            if self.err is None and b'data: {"error"' in data:
                i = data.find(b'data: {"error"')
                self.err = data[i + 6:data.find(b"\n", i)].decode(errors="replace")[:200]
            buf = self.tail + data  # the tail (11 bytes) cannot hold a whole `data: {`: nothing counts twice
            k = buf.count(b"data: {")
            if k:
                if self.first is None:
                    self.first = now
                    res["ttft"].append(now - self.t_sched)
                elif self.n % 16 == 0:
                    res["gaps"].append((now - self.last) / k)
                self.n += k
                self.last = now
                sec = int(now - res["t0"])
                per_s[sec] = per_s.get(sec, 0) + k
            if b"data: [DONE]" in buf:
                self.done = True
                self.tr.close()
            self.tail = buf[-11:]

        def connection_lost(self, exc):
            if exc is not None:
                self.lost = repr(exc)[:120]
            if not self.fut.done():
                self.fut.set_result(None)

    per_s = res["per_s"]

    async def one(t_sched: float):
        ids = [rng.randrange(1000, 120000) for _ in range(100)]
        body = json.dumps({"model": MODEL, "prompt": ids, "max_tokens": osl, "stream": True,
                           "temperature": 0}).encode()
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        try:
            _, st = await loop.create_connection(lambda: Stream(t_sched, body, fut), "127.0.0.1", port)
        except OSError as e:
            drop(f"connect: {type(e).__name__} {getattr(e, 'errno', '')}")
            return
        await fut
        if st.done and st.n >= osl:
            res["done"] += 1
        elif st.status is not None and st.status != 200:
            drop(f"http {st.status}")
        elif st.err is not None:
            drop(f"stream error: {st.err}")
        elif st.done:
            drop(f"[DONE] after {st.n} < {osl} tokens")
        else:
            drop(f"closed before [DONE] ({'no response' if st.status is None else 'mid-stream'})"
                 + (f": {st.lost}" if st.lost else ""))
        res["tokens"] += st.n

    async def main():
        tasks = []
        t0 = time.perf_counter()
        res["t0"] = t0
        t = t0
        while t - t0 < duration:
            t += rng.expovariate(rate)
            await asyncio.sleep(max(0.0, t - time.perf_counter()))
            tasks.append(asyncio.ensure_future(one(t)))
        await asyncio.gather(*tasks)
        res["t1"] = time.perf_counter()
    asyncio.run(main())
    import resource
    ru = resource.getrusage(resource.RUSAGE_SELF)
    res["cpu_s"] = ru.ru_utime + ru.ru_stime
    with open(out, "w") as f:
        json.dump(res, f)


# ---------------------------------------------------------------------------- driver
def _pct(v: list, q: float):
    if not v:
        return None
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def cpu_seconds(pid: int) -> float:
    import psutil
    tot = 0.0
    for p in [psutil.Process(pid)] + psutil.Process(pid).children(recursive=True):
        try:
            t = p.cpu_times()
            tot += t.user + t.system
        except psutil.NoSuchProcess:
            pass
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--role", default="driver")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--frontend", default="")
    ap.add_argument("--wid", default="fake-0")
    ap.add_argument("--tok-per-s", type=float, default=170000)
    ap.add_argument("--osl", type=int, default=500)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--clients", type=int, default=4)
    ap.add_argument("--duration", type=float, default=20.0)
    ap.add_argument("--step-ms", type=float, default=10.0)
    ap.add_argument("--rate", type=float, default=0.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.role == "worker":
        return fake_worker(a.port, a.frontend, a.wid, a.step_ms)
    if a.role == "client":
        return client(a.port, a.rate, a.duration, a.osl, a.seed, a.out)
    from tests.serving_utils import free_port
    import tempfile
    tmp = tempfile.mkdtemp(prefix="mxs-feload-")
    fe_port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    me = os.path.abspath(__file__)
    procs = []
    fe = subprocess.Popen([sys.executable, "-m", "mxserve.frontend", "--http-host", "127.0.0.1", "--http-port",
                           str(fe_port), "--num-procs", str(a.procs)], env=env)
    procs.append(fe)
    try:
        furl = f"http://127.0.0.1:{fe_port}"
        for i in range(a.workers):
            procs.append(subprocess.Popen([sys.executable, me, "--role", "worker", "--port", str(free_port()),
                                           "--frontend", furl, "--wid", f"fake-{i}", "--step-ms", str(a.step_ms)],
                                          env=env))
        import urllib.request

        def known() -> int:
            with urllib.request.urlopen(furl + "/internal/workers", timeout=2) as r:
                return len(json.loads(r.read())["workers"])
        # every frontend process must have heard of every worker (the discovery bus forwards a
        # registration from the process that took it): fresh connections land on the processes at
        # random (SO_REUSEPORT), so require 8 * procs answers in a row to know them all; a request
        # reaching a process that does not know the model yet would be answered 404
        t_end, streak = time.time() + 60, 0
        while time.time() < t_end and streak < 8 * a.procs:
            try:
                streak = streak + 1 if known() >= a.workers else 0
            except Exception:  # noqa: BLE001
                streak = 0
            if streak == 0:
                time.sleep(0.3)
        rate = a.rate or a.tok_per_s / a.osl
        c0 = cpu_seconds(fe.pid)
        import psutil
        sys0 = psutil.cpu_times()
        t0 = time.time()
        cl = [subprocess.Popen([sys.executable, me, "--role", "client", "--port", str(fe_port), "--rate",
                                str(rate / a.clients), "--duration", str(a.duration), "--osl", str(a.osl),
                                "--seed", str(a.seed + i), "--out", os.path.join(tmp, f"c{i}.json")], env=env)
              for i in range(a.clients)]
        for p in cl:
            p.wait(timeout=a.duration + 300)
        wall = time.time() - t0
        sys1 = psutil.cpu_times()
        busy = sum(getattr(sys1, f) - getattr(sys0, f) for f in ("user", "nice", "system", "irq", "softirq"))
        idle = sum(getattr(sys1, f) - getattr(sys0, f) for f in ("idle", "iowait"))
        c1 = cpu_seconds(fe.pid)
        w_cpu = sum(cpu_seconds(p.pid) for p in procs[1:])
        ttft, gaps, done, dropped, toks, spans, per_s, reasons = [], [], 0, 0, 0, [], {}, {}
        c_cpu = 0.0
        for i in range(a.clients):
            r = json.load(open(os.path.join(tmp, f"c{i}.json")))
            ttft += r["ttft"]
            gaps += r["gaps"]
            done += r["done"]
            dropped += r["dropped"]
            toks += r["tokens"]
            spans.append(r["t1"] - r["t0"])
            c_cpu += r.get("cpu_s", 0.0)
            for why, k in r.get("drop_reasons", {}).items():
                reasons[why] = reasons.get(why, 0) + k
            for sec, k in r["per_s"].items():
                per_s[int(sec)] = per_s.get(int(sec), 0) + k
        # steady state: after one request lifetime (osl x step) of ramp-up, until arrivals stop
        lo, hi = int(a.osl * a.step_ms / 1e3) + 1, int(a.duration)
        steady = [per_s.get(s_, 0) for s_ in range(lo, hi)]
        res = {"target_tok_per_s": a.tok_per_s,
               "delivered_tok_per_s": round(sum(steady) / max(1, len(steady)), 1),
               "steady_window_s": [lo, hi],
               "requests_done": done, "requests_dropped": dropped, "drop_reasons": reasons,
               "frontend_procs": a.procs, "workers": a.workers,
               "client_procs": a.clients, "osl": a.osl, "step_ms": a.step_ms,
               "ttft_ms_p50": round(1e3 * _pct(ttft, 0.5), 2), "ttft_ms_p90": round(1e3 * _pct(ttft, 0.9), 2),
               "chunk_gap_ms_p50": round(1e3 * _pct(gaps, 0.5), 2), "chunk_gap_ms_p90": round(1e3 * _pct(gaps, 0.9), 2),
               "frontend_cpu_ms_per_1k_tokens": round(1e6 * (c1 - c0) / max(1, toks), 2),
               "cpu_s": {"frontend": round(c1 - c0, 1), "fake_workers": round(w_cpu, 1), "clients": round(c_cpu, 1)},
               "wall_s": round(wall, 1),
               # the whole box's CPU use during the run (this test's processes and everything else)
               "system_cpu_busy": round(busy / max(1e-9, busy + idle), 3),
               "cpus": os.cpu_count()}
        line = json.dumps(res)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    finally:
        for p in procs[1:]:
            p.terminate()
        fe.send_signal(signal.SIGINT)
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()


if __name__ == "__main__":
    main()
