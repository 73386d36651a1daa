#!/usr/bin/env python3
"""Frontend CPU cost per streamed token, without a GPU: a fake worker (same discovery and request
plane as mxserve/worker/server.py, tokens from a 10 ms "step" loop instead of an engine) serves the
real frontend process, driven by the open-loop load generator.  Prints the frontend's CPU seconds
per 1,000 tokens and client-side TTFT / ITL; with --profile the frontend runs under cProfile and
the top functions by cumulative time are printed.

  python scripts/frontend_cpu_probe.py --qps 42 --requests 600 [--plane mux|stream] [--profile]
"""
import argparse
import asyncio
import json
import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fake_worker(port: int, frontend: str, step_ms: float) -> None:
    import uvicorn
    from fastapi import FastAPI, Request
    from fastapi.responses import StreamingResponse

    app = FastAPI()
    active: dict = {}  # rid -> [remaining, channel-or-queue, n]
    channels: dict = {}

    async def stepper():
        n_tok = 7
        while True:
            await asyncio.sleep(step_ms / 1e3)
            per_ch: dict = {}
            for rid, st in list(active.items()):
                st[0] -= 1
                st[2] += 1
                fin = st[0] <= 0
                d = {"t": 100 + (st[2] * n_tok) % 5000, "f": fin, "r": "length" if fin else None, "p": 100, "c": 0}
                sink = st[1]
                if isinstance(sink, asyncio.Queue):
                    sink.put_nowait((json.dumps(d) + "\n").encode())
                    if fin:
                        sink.put_nowait(None)
                else:
                    per_ch.setdefault(id(sink), (sink, []))[1].append([rid, d])
                if fin:
                    active.pop(rid, None)
            for ch, b in per_ch.values():
                ch["q"].put_nowait((json.dumps({"b": b}) + "\n").encode())

    async def _start():
        asyncio.get_running_loop().create_task(stepper())

        async def register():
            import aiohttp
            async with aiohttp.ClientSession() as s:
                reg = {"worker_id": "fake-0", "url": f"http://127.0.0.1:{port}", "model": "meta-llama/Llama-3.2-1B-Instruct",
                       "role": "agg", "block_size": 16, "kv_total_blocks": 500000, "tp": 1, "max_model_len": 8192}
                while True:
                    try:
                        async with s.post(frontend + "/internal/register", json=reg) as r:
                            if r.status == 200:
                                break
                    except Exception:  # noqa: BLE001
                        pass
                    await asyncio.sleep(0.5)
                while True:
                    await asyncio.sleep(1.0)
                    try:
                        async with s.post(frontend + "/internal/heartbeat",
                                          json={"worker_id": "fake-0", "load": {}, "stored": [], "removed": []}) as r:
                            await r.read()
                    except Exception:  # noqa: BLE001
                        pass
        asyncio.get_running_loop().create_task(register())

    app.router.on_startup.append(_start)

    @app.post("/mux")
    async def mux(request: Request):
        body = await request.json()
        ch = {"q": asyncio.Queue()}
        channels[body["sid"]] = ch

        async def lines():
            yield (json.dumps({"hello": body["sid"]}) + "\n").encode()
            while True:
                yield await ch["q"].get()
        return StreamingResponse(lines(), media_type="application/x-ndjson")

    @app.post("/submit")
    async def submit(request: Request):
        body = await request.json()
        active[body["request_id"]] = [int(body["sampling"].get("max_tokens", 16)), channels[body["sid"]], 0]
        return {"ok": True}

    @app.post("/abort")
    async def abort(request: Request):
        active.pop((await request.json())["request_id"], None)
        return {"aborted": True}

    @app.post("/generate")
    async def generate(request: Request):
        body = await request.json()
        q: asyncio.Queue = asyncio.Queue()
        active[body["request_id"]] = [int(body["sampling"].get("max_tokens", 16)), q, 0]

        async def lines():
            while True:
                x = await q.get()
                if x is None:
                    return
                yield x
        return StreamingResponse(lines(), media_type="application/x-ndjson")

    uvicorn.run(app, host="127.0.0.1", port=port, log_level="warning", access_log=False)


def cpu_seconds(pid: int) -> float:
    """CPU time of the frontend process and its children (a multi-process frontend)."""
    import psutil
    root = psutil.Process(pid)
    tot = 0.0
    for p in [root] + root.children(recursive=True):
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
    ap.add_argument("--qps", type=float, default=42)
    ap.add_argument("--requests", type=int, default=600)
    ap.add_argument("--osl", type=int, default=500)
    ap.add_argument("--step-ms", type=float, default=10.0)
    ap.add_argument("--plane", default="mux")
    ap.add_argument("--procs", type=int, default=1, help="frontend processes (--num-procs)")
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--out", default="/tmp/fe_probe")
    a = ap.parse_args()
    if a.role == "worker":
        return fake_worker(a.port, a.frontend, a.step_ms)
    from tests.serving_utils import free_port
    os.makedirs(a.out, exist_ok=True)
    fe_port, w_port = free_port(), free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, MXS_REQUEST_PLANE=a.plane)
    fe_cmd = [sys.executable] + (["-m", "cProfile", "-o", f"{a.out}/frontend.prof"] if a.profile else []) + [
        "-m", "mxserve.frontend", "--http-host", "127.0.0.1", "--http-port", str(fe_port), "--num-procs", str(a.procs)]
    fe = subprocess.Popen(fe_cmd, env=env)
    w = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--role", "worker", "--port", str(w_port),
                          "--frontend", f"http://127.0.0.1:{fe_port}", "--step-ms", str(a.step_ms)], env=env)
    try:
        import urllib.request
        for _ in range(120):
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{fe_port}/v1/models", timeout=2) as r:
                    if b'"id"' in r.read():
                        break
            except Exception:  # noqa: BLE001
                pass
            time.sleep(0.5)
        c0, t0 = cpu_seconds(fe.pid), time.time()
        subprocess.run([sys.executable, "-m", "benchmarks.utils.benchmark", "--benchmark-name", "fe_probe",
                        "--endpoint-url", f"http://127.0.0.1:{fe_port}", "--model", "meta-llama/Llama-3.2-1B-Instruct",
                        "--output-dir", a.out, "--concurrency", "", "--request-rate", str(a.qps), "--num-requests",
                        str(a.requests), "--isl", "100", "--osl", str(a.osl), "--token-ids", "--vocab", "128256",
                        "--warmup-s", "5"], env=env, check=True, cwd=ROOT)
        c1, t1 = cpu_seconds(fe.pid), time.time()
        res = {}
        d = os.path.join(a.out, "fe_probe")
        for fn in os.listdir(d):
            if fn.startswith("rate_"):
                res = json.load(open(os.path.join(d, fn)))
        toks = a.requests * a.osl
        print(json.dumps({"plane": a.plane, "procs": a.procs, "qps": a.qps, "frontend_cpu_s": round(c1 - c0, 2), "wall_s": round(t1 - t0, 1),
                          "frontend_cpu_ms_per_1k_tokens": round(1e3 * (c1 - c0) / toks * 1e3, 2),
                          "ttft_ms_p50": res.get("ttft_ms_p50"), "itl_ms_p50": res.get("itl_ms_p50"),
                          "steady_ttft_ms_p50": res.get("steady_ttft_ms_p50"),
                          "output_tok_per_s": res.get("output_tok_per_s")}))
    finally:
        w.terminate()
        fe.send_signal(signal.SIGINT)
        try:
            fe.wait(timeout=30)
        except subprocess.TimeoutExpired:
            fe.kill()
        w.wait(timeout=10)
    if a.profile:
        import pstats
        pstats.Stats(f"{a.out}/frontend.prof").sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
