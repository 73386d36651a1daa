"""Multi-process OpenAI frontend: N processes accept on one port (SO_REUSEPORT), so the per-token
work (request-plane demux, detokenize, SSE) spreads over N cores instead of one interpreter.

The reference's frontend is one multi-threaded Rust process (Dynamo; examples/deploy/vllm/agg.yaml:
12-17); a Python process tops out around 20 k streamed tokens/s, which is what one MI355X produces
at the headline point, so the served TTFT would measure the frontend's queue instead of the engine.

Discovery stays in every process: a worker's register / heartbeat POST lands on ONE process (the
kernel picks), which applies it and publishes it on the bus; the parent forwards it to the other
processes, in arrival order, so every process has the whole registry and KV-event stream and each
runs its own router and lease reaper.  Frontend metrics use prometheus_client's multiprocess mode
(gauges summed over live processes), so /metrics on any process reports the whole frontend.
Request traces (/debug/traces) are per process.
"""
from __future__ import annotations

import logging
import multiprocessing as mp
import os
import queue
import shutil
import signal
import socket
import tempfile
import threading

log = logging.getLogger("mxserve.frontend")


class PeerBus:
    """One process's end: publish() to the parent, start() a thread that applies what the other
    processes published on the event loop."""

    def __init__(self, index: int, outbound, inbound):
        self.index = index
        self.outbound = outbound
        self.inbound = inbound

    def publish(self, kind: str, body: dict) -> None:
        self.outbound.put((self.index, kind, body))

    def start(self, loop, apply) -> None:
        def run():
            while True:
                msg = self.inbound.get()
                if msg is None:
                    return
                loop.call_soon_threadsafe(apply, msg[0], msg[1])
        threading.Thread(target=run, name="mxs-peer-bus", daemon=True).start()


def _listen(host: str, port: int) -> socket.socket:
    s = socket.socket(socket.AF_INET6 if ":" in host else socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    s.listen(2048)
    return s


def _child(index: int, args: dict, outbound, inbound) -> None:
    from ..utils.logs import setup_logging
    from .app import Frontend, serve_app
    setup_logging()
    fe = Frontend(router_mode=args["router_mode"], ttl=args["ttl"], namespace=args["namespace"],
                  reasoning_parser=args["reasoning_parser"])
    fe.bus = PeerBus(index, outbound, inbound)
    serve_app(fe, sock=_listen(args["host"], args["port"]))


def serve(args: dict, nprocs: int) -> int:
    """Run `nprocs` frontend processes on args["host"]:args["port"] until SIGTERM / SIGINT or until a
    process dies (then the rest are stopped and the exit code is non-zero: the pod restarts)."""
    mdir = tempfile.mkdtemp(prefix="mxs-frontend-metrics-")
    os.environ["PROMETHEUS_MULTIPROC_DIR"] = mdir  # inherited by the spawned processes
    ctx = mp.get_context("spawn")
    outbound = ctx.Queue()
    inbounds = [ctx.Queue() for _ in range(nprocs)]
    procs = [ctx.Process(target=_child, args=(i, args, outbound, inbounds[i]), name=f"mxs-frontend-{i}")
             for i in range(nprocs)]
    for p in procs:
        p.start()
    log.info("frontend: %d processes on %s:%d", nprocs, args["host"], args["port"])
    stop = threading.Event()

    def on_signal(signum, _frame):
        stop.set()
    signal.signal(signal.SIGTERM, on_signal)
    signal.signal(signal.SIGINT, on_signal)
    rc = 0
    try:
        while not stop.is_set():
            try:
                src, kind, body = outbound.get(timeout=0.5)
            except queue.Empty:
                dead = [p for p in procs if not p.is_alive()]
                if dead:
                    log.error("frontend process %s exited (%s); stopping", dead[0].name, dead[0].exitcode)
                    rc = 1
                    break
                continue
            for i, q in enumerate(inbounds):
                if i != src:
                    q.put((kind, body))
    finally:
        for q in inbounds:
            q.put(None)
        for p in procs:
            if p.is_alive():
                p.terminate()  # SIGTERM: uvicorn shuts down gracefully
        for p in procs:
            p.join(timeout=15)
            if p.is_alive():
                p.kill()
                p.join(timeout=5)
        shutil.rmtree(mdir, ignore_errors=True)
    return rc
