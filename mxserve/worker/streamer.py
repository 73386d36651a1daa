"""Streamer process: the worker's token request plane (POST /mux, /submit, /abort) in a process of its
own, so streaming tokens to frontends never competes with the engine thread for the GIL.

  frontend --/submit--> streamer --cmd ring--> engine thread (drains it at step boundaries)
  frontend <---/mux---- streamer <--out ring--- engine thread (one message per step)

Both rings are the native /dev/shm rings of csrc/runtime/shm_ring.cpp (single producer, single
reader): the streamer's event loop is the only writer of the command ring, the engine thread the
only writer of the output ring.  The engine process keeps its own HTTP server for everything else
(registration and heartbeats, /prefill and the KV transfer endpoints, /generate, metrics); it
advertises the streamer as `stream_url`, which the frontend uses for /mux, /submit and /abort.

The streamer imports neither torch nor the engine, and is started before the worker touches the GPU.
"""
from __future__ import annotations

import argparse
import asyncio
import collections
import json
import logging
import os
import subprocess
import sys
import threading
import time
import uuid
from typing import Optional

import msgpack
from fastapi import FastAPI, Request  # module level: the handlers' annotations resolve here
from fastapi.responses import JSONResponse, StreamingResponse

log = logging.getLogger("mxserve.streamer")

# output tuple: (request_id, token_id, finished, finish_reason, prompt_tokens, cached_tokens, logprob,
# top_logprobs, timing)
_OUT_SLOT = 256 << 10


def _batch_dict(outs: list) -> dict:
    """The /generate line format (worker/server.py::_batch_dict) from output tuples."""
    last = outs[-1]
    if len(outs) == 1:
        d = {"t": last[1], "f": last[2], "r": last[3], "p": last[4], "c": last[5]}
        if last[6] is not None:
            d["lp"] = last[6]
            d["tlp"] = last[7] or []
    else:
        d = {"t": [o[1] for o in outs], "f": last[2], "r": last[3], "p": last[4], "c": last[5]}
        if any(o[6] is not None for o in outs):
            d["lp"] = [o[6] for o in outs]
            d["tlp"] = [o[7] or [] for o in outs]
    tm = next((o[8] for o in outs if o[8]), None)
    if tm:
        d["tm"] = tm
    return d


# ------------------------------------------------------------------------------ engine process end
class RingPlane:
    """Engine-process end of the rings (AsyncEngine.attach_ring handler).  poll / command / emit run
    on the engine thread."""

    # outputs held back while the ring is full (a GC pause or a slow SSE writer in the streamer):
    # re-sent, in order, ahead of the next step's; past this many messages the streamer is wedged
    BACKLOG_MAX = 4096

    def __init__(self, worker, cmd_ring, out_ring, proc=None):
        self.w = worker
        self.cmd = cmd_ring
        self.out = out_ring
        self.proc = proc  # the streamer process: `dead` only once it has exited (or is wedged)
        self.dropped = 0
        self.backlog: collections.deque = collections.deque()
        self.stalls = 0
        self.dead = False  # the streamer is gone: /health fails so the worker is replaced

    def poll(self, timeout: float):
        if self.backlog:  # an idle engine still delivers what a stall held back
            self.flush()
        data = self.cmd.pop(0, timeout)
        return None if data is None else msgpack.unpackb(data, raw=False)

    def command(self, cmd) -> None:
        kind = cmd[0]
        aeng = self.w.aeng
        if kind == "a":
            _, rid, toks, sp, t_unix, purl = cmd
            from .server import _sampling
            sampling = _sampling(sp or {})
            t_in = time.monotonic() - max(0.0, time.time() - t_unix)
            if purl and self.w.role == "decode" and self.w.loop is not None:
                self.w.loop.call_soon_threadsafe(self.w.start_remote_ring, rid, toks, sampling, purl, t_in)
                return
            self.add_local(toks, sampling, rid, t_in)
        elif kind == "x":
            rid = cmd[1]
            if aeng._queues.pop(rid, None) is not None:
                aeng.engine.abort(rid)

    def add_local(self, toks, sampling, rid: str, t_in: float) -> None:
        aeng = self.w.aeng
        aeng.own_by_ring(rid)
        try:
            self.w._add_request(toks, sampling, rid, t_in)
        except Exception as e:  # noqa: BLE001 - e.g. a duplicate id: fail the one request
            log.warning("request %s rejected: %r", rid, e)
            aeng._queues.pop(rid, None)
            self.emit_tuples([(rid, -1, True, "error", 0, 0, None, None, None)])

    def emit(self, outs) -> None:
        self.emit_tuples([(o.request_id, o.token_id, o.finished, o.finish_reason, o.num_prompt_tokens,
                           o.num_cached_tokens, o.logprob, o.top_logprobs, o.timing) for o in outs])

    def emit_tuples(self, tuples: list) -> None:
        data = msgpack.packb(tuples, use_bin_type=True)
        if len(data) > self.out.slot_bytes:  # split a large step (logprobs) into several messages
            half = len(tuples) // 2
            if half == 0:
                log.error("one output is larger than a ring slot; dropped")
                return
            self.emit_tuples(tuples[:half])
            self.emit_tuples(tuples[half:])
            return
        if self.dead:
            self.dropped += 1
            return
        self.backlog.append(data)
        self.flush()

    def flush(self) -> None:
        """Push held-back outputs in order without stalling the engine thread for long: a stall is
        transient (outputs wait in the backlog, nothing -- finish markers included -- is dropped)
        unless the streamer process has exited or the backlog overflows."""
        while self.backlog:
            if self.out.push(self.backlog[0], 0.002 if len(self.backlog) > 1 else 0.05):
                self.backlog.popleft()
                continue
            self.stalls += 1
            if self.streamer_exited() or len(self.backlog) > self.BACKLOG_MAX:
                self.dead = True
                self.dropped += len(self.backlog)
                self.backlog.clear()
                log.error("streamer process %s; dropping its outputs and failing /health",
                          "exited" if self.streamer_exited() else f"wedged ({self.BACKLOG_MAX} outputs queued)")
            return

    def streamer_exited(self) -> bool:
        return self.proc is not None and self.proc.poll() is not None


def start_streamer(host: str, port: int, max_prompt_tokens: int) -> tuple:
    """Create the rings and start the streamer process.  Returns (proc, cmd_ring, out_ring).  Call
    before this process initialises the GPU (the streamer is a fresh interpreter, not a fork)."""
    from .. import _native
    rt = _native.rt()
    tag = f"{os.getpid()}-{uuid.uuid4().hex[:8]}"
    cmd_name, out_name = f"/mxs-cmd-{tag}", f"/mxs-out-{tag}"
    cmd_slot = max(64 << 10, 8 * int(max_prompt_tokens) + 4096)
    cmd = rt.ShmRing(cmd_name, True, cmd_slot, 64, 1)  # a burst of submits between two engine steps
    out = rt.ShmRing(out_name, True, _OUT_SLOT, 32, 1)
    env = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    proc = subprocess.Popen([sys.executable, "-m", "mxserve.worker.streamer", "--host", host, "--port", str(port),
                             "--cmd", cmd_name, "--out", out_name, "--parent-pid", str(os.getpid())], env=env)
    return proc, cmd, out


# ------------------------------------------------------------------------------ streamer process
class _Chan:
    def __init__(self, sid: str):
        self.sid = sid
        self.pending: list = []
        self.wake = asyncio.Event()
        self.rids: set = set()
        self.closed = False


def build_app(cmd_ring, out_ring, parent_pid: Optional[int] = None):
    chans: dict[str, _Chan] = {}
    owner: dict[str, _Chan] = {}

    def push_cmd(msg) -> bool:
        return bool(cmd_ring.push(msgpack.packb(msg, use_bin_type=True), 5.0))

    def dispatch(batch) -> None:
        for t in batch:
            ch = owner.get(t[0])
            if ch is None:
                continue
            ch.pending.append(t)
            ch.wake.set()
            if t[2]:
                owner.pop(t[0], None)
                ch.rids.discard(t[0])

    def reader(loop) -> None:
        while True:
            data = out_ring.pop(0, 0.5)
            if data is None:
                if parent_pid is not None and os.getppid() != parent_pid:
                    os._exit(0)  # the engine process is gone
                continue
            loop.call_soon_threadsafe(dispatch, msgpack.unpackb(data, raw=False))

    async def lifespan(app):
        threading.Thread(target=reader, args=(asyncio.get_running_loop(),), name="mxs-out-ring", daemon=True).start()
        yield

    import contextlib
    app = FastAPI(title="mxserve streamer", lifespan=contextlib.asynccontextmanager(lifespan))

    @app.post("/mux")
    async def mux(request: Request):
        body = await request.json()
        sid = str(body.get("sid") or uuid.uuid4().hex)
        if sid in chans:
            chans[sid].closed = True
        ch = chans[sid] = _Chan(sid)

        async def lines():
            why = "frontend closed the channel"
            try:
                yield (json.dumps({"hello": sid}) + "\n").encode()
                while True:
                    await ch.wake.wait()
                    ch.wake.clear()
                    outs, ch.pending = ch.pending, []
                    by_rid: dict = {}
                    for t in outs:
                        by_rid.setdefault(t[0], []).append(t)
                    yield (json.dumps({"b": [[rid, _batch_dict(os_)] for rid, os_ in by_rid.items()]}) + "\n").encode()
            except BaseException as e:  # noqa: BLE001 - logged, then re-raised
                why = "frontend disconnected" if isinstance(e, (GeneratorExit, asyncio.CancelledError)) else repr(e)
                raise
            finally:  # the frontend went away: abort its requests
                if ch.rids:
                    log.warning("mux channel %s closed (%s): aborting %d in-flight requests", sid,
                                "replaced by a new channel" if chans.get(sid) is not ch else why, len(ch.rids))
                ch.closed = True
                for rid in list(ch.rids):
                    owner.pop(rid, None)
                    push_cmd(("x", rid))
                ch.rids.clear()
                if chans.get(sid) is ch:
                    chans.pop(sid, None)
        return StreamingResponse(lines(), media_type="application/x-ndjson")

    @app.post("/submit")
    async def submit(request: Request):
        body = await request.json()
        ch = chans.get(body.get("sid", ""))
        if ch is None or ch.closed:
            return JSONResponse({"error": "unknown channel"}, status_code=404)
        rid = body.get("request_id") or uuid.uuid4().hex
        owner[rid] = ch
        ch.rids.add(rid)
        if not push_cmd(("a", rid, list(body["token_ids"]), body.get("sampling", {}), time.time(),
                         body.get("prefill_url"))):
            owner.pop(rid, None)
            ch.rids.discard(rid)
            return JSONResponse({"error": "engine not consuming requests"}, status_code=503)
        return {"ok": True}

    @app.post("/abort")
    async def abort(request: Request):
        rid = str((await request.json()).get("request_id", ""))
        ch = owner.pop(rid, None)
        if ch is not None:
            ch.rids.discard(rid)
            push_cmd(("x", rid))
        return {"aborted": ch is not None}

    @app.get("/health")
    async def health():
        return {"status": "ready", "role": "streamer", "channels": len(chans), "requests": len(owner)}

    return app


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(prog="python -m mxserve.worker.streamer")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--cmd", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--parent-pid", type=int, default=None)
    a = ap.parse_args(argv)
    import uvicorn
    from .. import _native
    from ..utils.logs import setup_logging
    setup_logging()
    rt = _native.rt()
    cmd, out = rt.ShmRing(a.cmd, False), rt.ShmRing(a.out, False)
    from ..utils.gcpause import freeze_heap
    freeze_heap()  # the SSE loop of every stream runs here: keep full collections off it
    uvicorn.run(build_app(cmd, out, a.parent_pid), host=a.host, port=a.port, log_level="warning", access_log=False)


if __name__ == "__main__":
    main()
