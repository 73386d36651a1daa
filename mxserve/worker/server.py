"""Worker process: one engine (one GPU, or a TP group) behind an HTTP control/request plane.

Replaces `python3 -m dynamo.{vllm,sglang,trtllm}` (examples/deploy/*/agg.yaml:29-35).  Endpoints
  POST /generate   token-level request plane used by the frontend: NDJSON stream of token ids
                   (`prefill_url` set on a decode worker = disaggregated: reserve blocks, ask the
                   prefill worker to fill them over xGMI, then decode; falls back to local prefill)
  POST /mux        the multiplexed form: one long-lived NDJSON channel per frontend process that
  POST /submit     carries every request's tokens, one line per engine step ({"b": [[rid, batch],
  POST /abort      ...]}); requests join a channel with /submit and leave early with /abort.  At
                   ~200 running requests this is one write per step instead of 200 streamed
                   responses, so the HTTP side stops competing with the engine thread for the GIL
  POST /prefill    prefill worker: compute the prompt, push its KV blocks into the decode worker's
                   pool, return the first token
  POST /kv_write   host-staged KV backend (decode side)
  GET  /health /live /metrics /stats
Discovery: registers with the frontend (MXS_FRONTEND_URL) and heartbeats load + KV events (the
router's prefix index) every second; the lease expires if the worker dies.
"""
from __future__ import annotations

import asyncio
import contextlib
import json
import logging
import os
import socket
import threading
import time
import uuid
from typing import Optional

import msgpack
from fastapi import FastAPI, Request as HTTPRequest
from fastapi.responses import JSONResponse, PlainTextResponse, Response, StreamingResponse

from ..disagg.kv_transfer import KVTransferAgent
from ..engine.engine import AsyncEngine, LLMEngine, StepOutput
from ..engine.request import SamplingParams
from ..frontend.metrics import WorkerMetrics
from ..utils.tracing import FAULTS
from .args import WorkerArgs

log = logging.getLogger("mxserve.worker")


def _sampling(d: dict) -> SamplingParams:
    return SamplingParams(max_tokens=int(d.get("max_tokens", 16)), temperature=float(d.get("temperature", 1.0)),
                          top_p=float(d.get("top_p", 1.0)), top_k=int(d.get("top_k", 0)), seed=d.get("seed"),
                          stop_token_ids=list(d.get("stop_token_ids", [])), ignore_eos=bool(d.get("ignore_eos")),
                          min_tokens=int(d.get("min_tokens", 0)),
                          logprobs=None if d.get("logprobs") is None else int(d["logprobs"]),
                          repetition_penalty=float(d.get("repetition_penalty", 1.0)),
                          frequency_penalty=float(d.get("frequency_penalty", 0.0)),
                          presence_penalty=float(d.get("presence_penalty", 0.0)))


def _line(o: StepOutput) -> bytes:
    d = {"t": o.token_id, "f": o.finished, "r": o.finish_reason, "p": o.num_prompt_tokens, "c": o.num_cached_tokens}
    if o.logprob is not None:
        d["lp"] = o.logprob
        d["tlp"] = o.top_logprobs or []
    if o.timing:
        d["tm"] = o.timing
    return (json.dumps(d) + "\n").encode()


def _batch_line(outs: list) -> bytes:
    """Every token of a request that is ready when the stream writes: one NDJSON line (a list of
    ids).  A consumer that keeps up still gets one token per line; one that falls behind (a busy
    frontend at tens of thousands of tokens/s) gets fewer, larger lines instead of a backlog."""
    if len(outs) == 1:
        return _line(outs[0])
    return (json.dumps(_batch_dict(outs)) + "\n").encode()


def _batch_dict(outs: list) -> dict:
    last = outs[-1]
    d = {"t": [o.token_id for o in outs], "f": last.finished, "r": last.finish_reason, "p": last.num_prompt_tokens,
         "c": last.num_cached_tokens}
    if any(o.logprob is not None for o in outs):
        d["lp"] = [o.logprob for o in outs]
        d["tlp"] = [o.top_logprobs or [] for o in outs]
    tm = next((o.timing for o in outs if o.timing), None)
    if tm:
        d["tm"] = tm
    return d


_RING = object()  # sink marker: the request's outputs go to the streamer ring


class _MuxSink:
    """Stands in for a request's asyncio.Queue in AsyncEngine._queues: outputs go to its channel
    (put_nowait runs on the event loop, from AsyncEngine._deliver's one wakeup per step)."""
    __slots__ = ("ch",)

    def __init__(self, ch: "MuxChannel"):
        self.ch = ch

    def put_nowait(self, o) -> None:
        self.ch.pending.append(o)
        self.ch.wake.set()


class _DropSink(_MuxSink):
    """Fault injection (MXS_FAULT drop_stream) on the mux plane: after the first token the request
    is aborted and its stream ends with a "dropped" marker (token -2), which the frontend treats as
    a lost connection (retry / migrate)."""
    __slots__ = ("n", "on_drop")

    def __init__(self, ch: "MuxChannel", on_drop):
        super().__init__(ch)
        self.n = 0
        self.on_drop = on_drop

    def put_nowait(self, o) -> None:
        self.n += 1
        if self.n == 1:
            super().put_nowait(o)
        elif self.n == 2:
            super().put_nowait(StepOutput(o.request_id, -2, True, "abort", 0, 0, 0))
            self.on_drop(o.request_id)


class MuxChannel:
    """One frontend process's request-plane channel (POST /mux): the tokens of all its requests,
    one NDJSON line per wakeup (one engine step): {"b": [[request_id, batch], ...]}, where batch is
    the /generate line format."""

    def __init__(self, sid: str):
        self.sid = sid
        self.pending: list = []
        self.wake = asyncio.Event()
        self.rids: set = set()
        self.closed = False

    async def lines(self, aeng: AsyncEngine):
        why = "frontend closed the channel"
        try:
            yield (json.dumps({"hello": self.sid}) + "\n").encode()
            while True:
                await self.wake.wait()
                self.wake.clear()
                outs, self.pending = self.pending, []
                by_rid: dict = {}
                for o in outs:
                    by_rid.setdefault(o.request_id, []).append(o)
                batch = []
                for rid, os_ in by_rid.items():
                    batch.append([rid, _batch_dict(os_)])
                    if os_[-1].finished:
                        self.rids.discard(rid)
                if batch:
                    yield (json.dumps({"b": batch}) + "\n").encode()
        except BaseException as e:  # noqa: BLE001 - logged, then re-raised
            why = "frontend disconnected" if isinstance(e, (GeneratorExit, asyncio.CancelledError)) else repr(e)
            raise
        finally:  # the frontend went away: its requests have nobody to stream to
            if self.rids:
                log.warning("mux channel %s closed (%s): aborting %d in-flight requests", self.sid,
                            "replaced by a new channel" if self.closed else why, len(self.rids))
            self.closed = True
            for rid in list(self.rids):
                if aeng._queues.pop(rid, None) is not None:
                    aeng.submit_nowait(aeng.engine.abort, rid)
            self.rids.clear()


class Worker:
    def __init__(self, wargs: WorkerArgs, engine: Optional[LLMEngine] = None):
        self.wargs = wargs
        self.args = wargs.engine
        self.config_warnings = list(getattr(wargs, "warnings", []) or [])
        self.engine = engine or LLMEngine(self.args)
        self.aeng = AsyncEngine(self.engine)
        self.role = self.args.disagg_mode
        self.model = self.args.name
        self.metrics = WorkerMetrics()
        self.faults = FAULTS  # tests may give one worker its own Faults
        self.agent = KVTransferAgent(self.engine.runner, self.args.kv_transfer_backend)
        if self.role == "decode":  # allocate + export the staging arena before traffic arrives
            self.agent.descriptor()
        self.worker_id = wargs.worker_id or f"{self.role}-{socket.gethostname()}-{uuid.uuid4().hex[:6]}"
        self.url: Optional[str] = None
        self._events_lock = threading.Lock()
        self._stored: list = []
        self._removed: list = []
        self.aeng.on_step = self._on_step
        self.ready = True
        self._http = None
        self._channels: dict[str, MuxChannel] = {}
        self.stream_url: Optional[str] = None  # the streamer process's request plane (attach_streamer)
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self._ring_plane = None
        self.kv_quarantined = 0  # remote prefills whose extents / blocks wait for the prefill side
        self.app = self._build_app()

    # ---------------------------------------------------------------- engine-thread hook
    def _on_step(self, outs) -> None:
        stored, removed = self.engine.kv.take_events()
        if stored or removed:
            with self._events_lock:
                self._stored.extend(stored)
                self._removed.extend(removed)
        self.metrics.gen_tokens.labels(self.model).inc(len(outs))
        if self.faults.active():
            self.faults.step_delay()
            self.faults.count_tokens(len(outs))

    def take_events(self):
        with self._events_lock:
            s, r = self._stored, self._removed
            self._stored, self._removed = [], []
        return s, r

    # ---------------------------------------------------------------- http client
    async def http(self):
        if self._http is None:
            import aiohttp
            self._http = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None, sock_connect=10))
        return self._http

    # ---------------------------------------------------------------- handlers
    async def _generate_stream(self, body: dict):
        rid = body.get("request_id") or uuid.uuid4().hex
        toks = list(body["token_ids"])
        sp = _sampling(body.get("sampling", {}))
        purl = body.get("prefill_url")
        if purl and self.role == "decode":
            q = await self._remote_prefill(rid, toks, sp, purl)
            if q is not None:
                async for outs in self.aeng.stream_batches(rid, q):
                    yield _batch_line(outs)
                return
        drop = self.faults.hit("drop_stream")
        if drop:
            n = 0
            async for o in self.aeng.generate(toks, sp, rid):
                n += 1
                if n > 1:  # fault injection: abort mid-stream
                    await self.aeng.submit(self.engine.abort, rid)
                    raise ConnectionError("fault injection: stream dropped")
                yield _line(o)
            return
        q = self.aeng.open_stream(rid)
        try:
            await self.aeng.submit(self._add_request, toks, sp, rid, time.monotonic())
        except BaseException:
            self.aeng._queues.pop(rid, None)
            raise
        async for outs in self.aeng.stream_batches(rid, q):
            yield _batch_line(outs)

    async def _submit(self, body: dict) -> dict:
        """Multiplexed request plane: start a request whose tokens go to channel body["sid"]."""
        ch = self._channels.get(body.get("sid", ""))
        if ch is None or ch.closed:
            return {"error": "unknown channel"}
        rid = body.get("request_id") or uuid.uuid4().hex
        toks = list(body["token_ids"])
        sp = _sampling(body.get("sampling", {}))
        purl = body.get("prefill_url")
        sink = _DropSink(ch, self._abort) if self.faults.hit("drop_stream") else _MuxSink(ch)
        ch.rids.add(rid)
        if purl and self.role == "decode":
            if await self._remote_prefill(rid, toks, sp, purl, sink=sink) is not None:
                return {"ok": True}
        self.aeng._queues[rid] = (asyncio.get_running_loop(), sink)
        try:
            await self.aeng.submit(self._add_request, toks, sp, rid, time.monotonic())
        except BaseException:
            self.aeng._queues.pop(rid, None)
            ch.rids.discard(rid)
            raise
        return {"ok": True}

    def _add_request(self, toks: list, sp: SamplingParams, rid: str, t_in: float):
        """Engine thread: add the request, stamping when the HTTP layer received it."""
        req = self.engine.add_request(toks, sp, rid, None)
        req.submit_time = t_in
        return req

    # ---------------------------------------------------------------- streamer process
    def attach_streamer(self, cmd_ring, out_ring, stream_url: str, proc=None) -> None:
        """The token request plane moves to the streamer process (worker/streamer.py)."""
        from .streamer import RingPlane
        self._ring_plane = RingPlane(self, cmd_ring, out_ring, proc)
        self.stream_url = stream_url
        self.aeng.attach_ring(self._ring_plane)

    def start_remote_ring(self, rid: str, toks: list, sp: SamplingParams, purl: str, t_in: float) -> None:
        """Event loop: a streamer request with a prefill URL (disaggregated decode)."""
        t = asyncio.ensure_future(self._remote_ring(rid, toks, sp, purl, t_in))
        t.add_done_callback(lambda f: f.cancelled() or f.exception() is None or
                            log.error("remote prefill of %s failed: %r", rid, f.exception()))

    async def _remote_ring(self, rid: str, toks: list, sp: SamplingParams, purl: str, t_in: float) -> None:
        if await self._remote_prefill(rid, toks, sp, purl, sink=_RING) is None:  # prefill locally
            self.aeng.submit_nowait(self._ring_plane.add_local, toks, sp, rid, t_in)

    def _abort(self, rid: str) -> bool:
        ent = self.aeng._queues.pop(rid, None)
        if ent is None:
            return False
        if isinstance(ent[1], _MuxSink):
            ent[1].ch.rids.discard(rid)
        self.aeng.submit_nowait(self.engine.abort, rid)
        return True

    async def _remote_prefill(self, rid: str, toks: list, sp: SamplingParams, purl: str, sink=None):
        """Decode side of the disaggregated protocol.  Returns the token queue (or `sink`, the
        request's mux channel sink, when given), or None to fall back to local prefill."""
        req = await self.aeng.submit(self.engine.reserve_remote_prefill, toks, sp, rid)
        if req is None:
            return None
        if sink is _RING:
            self.aeng.own_by_ring(rid)
            q = sink
        elif sink is not None:
            self.aeng._queues[rid] = (asyncio.get_running_loop(), sink)
            q = sink
        else:
            q = self.aeng.open_stream(rid)
        skip = req.num_cached_tokens // self.args.block_size
        nblk = -(-len(toks) // self.args.block_size)
        dst = list(req.block_ids[skip:nblk])
        try:
            target = self.agent.descriptor(self.url)
        except Exception as e:  # noqa: BLE001 - no staging arena: give the reservation back, prefill here
            log.warning("KV staging arena unavailable (%r); prefilling %s locally", e, rid)
            self.aeng._queues.pop(rid, None)
            self.aeng.submit_nowait(self.engine.abort, rid)
            return None
        # reserve an extent in every staging arena this worker has (GPU arena over xGMI IPC, host
        # arena in /dev/shm); the prefill worker uses the first it can reach and says which
        start = self.agent.acquire(len(dst)) if target["backend"] == "xgmi" else None
        shm_start = self.agent.acquire_shm(len(dst)) if target.get("shm_name") else None
        if start is None:
            target["backend"] = "host"
        target["block_ids"] = dst
        target["skip_blocks"] = skip
        target["arena_start"] = start
        target["shm_start"] = shm_start
        payload = {"request_id": rid, "token_ids": toks, "sampling": _sp_dict(sp), "kv_target": target}
        completed = False
        answered = False  # the prefill worker replied: it no longer writes our extents or blocks
        post = None
        t_post = time.perf_counter()
        try:
            sess = await self.http()

            async def do_post():
                async with sess.post(purl.rstrip("/") + "/prefill", json=payload) as r:
                    return r.status, (await r.json() if r.status == 200 else await r.text())
            # shielded: a client going away cancels this coroutine, not the POST, whose reply is
            # what tells us the prefill worker has stopped pushing into our extents and blocks
            post = asyncio.ensure_future(do_post())
            status, res = await asyncio.shield(post)
            answered = True
            if status != 200:
                raise RuntimeError(f"prefill worker returned {status}: {res}")

            via = res.get("via", target["backend"])

            def land_and_complete(tok: int):
                # the arena the prefill worker wrote -> pool blocks, on the engine's stream (ordered
                # before the next step); the other extents are recycled unused
                if via == "xgmi":
                    self.agent.land(start, dst)
                elif start is not None:
                    self.agent.release(start, len(dst))
                if via == "shm":
                    self.agent.land_shm(shm_start, dst)
                elif shm_start is not None:
                    self.agent.release_shm(shm_start, len(dst))
                return self.engine.complete_remote_prefill(rid, tok, res.get("logprob"), res.get("top_logprobs"))

            out = await self.aeng.submit(land_and_complete, int(res["first_token"]))
            completed = True  # the landing copies now own (and recycle) the extents
            xfer_ms = 1e3 * float(res.get("transfer_s", 0.0))
            out.timing = {"remote_prefill_ms": round((time.perf_counter() - t_post) * 1e3 - xfer_ms, 3),
                          "kv_transfer_ms": round(xfer_ms, 3), "kv_path": via,
                          **{f"prefill_worker_{k}": v for k, v in (res.get("timing") or {}).items()}}
            self.aeng.push(out)
            if "transfer_s" in res:
                self.metrics.kv_xfer_lat.labels(self.model).observe(float(res["transfer_s"]))
                self.metrics.kv_xfer_bytes.labels(self.model, via).inc(len(target["block_ids"]) * self.agent.block_bytes)
            return q
        except Exception as e:  # noqa: BLE001 - SURVEY §5.3: fall back to local prefill
            log.warning("remote prefill failed for %s (%r); prefilling locally", rid, e)
            return None
        finally:
            # any non-completion -- an error above, or the client/frontend going away mid-POST
            # (CancelledError is a BaseException): give back the arena extents, the reserved KV
            # blocks and the token queue, or they leak until every reservation fails -- but only
            # once the prefill worker can no longer push into them (a late push into a
            # reused extent or block would land the wrong KV in another request)
            if not completed:
                self.aeng._queues.pop(rid, None)
                if answered or post is None:
                    self._release_remote(rid, start, shm_start, len(dst))
                else:
                    self._quarantine_remote(rid, post, start, shm_start, len(dst))

    def _release_remote(self, rid: str, start, shm_start, n: int) -> None:
        if start is not None:
            self.agent.release(start, n)
        if shm_start is not None:
            self.agent.release_shm(shm_start, n)
        self.aeng.submit_nowait(self.engine.abort, rid)

    # how long extents and blocks of a remote prefill whose POST failed without a reply stay held:
    # the prefill worker may have received it and still push (a reply settles it at once)
    QUARANTINE_S = float(os.environ.get("MXS_KV_QUARANTINE_S", "60"))

    def _quarantine_remote(self, rid: str, post: "asyncio.Future", start, shm_start, n: int) -> None:
        """The POST has no reply yet (cancelled) or failed without one: detach the request now (its
        id is free for the local fallback) and free its blocks and extents when the prefill worker
        has replied, or QUARANTINE_S after a reply-less failure."""
        held: dict = {}
        self.aeng.submit_nowait(lambda: held.__setitem__("req", self.engine.detach_remote_prefill(rid)))
        loop = asyncio.get_running_loop()

        def free() -> None:
            if start is not None:
                self.agent.release(start, n)
            if shm_start is not None:
                self.agent.release_shm(shm_start, n)
            self.aeng.submit_nowait(lambda: held.get("req") is not None and self.engine.release_detached(held["req"]))
            self.kv_quarantined -= 1

        def done(f: "asyncio.Future") -> None:
            replied = not f.cancelled() and f.exception() is None
            if replied:
                free()
            else:
                loop.call_later(self.QUARANTINE_S, free)
        self.kv_quarantined += 1
        post.add_done_callback(done)

    async def _push(self, loop, jobs: list, after) -> float:
        """Issue a KV push (an executor thread: a first IPC mapping may take milliseconds) and wait
        for its event without blocking any thread; returns seconds from issue to completion."""
        t0 = time.perf_counter()
        ev = await loop.run_in_executor(None, self.agent.push_async, jobs, after)
        while ev is not None and not ev.query():
            await asyncio.sleep(0.0002)
        return time.perf_counter() - t0

    async def _prefill(self, body: dict) -> dict:
        """Prefill side: compute, push KV into the decode worker's pool, return the first token."""
        rid = body["request_id"]
        if self.faults.hit("fail_prefill"):
            raise RuntimeError("fault injection: prefill rejected")
        toks = list(body["token_ids"])
        sp = _sampling(body.get("sampling", {}))
        sp.max_tokens = 1
        first = first_lp = None
        async for o in self.aeng.generate(toks, sp, rid, disagg_role="prefill_only"):
            first, first_lp = o.token_id, o
        timing = first_lp.timing if first_lp is not None else None
        req = self.engine.requests.get(rid)
        target = body["kv_target"]
        skip = int(target.get("skip_blocks", 0))
        dst = list(target["block_ids"])
        src = list(req.block_ids[skip:skip + len(dst)]) if req is not None else []
        xfer_s = 0.0
        via = None
        loop = asyncio.get_running_loop()
        try:
            if len(src) != len(dst):
                raise RuntimeError(f"block count mismatch: {len(src)} local vs {len(dst)} remote")
            # the push waits (on the transfer stream) for the step that wrote this prompt's last KV
            # block, not for whatever the engine queued after it; the event is polled here, so
            # neither the engine thread nor an executor thread blocks on the copy
            after = getattr(req, "kv_ready", None)
            if target["backend"] == "xgmi" and self.agent.backend == "xgmi" and target.get("arena_start") is not None:
                try:
                    xfer_s = await self._push(loop, [(src, target, int(target["arena_start"]), "xgmi")], after)
                    via = "xgmi"
                except (RuntimeError, OSError) as e:  # the decode GPU's arena cannot be mapped here
                    log.warning("xGMI push to %s failed (%r); trying the shm / host paths", target.get("url"), e)
            if via is None and target.get("shm_start") is not None:
                try:
                    xfer_s = await self._push(loop, [(src, target, int(target["shm_start"]), "shm")], after)
                    via = "shm"
                except OSError:  # the decode worker's /dev/shm is not ours (another pod / host)
                    pass
            if via is None:
                via = "host"
                t0 = time.perf_counter()
                data = await asyncio.get_running_loop().run_in_executor(None, self.agent.read_blocks, src)
                sess = await self.http()
                async with sess.post(target["url"].rstrip("/") + "/kv_write",
                                     data=msgpack.packb({"block_ids": dst, "data": data}),
                                     headers={"content-type": "application/msgpack"}) as r:
                    if r.status != 200:
                        raise RuntimeError(f"kv_write failed: {r.status}")
                xfer_s = time.perf_counter() - t0
        finally:
            self.aeng.submit_nowait(self.engine.release_prefill_blocks, rid)
        res = {"first_token": first, "num_cached_tokens": req.num_cached_tokens if req else 0,
               "transfer_s": xfer_s, "blocks": len(dst), "via": via, "timing": timing}
        if first_lp is not None and first_lp.logprob is not None:
            res.update(logprob=first_lp.logprob, top_logprobs=first_lp.top_logprobs or [])
        return res

    # ---------------------------------------------------------------- app
    def _build_app(self) -> FastAPI:
        app = FastAPI(title="mxserve worker", lifespan=self._lifespan)
        w = self

        @app.post("/generate")
        async def generate(request: HTTPRequest):
            body = await request.json()
            return StreamingResponse(w._generate_stream(body), media_type="application/x-ndjson")

        @app.post("/mux")
        async def mux(request: HTTPRequest):
            body = await request.json()
            sid = str(body.get("sid") or uuid.uuid4().hex)
            old = w._channels.get(sid)
            if old is not None:
                old.closed = True
            ch = w._channels[sid] = MuxChannel(sid)

            async def lines():
                try:
                    async for line in ch.lines(w.aeng):
                        yield line
                finally:
                    if w._channels.get(sid) is ch:
                        w._channels.pop(sid, None)
            return StreamingResponse(lines(), media_type="application/x-ndjson")

        @app.post("/submit")
        async def submit(request: HTTPRequest):
            res = await w._submit(await request.json())
            return JSONResponse(res, status_code=404 if "error" in res else 200)

        @app.post("/abort")
        async def abort(request: HTTPRequest):
            return {"aborted": w._abort(str((await request.json()).get("request_id", "")))}

        @app.post("/prefill")
        async def prefill(request: HTTPRequest):
            try:
                return JSONResponse(await w._prefill(await request.json()))
            except Exception as e:  # noqa: BLE001
                log.exception("prefill failed")
                return JSONResponse({"error": {"message": str(e)}}, status_code=500)

        @app.post("/kv_write")
        async def kv_write(request: HTTPRequest):
            d = msgpack.unpackb(await request.body())
            await asyncio.get_running_loop().run_in_executor(None, w.agent.write_blocks, d["block_ids"], d["data"])
            return {"ok": True}

        @app.get("/kv_pool")
        async def kv_pool():
            return w.agent.descriptor(w.url)

        @app.get("/health")
        async def health():
            if not w.ready:
                return JSONResponse({"status": "starting"}, status_code=503)
            rp = getattr(w, "_ring_plane", None)
            if rp is not None and (rp.dead or rp.streamer_exited()):  # its token plane is gone
                return JSONResponse({"status": "streamer down"}, status_code=503)
            out = {"status": "ready", "model": w.model, "role": w.role, "worker_id": w.worker_id}
            if w.config_warnings:
                out["config_warnings"] = list(w.config_warnings)
            return out

        @app.get("/live")
        async def live():
            return {"status": "alive"}

        @app.get("/stats")
        async def stats():
            return w.aeng.last_stats

        @app.get("/metrics")
        async def metrics():
            w.metrics.update(w.model, w.aeng.last_stats)
            return Response(w.metrics.render(), media_type="text/plain; version=0.0.4")

        return app

    @contextlib.asynccontextmanager
    async def _lifespan(self, app):
        self.loop = asyncio.get_running_loop()
        task = None
        if self.wargs.frontend_url:
            task = asyncio.get_running_loop().create_task(self._heartbeat_loop())
        yield
        if task is not None:
            task.cancel()
        if self._http is not None:
            await self._http.close()
            self._http = None

    # ---------------------------------------------------------------- discovery
    def registration(self) -> dict:
        st = self.aeng.last_stats
        return {"worker_id": self.worker_id, "url": self.url, "model": self.model, "role": self.role,
                "block_size": self.args.block_size, "kv_total_blocks": st.get("kv_total_blocks", 0),
                "tp": self.args.tensor_parallel_size, "max_model_len": self.args.max_model_len,
                "pair": os.environ.get("MXS_PAIR_ID", ""), "stream_url": self.stream_url}

    async def _heartbeat_loop(self) -> None:
        base = self.wargs.frontend_url.rstrip("/")
        registered = False
        while True:
            rp = self._ring_plane
            if rp is not None and (rp.dead or rp.streamer_exited()):
                # the token plane is gone: stop renewing the lease, so the frontend's registry
                # expires this worker and routes elsewhere (/health fails too)
                await asyncio.sleep(1.0)
                continue
            try:
                sess = await self.http()
                if not registered and self.stream_url:
                    # advertise the streamer's request plane only once it accepts connections: a
                    # request routed to it earlier is refused and the frontend drops this worker
                    async with sess.get(self.stream_url + "/health") as r:
                        if r.status != 200:
                            raise ConnectionError(f"streamer not ready ({r.status})")
                if not registered:
                    async with sess.post(base + "/internal/register", json=self.registration()) as r:
                        registered = r.status == 200
                        if registered:
                            log.info("registered with frontend %s as %s", base, self.worker_id)
                else:
                    stored, removed = self.take_events()
                    body = {"worker_id": self.worker_id, "load": self.aeng.last_stats, "stored": stored,
                            "removed": removed}
                    async with sess.post(base + "/internal/heartbeat", json=body) as r:
                        if r.status == 404:
                            registered = False
            except Exception as e:  # noqa: BLE001 - frontend not up yet / restarting
                log.debug("heartbeat failed: %r", e)
                registered = False
            await asyncio.sleep(1.0)


def _sp_dict(sp: SamplingParams) -> dict:
    return {"max_tokens": sp.max_tokens, "temperature": sp.temperature, "top_p": sp.top_p, "top_k": sp.top_k,
            "seed": sp.seed, "stop_token_ids": list(sp.stop_token_ids), "ignore_eos": sp.ignore_eos,
            "min_tokens": sp.min_tokens, "logprobs": sp.logprobs, "repetition_penalty": sp.repetition_penalty,
            "frequency_penalty": sp.frequency_penalty, "presence_penalty": sp.presence_penalty}


def advertise_url(wargs: WorkerArgs, port: int) -> str:
    host = wargs.advertise_host
    if not host:
        host = "127.0.0.1" if wargs.host in ("127.0.0.1", "localhost") else socket.gethostbyname(socket.gethostname())
    return f"http://{host}:{port}"


def serve(wargs: WorkerArgs) -> None:
    import sys
    import uvicorn
    from ..utils.logs import setup_logging
    setup_logging()
    # the engine thread and the HTTP event loop share the GIL: a thread that wants it waits up to
    # the switch interval (5 ms by default) while the other runs Python -- a whole decode step at
    # the headline point.  A shorter interval bounds the engine thread's wait.
    sys.setswitchinterval(float(os.environ.get("MXS_GIL_SWITCH_MS", "0.5")) / 1e3)
    # the token request plane in a streamer process (agg / decode workers), started before anything
    # here touches the GPU: a fresh interpreter, not a fork of a GPU process
    streamer = None
    if wargs.engine.disagg_mode != "prefill" and os.environ.get("MXS_STREAMER", "1") == "1":
        from .streamer import start_streamer
        sport = int(os.environ.get("MXS_STREAM_PORT", str(wargs.port + 100)))
        try:
            streamer = start_streamer(wargs.host, sport, wargs.engine.max_model_len) + (sport,)
        except Exception as e:  # noqa: BLE001 - no /dev/shm: the worker serves the plane itself
            log.warning("streamer process unavailable (%r); serving /mux in the worker", e)
    off = int(os.environ.get("MXS_DEVICE_OFFSET", "0"))
    if off and wargs.engine.resolved_device() == "cuda":  # second worker of a P/D pair pod
        import torch
        torch.cuda.set_device(off % torch.cuda.device_count())  # (a 1-GPU functional run shares GPU 0)
    if wargs.engine.tensor_parallel_size > 1:
        from .tp import start_tp_group
        start_tp_group(wargs.engine)
    w = Worker(wargs)
    w.url = advertise_url(wargs, wargs.port)
    if streamer is not None:
        proc, cmd_ring, out_ring, sport = streamer
        w.attach_streamer(cmd_ring, out_ring, advertise_url(wargs, sport), proc)
        log.info("token request plane: streamer process %d at %s", proc.pid, w.stream_url)
    log.info("worker %s (%s, %s) serving %s on %s", w.worker_id, w.role, w.agent.backend, w.model, w.url)
    try:
        uvicorn.run(w.app, host=wargs.host, port=wargs.port, log_level="warning", access_log=False)
    finally:
        w.engine.shutdown()
        if streamer is not None:
            streamer[0].terminate()
            try:
                streamer[0].wait(timeout=10)
            except Exception:  # noqa: BLE001
                streamer[0].kill()
