"""Minimal HTTP/1.1 server for the frontend (replaces uvicorn + h11 on the serving path).

The reference frontend is one multi-threaded Rust process (examples/deploy/vllm/agg.yaml:12-17).
Ours is Python, and at ~20 k streamed tokens/s per GPU its per-token cost decides how many cores a
node's frontend needs.  Under uvicorn's pure-Python h11 protocol every SSE chunk crossed five async
generators, a task wakeup, Starlette's send wrappers and h11's state machine (~57 us of CPU per
token, scripts/frontend_cpu_probe.py).  This server keeps the socket in hand instead:

  * every request is parsed here (request line, headers, Content-Length body; keep-alive);
  * a `fast` hook (Frontend.fast_request) may take a request over -- the streaming chat / completion
    requests, whose tokens are then PUSHED from the worker channel's reader straight into this
    connection (`write`), with no per-token task switch;
  * everything else runs through the FastAPI app over a small ASGI bridge (lifespan included), so
    every route and error shape stays what the app defines.
"""
from __future__ import annotations

import asyncio
import logging
import os
import signal
import socket
from typing import Awaitable, Callable, Optional

log = logging.getLogger("mxserve.frontend.httpd")

MAX_HEAD = 64 << 10
MAX_BODY = 256 << 20
# a request's head and body must arrive within HEADER_TIMEOUT_S of its first byte (slowloris); an idle
# keep-alive connection is closed after IDLE_TIMEOUT_S
HEADER_TIMEOUT_S = float(os.environ.get("MXS_HTTP_HEADER_TIMEOUT_S", "30"))
IDLE_TIMEOUT_S = float(os.environ.get("MXS_HTTP_IDLE_TIMEOUT_S", "75"))
_REASONS = {200: "OK", 204: "No Content", 400: "Bad Request", 404: "Not Found", 405: "Method Not Allowed",
            408: "Request Timeout", 411: "Length Required", 413: "Payload Too Large", 422: "Unprocessable Entity",
            429: "Too Many Requests", 500: "Internal Server Error", 503: "Service Unavailable"}


class Request:
    __slots__ = ("method", "path", "query", "headers", "body", "version")

    def __init__(self, method: str, target: str, version: str, headers: list, body: bytes):
        self.method = method
        self.path, _, self.query = target.partition("?")
        self.version = version
        self.headers = headers  # [(lower-case name bytes, value bytes)]
        self.body = body

    def header(self, name: bytes) -> Optional[bytes]:
        for k, v in self.headers:
            if k == name:
                return v
        return None


class Connection(asyncio.Protocol):
    """One client connection: parses requests one at a time (keep-alive), hands each to the fast
    hook or the ASGI app, and owns the writes."""

    def __init__(self, server: "Server"):
        self.server = server
        self.transport: Optional[asyncio.Transport] = None
        self.buf = bytearray()
        self.busy = False  # a request is being answered; later bytes wait in buf
        self._timer: Optional[asyncio.TimerHandle] = None
        self._timer_kind = ""  # "idle" | "head" | ""
        self._continued = False  # 100 Continue already sent for the request being received
        self.closed = False
        self.on_close: list = []  # callbacks run once the client is gone (abort its request)
        self.keep_alive = True
        self._drain: Optional[asyncio.Future] = None
        self._paused = False

    # ------------------------------------------------------------------ asyncio.Protocol
    def connection_made(self, transport) -> None:
        self.transport = transport
        sock = transport.get_extra_info("socket")
        if sock is not None:
            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        self.server.conns.add(self)
        self._arm()

    # ------------------------------------------------------------------ timeouts
    def _arm(self, progress: bool = False) -> None:
        """Idle connection: IDLE_TIMEOUT_S; a request head partly received: HEADER_TIMEOUT_S from its
        first byte; a head received and its body still arriving: HEADER_TIMEOUT_S from the LAST
        chunk (`progress` re-arms it), so a large upload that keeps moving is never cut off; a
        request being answered: no timer."""
        if self.busy or self.closed:
            want = ""
        elif not self.buf:
            want = "idle"
        else:  # find() stops at the first match: cheap even with a large body buffered
            want = "body" if self.buf.find(b"\r\n\r\n") >= 0 else "head"
        if want == self._timer_kind and not (progress and want == "body"):
            return
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
        self._timer_kind = want
        if want:
            loop = asyncio.get_event_loop()
            self._timer = loop.call_later(IDLE_TIMEOUT_S if want == "idle" else HEADER_TIMEOUT_S, self._expire, want)

    def _expire(self, kind: str) -> None:
        self._timer = None
        self._timer_kind = ""
        if self.closed or self.busy:
            return
        if kind in ("head", "body"):
            self._fail(408, "request not received in time")
        elif self.transport is not None:
            self.transport.close()

    def connection_lost(self, exc) -> None:
        self.closed = True
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
        self.server.conns.discard(self)
        if self._drain is not None and not self._drain.done():
            self._drain.set_result(None)
        cbs, self.on_close = self.on_close, []
        for cb in cbs:
            try:
                cb()
            except Exception:  # noqa: BLE001
                log.exception("on_close callback failed")

    def pause_writing(self) -> None:
        self._paused = True

    def resume_writing(self) -> None:
        self._paused = False
        if self._drain is not None and not self._drain.done():
            self._drain.set_result(None)

    async def drain(self) -> None:
        if self._paused and not self.closed:
            self._drain = asyncio.get_running_loop().create_future()
            await self._drain

    def data_received(self, data: bytes) -> None:
        self.buf += data
        if not self.busy:
            self._next()
        self._arm(progress=True)

    # ------------------------------------------------------------------ parsing
    def _next(self) -> None:
        while not self.busy and not self.closed:
            req = self._parse()
            if req is None:
                return
            self.busy = True
            self._continued = False
            self._arm()
            asyncio.ensure_future(self._handle(req))

    def _parse(self) -> Optional[Request]:
        end = self.buf.find(b"\r\n\r\n")
        if end < 0:
            if len(self.buf) > MAX_HEAD:
                self._fail(413, "request head too large")
            return None
        head = bytes(self.buf[:end]).decode("latin-1").split("\r\n")
        try:
            method, target, version = head[0].split(" ", 2)
        except ValueError:
            self._fail(400, "bad request line")
            return None
        headers = []
        clen = None
        expect_continue = False
        for line in head[1:]:
            k, _, v = line.partition(":")
            k, v = k.strip().lower(), v.strip()
            headers.append((k.encode("latin-1"), v.encode("latin-1")))
            if k == "content-length":
                # digits only (int() would take "-5", "+5", "1_0"); a repeated header must agree
                if not v or not v.isascii() or not v.isdigit():
                    self._fail(400, "bad content-length")
                    return None
                if clen is not None and int(v) != clen:
                    self._fail(400, "conflicting content-length headers")
                    return None
                clen = int(v)
            elif k == "expect" and v.lower() == "100-continue":
                expect_continue = True
            elif k == "transfer-encoding" and v.lower() != "identity":
                self._fail(411, "chunked request bodies are not supported; send Content-Length")
                return None
            elif k == "connection":
                self.keep_alive = v.lower() != "close"
        if version == "HTTP/1.0":
            self.keep_alive = any(k == b"connection" and v.lower() == b"keep-alive" for k, v in headers)
        clen = clen or 0
        if clen > MAX_BODY:
            self._fail(413, "request body too large")
            return None
        if len(self.buf) < end + 4 + clen:
            if expect_continue and not self._continued and version != "HTTP/1.0":
                self._continued = True
                self.write(b"HTTP/1.1 100 Continue\r\n\r\n")
            return None
        body = bytes(self.buf[end + 4:end + 4 + clen])
        del self.buf[:end + 4 + clen]
        return Request(method, target, version, headers, body)

    def _fail(self, status: int, msg: str) -> None:
        import json
        body = json.dumps({"error": {"message": msg, "type": "invalid_request_error", "code": status}}).encode()
        self.write_head(status, [(b"content-type", b"application/json"), (b"content-length", str(len(body)).encode())],
                        close=True)
        self.write(body)
        self.finish()

    # ------------------------------------------------------------------ responses
    def write_head(self, status: int, headers: list, close: bool = False) -> None:
        if close:
            self.keep_alive = False
        parts = [f"HTTP/1.1 {status} {_REASONS.get(status, 'Status')}\r\n".encode()]
        for k, v in headers:
            parts.append(k + b": " + v + b"\r\n")
        if not self.keep_alive:
            parts.append(b"connection: close\r\n")
        parts.append(b"\r\n")
        self.write(b"".join(parts))

    def write(self, data: bytes) -> None:
        if not self.closed and data:
            self.transport.write(data)

    def write_chunk(self, data: bytes) -> None:
        """One piece of a chunked (Transfer-Encoding) body."""
        if not self.closed and data:
            self.transport.write(b"%x\r\n%b\r\n" % (len(data), data))

    def end_chunked(self) -> None:
        self.write(b"0\r\n\r\n")

    def buffered(self) -> int:
        return 0 if self.closed else self.transport.get_write_buffer_size()

    def finish(self) -> None:
        """The current response is complete: next request, or close."""
        self.on_close = []
        if self.closed:
            return
        if not self.keep_alive:
            self.transport.close()
            return
        self.busy = False
        if self.buf:
            self._next()
        self._arm()

    async def _handle(self, req: Request) -> None:
        try:
            fast = self.server.fast
            if fast is None or not await fast(req, self):
                await self.server.asgi(req, self)
        except Exception:  # noqa: BLE001 - a handler bug must not kill the server
            log.exception("request %s %s failed", req.method, req.path)
            if not self.closed:
                self.transport.close()


class Server:
    """`fast(req, conn) -> bool` takes a request over (True) or leaves it to the ASGI `app`."""

    def __init__(self, app, fast: Optional[Callable[[Request, Connection], Awaitable[bool]]] = None):
        self.app = app  # None: the fast hook serves every request (no ASGI app, no lifespan)
        self.fast = fast
        self.conns: set = set()
        self._lifespan_q: Optional[asyncio.Queue] = None
        self._lifespan_task: Optional[asyncio.Task] = None

    # ------------------------------------------------------------------ ASGI bridge
    async def asgi(self, req: Request, conn: Connection) -> None:
        scope = {"type": "http", "asgi": {"version": "3.0"}, "http_version": req.version.split("/")[-1],
                 "method": req.method, "scheme": "http", "path": req.path, "raw_path": req.path.encode(),
                 "query_string": req.query.encode(), "root_path": "", "headers": req.headers,
                 "server": None, "client": conn.transport.get_extra_info("peername")}
        sent_body = False
        disconnected = asyncio.get_running_loop().create_future()
        conn.on_close.append(lambda: disconnected.done() or disconnected.set_result(None))
        state = {"chunked": False, "started": False, "done": False}

        async def receive():
            nonlocal sent_body
            if not sent_body:
                sent_body = True
                return {"type": "http.request", "body": req.body, "more_body": False}
            await disconnected
            return {"type": "http.disconnect"}

        async def send(msg):
            t = msg["type"]
            if t == "http.response.start":
                state["start"] = msg
            elif t == "http.response.body":
                body = msg.get("body", b"")
                more = msg.get("more_body", False)
                if not state["started"]:
                    state["started"] = True
                    start = state["start"]
                    hdrs = [(k.lower(), v) for k, v in start.get("headers", [])]
                    if not any(k == b"content-length" for k, _ in hdrs):
                        if more:
                            hdrs.append((b"transfer-encoding", b"chunked"))
                            state["chunked"] = True
                        else:
                            hdrs.append((b"content-length", str(len(body)).encode()))
                    conn.write_head(int(start["status"]), hdrs)
                if state["chunked"]:
                    conn.write_chunk(body)
                    if not more:
                        conn.end_chunked()
                else:
                    conn.write(body)
                if more:
                    await conn.drain()
                elif not state["done"]:
                    state["done"] = True
                    conn.finish()

        try:
            await self.app(scope, receive, send)
        finally:
            if not state["done"]:
                if state["started"]:
                    conn.keep_alive = False  # the body was cut short: the client must not reuse it
                    if state["chunked"]:
                        conn.end_chunked()
                else:
                    conn.write_head(500, [(b"content-length", b"0")], close=True)
                conn.finish()

    # ------------------------------------------------------------------ lifespan
    async def startup(self) -> None:
        if self.app is None:
            return
        self._lifespan_q = asyncio.Queue()
        started = asyncio.get_running_loop().create_future()
        stopped = asyncio.get_running_loop().create_future()

        async def receive():
            return await self._lifespan_q.get()

        async def send(msg):
            t = msg["type"]
            if t.startswith("lifespan.startup"):
                started.set_result(t)
            elif t.startswith("lifespan.shutdown"):
                stopped.set_result(t)
        self._stopped = stopped
        self._lifespan_task = asyncio.ensure_future(self.app({"type": "lifespan", "asgi": {"version": "3.0"}},
                                                             receive, send))
        await self._lifespan_q.put({"type": "lifespan.startup"})
        if (await started) != "lifespan.startup.complete":
            raise RuntimeError("application startup failed")

    async def shutdown(self) -> None:
        if self._lifespan_q is None:
            return
        await self._lifespan_q.put({"type": "lifespan.shutdown"})
        try:
            await asyncio.wait_for(self._stopped, 10.0)
        except asyncio.TimeoutError:
            pass

    # ------------------------------------------------------------------ run
    async def serve(self, sock: socket.socket, stop: Optional[asyncio.Event] = None) -> None:
        loop = asyncio.get_running_loop()
        await self.startup()
        srv = await loop.create_server(lambda: Connection(self), sock=sock, backlog=2048)
        stop = stop or asyncio.Event()
        for sig in (signal.SIGTERM, signal.SIGINT):
            try:
                loop.add_signal_handler(sig, stop.set)
            except (NotImplementedError, RuntimeError):  # not the main thread (tests)
                pass
        try:
            await stop.wait()
        finally:
            srv.close()
            for c in list(self.conns):
                if c.transport is not None:
                    c.transport.close()
            await self.shutdown()


def listen(host: str, port: int, reuse_port: bool = False) -> socket.socket:
    s = socket.socket(socket.AF_INET6 if ":" in host else socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    if reuse_port:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    s.listen(2048)
    s.setblocking(False)
    return s


def run(app, host: str, port: int, fast=None, sock: Optional[socket.socket] = None) -> None:
    """Serve `app` (+ the fast hook) until SIGTERM / SIGINT."""
    asyncio.run(Server(app, fast).serve(sock or listen(host, port)))
