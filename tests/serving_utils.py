"""Helpers to run frontend / worker ASGI apps on localhost ports inside the test process."""
from __future__ import annotations

import socket
import threading
import time

import httpx


def free_port() -> int:
    """A free port BELOW the kernel's ephemeral range (32768+): the port is closed again before the
    test binds it, and an ephemeral one can be handed to some other connection in between."""
    import os
    import random
    rng = random.Random(os.getpid() ^ time.monotonic_ns())
    for _ in range(200):
        p = rng.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Server:
    def __init__(self, app, port: int | None = None):
        import uvicorn
        self.port = port or free_port()
        self.url = f"http://127.0.0.1:{self.port}"
        cfg = uvicorn.Config(app, host="127.0.0.1", port=self.port, log_level="warning", access_log=False)
        self.server = uvicorn.Server(cfg)
        self.thread = threading.Thread(target=self.server.run, daemon=True)

    def start(self, timeout: float = 20.0) -> "Server":
        self.thread.start()
        t0 = time.time()
        while not self.server.started:
            if time.time() - t0 > timeout:
                raise TimeoutError("server did not start")
            time.sleep(0.05)
        return self

    def stop(self) -> None:
        self.server.should_exit = True
        self.thread.join(timeout=10)


def wait_for(cond, timeout: float = 20.0, interval: float = 0.1) -> None:
    t0 = time.time()
    while not cond():
        if time.time() - t0 > timeout:
            raise TimeoutError("condition not met")
        time.sleep(interval)


def get_json(url: str):
    return httpx.get(url, timeout=30).json()


class FrontendServer:
    """A Frontend served the way `python -m mxserve.frontend` serves it: mxserve/frontend/httpd.py
    with the push-streaming fast path (fastpath.py), on its own event loop in a thread."""

    def __init__(self, fe, port: int | None = None):
        self.fe = fe
        self.port = port or free_port()
        self.url = f"http://127.0.0.1:{self.port}"
        self.loop = None
        self.stop_ev = None
        self.thread = threading.Thread(target=self._run, daemon=True)

    def _run(self) -> None:
        import asyncio

        from mxserve.frontend import fastpath, httpd
        self.loop = asyncio.new_event_loop()
        asyncio.set_event_loop(self.loop)

        async def main():
            self.stop_ev = asyncio.Event()
            srv = httpd.Server(self.fe.app, lambda req, conn: fastpath.handle(self.fe, req, conn))
            await srv.serve(httpd.listen("127.0.0.1", self.port), stop=self.stop_ev)
        self.loop.run_until_complete(main())

    def start(self, timeout: float = 20.0) -> "FrontendServer":
        self.thread.start()
        t0 = time.time()
        while True:
            try:
                with socket.create_connection(("127.0.0.1", self.port), timeout=0.5):
                    return self
            except OSError:
                if time.time() - t0 > timeout:
                    raise TimeoutError("frontend did not start")
                time.sleep(0.05)

    def stop(self) -> None:
        if self.loop is not None and self.stop_ev is not None:
            self.loop.call_soon_threadsafe(self.stop_ev.set)
        self.thread.join(timeout=10)
