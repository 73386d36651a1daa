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
